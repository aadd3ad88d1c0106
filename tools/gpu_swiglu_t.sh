#!/bin/bash
# Fused SwiGLU MLP node: full GPU tests, then Llama-3-8B bench A/B (KOP_SWIGLU_T).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_gpu.log 2>&1 || { tail -30 gpurun_out/tests_gpu.log; exit 1; }
tail -1 gpurun_out/tests_gpu.log
for i in 1 2; do
  for m in 0 1; do
    KOP_SWIGLU_T=$m timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/l8b_swt${m}_$i.log 2>&1 || { tail -20 gpurun_out/l8b_swt${m}_$i.log; exit 1; }
    echo "swt=$m $(grep -o '"value": [0-9.]*' gpurun_out/l8b_swt${m}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/l8b_swt${m}_$i.log) $(grep -o '"peak_mem_gb_rank0": [0-9.]*' gpurun_out/l8b_swt${m}_$i.log)"
  done
done
