#!/bin/bash
# Fused SwiGLU backward + transposed gradient: kernel micro-bench, then Llama-3-8B bench A/B (KOP_SWIGLU_T).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python tools/bench_swiglu_t.py > gpurun_out/swt_kernel.json 2>&1 || { tail -20 gpurun_out/swt_kernel.json; exit 1; }
cat gpurun_out/swt_kernel.json
for i in 1 2; do
  for m in 0 1; do
    KOP_SWIGLU_T=$m timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/l8b_swt${m}_$i.log 2>&1 || { tail -20 gpurun_out/l8b_swt${m}_$i.log; exit 1; }
    echo "swt=$m $(grep -o '"value": [0-9.]*' gpurun_out/l8b_swt${m}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/l8b_swt${m}_$i.log)"
  done
done
