#!/bin/bash
# HIP-graph replay: full GPU test suite, then GPT-2-small at small micro-batches eager vs graphed.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_gpu.log 2>&1 || { tail -30 gpurun_out/tests_gpu.log; exit 1; }
tail -2 gpurun_out/tests_gpu.log
for mbs in 1 2; do
  for g in 0 1; do
    timeout -k 10 300 python bench.py --model gpt2_small --seq 1024 --mbs $mbs --steps 30 --warmup 5 --cuda-graph $g > gpurun_out/graph_g2_mbs${mbs}_g$g.log 2>&1 || { tail -20 gpurun_out/graph_g2_mbs${mbs}_g$g.log; exit 1; }
  done
done
for f in gpurun_out/graph_g2_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
