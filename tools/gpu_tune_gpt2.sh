#!/bin/bash
# GEMM tuning for the GPT-2-small chart shapes (mbs 32, seq 1024) on top of the committed Llama-3-8B winners,
# then GPT-2-small bench with heuristic vs tuned selection (alternating).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=0 KOP_TUNE_MS=100 KOP_TUNE_ITERS=30 timeout -k 10 700 python tools/tune_gemms.py --model gpt2_small --seq 1024 --mbs 32 > gpurun_out/tune_gpt2.log 2>&1 || exit 1
cp kubeoperator_amd/tuning/tunableop_results_gfx950.csv gpurun_out/tunableop_results_gfx950.csv
for i in 1 2; do
  for m in off use; do
    timeout -k 10 300 python bench.py --model gpt2_small --seq 1024 --mbs 32 --steps 20 --warmup 5 --gemm-tuning $m > gpurun_out/g2_${m}_$i.log 2>&1 || exit 1
  done
done
tail -3 gpurun_out/tune_gpt2.log
for f in gpurun_out/g2_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
