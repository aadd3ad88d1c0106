#!/bin/bash
# Attention backward tests (incl. Hq == Hkv direct dK/dV) then GPT-2-small and Llama-3-8B benches.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -k "attention or gradients or rope" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --model gpt2_small --seq 1024 --mbs 32 --steps 20 --warmup 5 > gpurun_out/g2_direct.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/l8b_direct.log 2>&1
rc=$?; tail -2 gpurun_out/attn_tests.log
for f in gpurun_out/g2_direct.log gpurun_out/l8b_direct.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
exit $rc
