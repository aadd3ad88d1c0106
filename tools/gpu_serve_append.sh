#!/bin/bash
# Serving tests after the fused decode RoPE + cache-append kernel, then the decode benchmark (batch 1 graphed,
# 16 / 64 / 128 eager).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/gpu_serve_tests.sh || exit $?
timeout -k 10 400 python tools/bench_decode.py --batch 1 --graph 1 --prompt 2048 --steps 32 > gpurun_out/decode_append_b1.log 2>&1
rc=$?; echo "b1 rc=$rc"; grep '"bench"' gpurun_out/decode_append_b1.log | cut -c1-260; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_decode.py --batch 16,64,128 --graph 0 --prompt 2048 --steps 32 > gpurun_out/decode_append.log 2>&1
rc=$?; echo "b16-128 rc=$rc"; grep '"bench"' gpurun_out/decode_append.log | cut -c1-260; exit $rc
