#!/bin/bash
# Serving with E4M3 block-projection weights (opt-in): the serving tests, then the decode benchmark bf16 vs fp8
# weights (graphed at batch 1, eager from 16 up) in one session.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_serve.py -x -q --timeout 120 --timeout-method thread > gpurun_out/serve_fp8_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/serve_fp8_tests.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_decode.py --batch 1 --graph 1 --fp8 0,1 --prompt 2048 --steps 32 > gpurun_out/decode_fp8_b1.log 2>&1
rc=$?; echo "b1 rc=$rc"; grep decode gpurun_out/decode_fp8_b1.log | cut -c1-260; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_decode.py --batch 16,64,128 --graph 0 --fp8 0,1 --prompt 2048 --steps 32 > gpurun_out/decode_fp8.log 2>&1
rc=$?; echo "b16-128 rc=$rc"; grep decode gpurun_out/decode_fp8.log | cut -c1-260; exit $rc
