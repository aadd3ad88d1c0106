#!/bin/bash
# FP8 training path after a change to ops.functional: its GPU tests and the opt-in --fp8 Llama-3-8B bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py tests/test_serve.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/fp8_tests.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 8 --warmup 3 --fp8 1 > gpurun_out/fp8_bench.log 2>&1
rc=$?; echo "fp8 bench rc=$rc $(grep -oE '"value": [0-9.]+|"ms_per_step": [0-9.]+' gpurun_out/fp8_bench.log | tr '\n' ' ')"; exit $rc
