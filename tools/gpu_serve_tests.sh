#!/bin/bash
# The serving tests on one MI355X (decode-attention numerics, generator vs CPU reference eager / graphed /
# padded prompts / continuous batching, FP8 weights).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_serve.py -x -v --timeout 120 --timeout-method thread > gpurun_out/serve_tests.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/serve_tests.log | tail -14; exit $rc
