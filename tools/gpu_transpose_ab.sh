#!/bin/bash
# Transpose kernel: exactness tests and bandwidth of the tile shapes / block orders.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for m in rows wide square; do
  KOP_TRANSPOSE=$m timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "transpose" -x -q --timeout 120 --timeout-method thread > gpurun_out/tr_tests_$m.log 2>&1 || exit 1
  KOP_TRANSPOSE=$m timeout -k 10 120 python tools/bench_transpose.py > gpurun_out/tr_$m.json 2>gpurun_out/tr_$m.err || exit 1
done
tail -1 gpurun_out/tr_tests_rows.log; cat gpurun_out/tr_*.json
