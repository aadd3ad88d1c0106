#!/bin/bash
# Attention A/B inside one box session: attention numerics tests once, then the micro-benchmark per
# "NAME=VALUE" in AB, in order (repeat a setting to see the spread).
set -o pipefail
mkdir -p gpurun_out/attn_ab
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "flash or rope_attention" > gpurun_out/attn_ab/tests.log 2>&1
rc=$?; echo "attn tests rc=$rc"; tail -1 gpurun_out/attn_ab/tests.log; [ $rc -eq 0 ] || exit $rc
i=0
for kv in ${AB:-X=0 X=0}; do
  i=$((i + 1))
  env $kv timeout -k 10 120 python tools/bench_kernels.py --only attn --no-sdpa > gpurun_out/attn_ab/b$i.log 2>&1 || exit 1
  echo "[$i] $kv $(grep -o '"kernel": "[a-z_]*", "B": [0-9]*, "S": [0-9]*.*"ms": [0-9.]*, "tflops": [0-9.]*' gpurun_out/attn_ab/b$i.log | sed -E 's/"Hq".*"ms"/ms/' | tr '\n' ' ')"
done
