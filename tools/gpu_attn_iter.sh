#!/bin/bash
# Attention iteration on one MI355X: numerics tests of every flash-attention path, the micro-benchmark,
# then (PMC=1, default) the PMC passes of tools/gpu_pmc_attn.sh. Stops at the first failing GPU step.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "flash or rope_attention" > gpurun_out/attn_tests.log 2>&1
rc=$?; echo "attn tests rc=$rc"; tail -3 gpurun_out/attn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_kernels.py --only attn --no-sdpa > gpurun_out/attn_bench.log 2>&1
rc=$?; echo "attn bench rc=$rc"; cat gpurun_out/attn_bench.log; [ $rc -eq 0 ] || exit $rc
if [ "${PMC:-1}" = "1" ]; then bash tools/gpu_pmc_attn.sh; fi
