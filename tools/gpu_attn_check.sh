#!/bin/bash
# Attention numerics (every flash-attention GPU test) then the probe; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernels_fuzz_gpu.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "flash or attention or attn" > gpurun_out/attn_tests.log 2>&1
rc=$?; echo "attn tests rc=$rc"; tail -3 gpurun_out/attn_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_attn_probe.sh
