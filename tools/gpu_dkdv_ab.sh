#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for c in 83 82; do
  KOP_DKDV_CFG=$c timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "flash or attention or attn" > gpurun_out/dkdv_tests_$c.log 2>&1
  rc=$?; echo "tests cfg $c rc=$rc"; tail -2 gpurun_out/dkdv_tests_$c.log; [ $rc -eq 0 ] || exit $rc
done
VARIANTS="base;KOP_DKDV_CFG=83;KOP_DKDV_CFG=82" SHAPES=llama,llama4k,guide bash tools/gpu_attn_probe.sh
