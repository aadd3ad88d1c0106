#!/bin/bash
# SURVEY 5.2 debug run: the whole GPU test suite with every kernel launch serialised and blocking
# (AMD_SERIALIZE_KERNEL=3: wait before and after each dispatch; HIP_LAUNCH_BLOCKING=1), so an asynchronous
# fault or a race between our streams (optimizer / RCCL / compute) surfaces at the launching call, and the
# results must still match the concurrent run.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
AMD_SERIALIZE_KERNEL=3 HIP_LAUNCH_BLOCKING=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/tests_gpu_serialized.log 2>&1
rc=$?; tail -3 gpurun_out/tests_gpu_serialized.log; exit $rc
