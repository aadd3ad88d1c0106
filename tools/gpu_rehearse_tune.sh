#!/bin/bash
set -o pipefail
# Data-parallel rehearsal (tools/gpu_dp_rehearsal.sh), then GEMM re-tuning of untuned shapes (tools/gpu_tune2.sh).
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
bash tools/gpu_dp_rehearsal.sh > gpurun_out/rh.log 2>&1; rc=$?; grep -E "rc=" gpurun_out/rh.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_tune2.sh
