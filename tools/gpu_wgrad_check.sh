#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python tools/wgrad_stream_check.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/wgrad_check.log
