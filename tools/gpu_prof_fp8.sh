#!/bin/bash
# rocprofv3 kernel trace + stats of the Llama-3-8B step with --fp8 1 (2 timed steps).
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/l8b_fp8 -o l8b --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --fp8 1 > gpurun_out/prof_l8b_fp8.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/prof_l8b_fp8.log; exit $rc
