#!/bin/bash
# Quick GPU check: the given pytest selection (default: the whole GPU suite), each run under its own timeout.
set -o pipefail
mkdir -p gpurun_out/quick
export HSA_ENABLE_IPC_MODE_LEGACY=0
sel=${1:-tests}
timeout -k 10 600 python -u -m pytest $sel -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/quick/pytest.log 2>&1
rc=$?
tail -25 gpurun_out/quick/pytest.log
exit $rc
