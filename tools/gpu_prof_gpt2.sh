#!/bin/bash
# rocprofv3 kernel trace + stats of the GPT-2-small bench step (seq 1024, mbs 32, accum 4), 3 timed steps.
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/gpt2 -o gpt2 --output-format csv -- \
  python3 bench.py --model gpt2_small --seq 1024 --mbs 32 --steps 3 --warmup 2 > gpurun_out/prof_gpt2.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/prof_gpt2.log | cut -c1-200; exit $rc
