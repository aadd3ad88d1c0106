#!/bin/bash
# Kernel-time profile of the Llama-3-8B training step (rocprofv3 --kernel-trace --stats), plus the GPT-2-small
# bench (BASELINE config #3). Output under gpurun_out/prof_full/.
set -o pipefail
mkdir -p gpurun_out/prof_full
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py --model gpt2_small --seq 1024 --mbs 32 --steps 20 --warmup 5 > gpurun_out/prof_full/gpt2.log 2>&1
echo "gpt2 rc=$?"; tail -1 gpurun_out/prof_full/gpt2.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full/l8b -o l8b --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_full/l8b.log 2>&1
echo "prof rc=$?"; tail -1 gpurun_out/prof_full/l8b.log
