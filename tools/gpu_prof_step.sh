#!/bin/bash
# rocprofv3 kernel trace + stats of the default Llama-3-8B bench step (accum 4) and GPT-2-small.
set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/l8b -o l8b --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_l8b.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/g2 -o g2 --output-format csv -- python3 bench.py --model gpt2_small --seq 1024 --mbs 32 --steps 3 --warmup 2 > gpurun_out/prof_g2.log 2>&1
echo "rc=$?"
