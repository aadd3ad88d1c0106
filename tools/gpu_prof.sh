#!/bin/bash
# rocprofv3 kernel-trace + stats of the attention micro-bench and of a short Llama-3-8B training run.
set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python __graft_entry__.py > gpurun_out/prof_build.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/attn -o attn --output-format csv -- python3 tools/bench_kernels.py --only attn > gpurun_out/prof_attn.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/l8b -o l8b --output-format csv -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof_l8b.log 2>&1
echo "rc=$?"
