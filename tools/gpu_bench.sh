#!/bin/bash
# GPU session: build, kernel tests, Llama-3-8B bench (allreduce + zero1 paths), rocprofv3 stats of the bench.
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a gpurun_out/steps.log; tail -4 gpurun_out/$name.log; return $rc; }
step build 600 python __graft_entry__.py && \
step tests 600 python -m pytest tests -m gpu -x -q && \
step bench 600 python bench.py --steps 10 --warmup 3 && \
step bench_zero1 600 python bench.py --steps 5 --warmup 2 --dp zero1 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
step prof_l8b 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/l8b -o l8b --output-format csv -- python3 bench.py --steps 3 --warmup 1
