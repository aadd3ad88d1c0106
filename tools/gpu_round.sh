#!/bin/bash
# One GPU session: kernel numerics tests, smoke, short benches. Each GPU step has its own time limit and
# the chain stops at the first failure (no GPU work after a fault / timeout).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name" ; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a gpurun_out/steps.log; tail -3 gpurun_out/$name.log; return $rc; }
step build 600 python __graft_entry__.py && \
step tests 600 python -m pytest tests -m gpu -x -q && \
step smoke 300 python __graft_entry__.py smoke && \
step bench_l8b 600 python bench.py --steps 5 --warmup 2 ${BENCH_ARGS}
