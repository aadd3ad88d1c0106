#!/bin/bash
# One GPU iteration: the whole GPU test suite, the memory-bound kernel micro-benchmarks, then the
# Llama-3-8B bench (BENCH_ARGS appended). Every step has its own limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-4} gpurun_out/$name.log; return $rc; }
step tests_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
TAILN=12 step bench_mem 300 python tools/bench_kernels.py --only mem && \
step bench 400 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS}
