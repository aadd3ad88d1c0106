#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; echo "=== $name" ; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a gpurun_out/steps.log; tail -4 gpurun_out/$name.log; return $rc; }
step build 600 python __graft_entry__.py && \
step attn_tests 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "attention" && \
step attn_bench 300 python tools/bench_kernels.py --only attn
