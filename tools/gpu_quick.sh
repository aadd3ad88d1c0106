#!/bin/bash
# Quick kernel check: build, flash-attention numerics, attention micro-bench, one full-model bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a gpurun_out/steps.log; tail -6 gpurun_out/$name.log; return $rc; }
step build 600 python __graft_entry__.py && \
step t_flash 300 python -m pytest tests/test_kernels_gpu.py -x -q && \
step b_attn 300 python tools/bench_kernels.py --only attn --no-sdpa && \
step bench 600 python bench.py --steps 10 --warmup 3 --gemm-tuning off
