#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a gpurun_out/steps.log; tail -6 gpurun_out/$name.log; return $rc; }
step build 600 python __graft_entry__.py && \
step t_flash 300 python -m pytest tests/test_kernels_gpu.py -x -q && \
KOP_FWD_VARIANT=8 KOP_DQ_VARIANT=8 step t_flash8 300 python -m pytest tests/test_kernels_gpu.py -x -q -k flash && \
KOP_FWD_VARIANT=8 KOP_DQ_VARIANT=8 step b_attn8 300 python tools/bench_kernels.py --only attn --no-sdpa && \
KOP_FWD_VARIANT=9 KOP_DQ_VARIANT=9 step b_attn9 300 python tools/bench_kernels.py --only attn --no-sdpa && \
step bench 600 python bench.py --steps 10 --warmup 3 --gemm-tuning off
