#!/bin/bash
# Attention kernel session: numerics of every forward variant, micro-bench of each, kernel-trace of the best.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a gpurun_out/steps.log; tail -6 gpurun_out/$name.log; return $rc; }
step build 600 python __graft_entry__.py && \
KOP_FWD_VARIANT=8 step t_v8 300 python -m pytest tests/test_kernels_gpu.py -x -q -k flash && \
KOP_FWD_VARIANT=9 step t_v9 300 python -m pytest tests/test_kernels_gpu.py -x -q -k flash && \
KOP_FWD_VARIANT=4 step b_v4 300 python tools/bench_kernels.py --only attn && \
KOP_FWD_VARIANT=8 step b_v8 300 python tools/bench_kernels.py --only attn && \
KOP_FWD_VARIANT=9 step b_v9 300 python tools/bench_kernels.py --only attn
