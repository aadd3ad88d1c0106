#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a gpurun_out/steps.log; tail -8 gpurun_out/$name.log; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
step build 600 python __graft_entry__.py && \
step t_dq 400 python -m pytest tests/test_kernels_gpu.py tests/test_kernels_fuzz_gpu.py -q -x -k "dq_variants or flash or attention" && \
step b_attn 300 python tools/bench_kernels.py --only attn --no-sdpa && \
step kt 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_dkdv2 -o kt --output-format csv -- python3 tools/bench_kernels.py --only attn --iters 3 --no-sdpa && \
step bench 400 python bench.py --steps 10 --warmup 3
