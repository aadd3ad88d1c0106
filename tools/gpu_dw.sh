#!/bin/bash
# GPU session: build, transpose/weight-grad tests + overlap test, layout timings, bench with dW layout nt vs tn.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a gpurun_out/steps.log; tail -8 gpurun_out/$name.log; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
step build 600 python __graft_entry__.py && \
step t_dw 300 python -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -q -k "transpose or weight_grad or overlapped" && \
step layouts 300 python tools/bench_gemm_layouts.py && \
KOP_DW_LAYOUT=nt step bench_nt 400 python bench.py --steps 10 --warmup 3 && \
KOP_DW_LAYOUT=tn step bench_tn 400 python bench.py --steps 10 --warmup 3
