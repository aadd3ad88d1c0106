#!/bin/bash
# GEMM tuning session: record the training step's GEMMs, tune each (progress per shape), then bench
# heuristic vs tuned selection.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a gpurun_out/steps.log; tail -4 gpurun_out/$name.log; return $rc; }
step build 600 python __graft_entry__.py && \
PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=0 KOP_TUNE_MS=100 KOP_TUNE_ITERS=30 step tune 700 python tools/tune_gemms.py && \
cp kubeoperator_amd/tuning/tunableop_results_gfx950.csv gpurun_out/ && \
step bench_off 600 python bench.py --steps 10 --warmup 3 --gemm-tuning off && \
step bench_use 600 python bench.py --steps 10 --warmup 3 --gemm-tuning use
