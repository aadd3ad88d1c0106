#!/bin/bash
# Tune the hipBLASLt solutions of every GEMM shape the training step calls that has no committed winner yet
# (tools/tune_gemms.py), then bench with the updated table. A heartbeat keeps the run visibly alive while a
# large shape tunes; the results file is copied to gpurun_out/ (the only directory merged back).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do sleep 45; echo "[heartbeat] $(date +%T)"; done ) &
hb=$!
PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=0 KOP_TUNE_MS=${KOP_TUNE_MS:-50} KOP_TUNE_ITERS=${KOP_TUNE_ITERS:-20} timeout -k 10 1500 python -u tools/tune_gemms.py > gpurun_out/tune2.log 2>&1
rc=$?; echo "tune rc=$rc"; tail -25 gpurun_out/tune2.log
cp kubeoperator_amd/tuning/tunableop_results_gfx950.csv gpurun_out/tunableop_results_gfx950.csv
if [ $rc -eq 0 ]; then
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/tune2_bench.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/tune2_bench.log
fi
kill $hb
exit $rc
