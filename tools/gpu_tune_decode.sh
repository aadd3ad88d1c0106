#!/bin/bash
# TunableOp tuning of the decode GEMM shapes (M = batch 1 / 16 / 64 / 128; a 128-token prompt keeps the prefill
# shapes small), winners written to gpurun_out/ (copied into kubeoperator_amd/tuning/ afterwards); then the
# decode benchmark with the new winners.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export KOP_TUNE_MS=60 KOP_TUNE_ITERS=20
timeout -k 10 900 python tools/bench_decode.py --batch 1,16,64,128 --prompt 128 --steps 2 --graph 0 --gemm-tuning tune \
  --gemm-results gpurun_out/tunableop_results_gfx950_decode.csv > gpurun_out/tune_decode.log 2>&1
rc=$?; echo "tune rc=$rc"; tail -4 gpurun_out/tune_decode.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_decode.py --batch 1,16,64,128 --prompt 2048 --steps 32 --graph 0,1 --gemm-tuning use \
  --gemm-results gpurun_out/tunableop_results_gfx950_decode.csv > gpurun_out/decode_bench_tuned.log 2>&1
rc=$?; echo "bench rc=$rc"; grep decode gpurun_out/decode_bench_tuned.log | cut -c1-330; exit $rc
