#!/bin/bash
# Decode-attention chunk size A/B (KOP_DECODE_CH 256 vs 128 keys per workgroup) in one box session: the kernel
# numerics tests under each setting, then the Llama-3-8B decode benchmark at batch 64 / 128, alternating.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for ch in 128 256; do
  KOP_DECODE_CH=$ch timeout -k 10 300 python -u -m pytest tests/test_serve.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dch_tests_$ch.log 2>&1
  rc=$?; echo "tests ch$ch rc=$rc $(tail -1 gpurun_out/dch_tests_$ch.log)"; [ $rc -eq 0 ] || exit $rc
done
for ch in 256 128 256 128; do
  KOP_DECODE_CH=$ch timeout -k 10 300 python tools/bench_decode.py --batch 64,128 --prompt 2048 --steps 32 --graph 0 > gpurun_out/dch_$ch.log 2>&1
  rc=$?; echo "ch$ch rc=$rc $(grep -oE '"batch": [0-9]+|"decode_ms_per_step": [0-9.]+' gpurun_out/dch_$ch.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
