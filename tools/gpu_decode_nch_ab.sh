#!/bin/bash
# Decode attention: one-shot 128-key workgroups (KOP_DECODE_NCH=1, default) vs the streaming kernel over 4 chunks
# (KOP_DECODE_NCH=4) -- numerics tests under both, then the decode benchmark alternating, one session.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 4 1; do
  KOP_DECODE_NCH=$n timeout -k 10 300 python -u -m pytest tests/test_serve.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dnch_tests_$n.log 2>&1
  rc=$?; echo "tests nch$n rc=$rc $(tail -1 gpurun_out/dnch_tests_$n.log)"; [ $rc -eq 0 ] || exit $rc
done
for n in 1 4 1 4; do
  KOP_DECODE_NCH=$n timeout -k 10 300 python tools/bench_decode.py --batch 16,64,128 --prompt 2048 --steps 32 --graph 0 > gpurun_out/dnch_$n.log 2>&1
  rc=$?; echo "nch$n rc=$rc $(grep -oE '"batch": [0-9]+|"decode_ms_per_step": [0-9.]+' gpurun_out/dnch_$n.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
