#!/bin/bash
# Last check: GPU training tests + smoke + the GPT-2-small bench with the new default (no side stream) and with it.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/last_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/last_tests.log)"; [ $rc -eq 0 ] || exit $rc
for ws in off auto; do
  timeout -k 10 300 python bench.py --model gpt2_small --seq 1024 --mbs 32 --steps 20 --warmup 5 --wgrad-stream $ws > gpurun_out/last_gpt2_$ws.log 2>&1
  rc=$?; echo "gpt2 wgrad=$ws rc=$rc $(grep -oE '"value": [0-9.]+|"ms_per_step": [0-9.]+' gpurun_out/last_gpt2_$ws.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
