#!/bin/bash
# A/B of env-selected kernel variants inside ONE box session (box-to-box clock differences are larger
# than the effects measured): GPU tests once, then the Llama-3-8B bench per "NAME=VALUE" setting in AB.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_kernels.py --only mem > gpurun_out/ab_mem.log 2>&1; echo "mem rc=$?"; cat gpurun_out/ab_mem.log
for kv in ${AB:-KOP_ADAMW_NT=1 KOP_ADAMW_NT=0 KOP_ADAMW_NT=1}; do
  env $kv timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ab_$kv.log 2>&1
  rc=$?; echo "$kv rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$kv.log)"; [ $rc -eq 0 ] || exit $rc
done
