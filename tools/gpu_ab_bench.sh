#!/bin/bash
# A/B of env-selected variants inside ONE box session (box-to-box clock differences are larger than the
# effects measured): GPU tests once, then the Llama-3-8B bench once per "NAME=VALUE" setting in AB (in order;
# repeat a setting to see the run-to-run spread).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
i=0
for kv in ${AB:-KOP_GEMM_RESULTS=gpurun_in/tun_old.csv KOP_GEMM_RESULTS= KOP_GEMM_RESULTS=gpurun_in/tun_old.csv KOP_GEMM_RESULTS=}; do
  i=$((i + 1))
  env $kv timeout -k 10 300 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/ab_$i.log 2>&1
  rc=$?; echo "[$i] $kv rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
