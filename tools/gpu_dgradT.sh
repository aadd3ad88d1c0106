#!/bin/bash
# Transposed-weight dX GEMMs: GPU tests, the DP rehearsal (ZeRO-1 gathers feeding the W^T refresh), then the
# Llama-3-8B bench with the copies on / off in one session.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dt_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/dt_tests.log; [ $rc -eq 0 ] || exit $rc
for kv in KOP_TRANSPOSED_W=1 KOP_TRANSPOSED_W=0 KOP_TRANSPOSED_W=1 KOP_TRANSPOSED_W=0; do
  env $kv timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/dt_$kv.log 2>&1
  rc=$?; echo "$kv rc=$rc $(grep -oE '"value": [0-9.]*|"ms_per_step": [0-9.]*|"peak_mem_gb_rank0": [0-9.]*' gpurun_out/dt_$kv.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
