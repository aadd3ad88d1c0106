#!/bin/bash
set -o pipefail
# GPT-2-small: norm numerics, then the bench with the weight-gradient layout forced to TN (transposes) / NT,
# alternating, in one box session.
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "norm" > gpurun_out/g2_tests.log 2>&1; echo "norm tests rc=$?"; tail -1 gpurun_out/g2_tests.log
for kv in KOP_DW_LAYOUT=tn KOP_DW_LAYOUT=nt KOP_DW_LAYOUT=tn KOP_DW_LAYOUT=nt; do
  env $kv timeout -k 10 200 python bench.py --model gpt2_small --seq 1024 --mbs 32 --accum 1 --steps 20 --warmup 5 > gpurun_out/g2_$kv.log 2>&1
  echo "$kv rc=$? $(grep -oE '"value": [0-9.]*|"ms_per_step": [0-9.]*' gpurun_out/g2_$kv.log | tr '\n' ' ')"
done
