#!/bin/bash
# GPT-2-small (D 64, 12/12 heads, S 1024): attention kernel variants end to end (one box session).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for kv in X=0 KOP_DQ_VARIANT=9 KOP_DQ_VARIANT=8 KOP_FWD_VARIANT=9 KOP_FWD_VARIANT=1 X=0; do
  env $kv timeout -k 10 300 python bench.py --model gpt2_small --seq 1024 --mbs 32 --steps 20 --warmup 5 > gpurun_out/g2v.log 2>&1 || { tail -20 gpurun_out/g2v.log; exit 1; }
  echo "$kv $(grep -o '"value": [0-9.]*' gpurun_out/g2v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/g2v.log)"
done
