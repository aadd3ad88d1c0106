#!/bin/bash
# GPT-2-small attention backward: dQ from the stored dS (variant 10, default) vs the recompute dQ kernels
# (9: 8-wave staggered, 0: 4-wave) -- isolated probe at the bench shape, then the GPT-2 bench alternating.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
VARIANTS="base;KOP_DQ_VARIANT=9;KOP_DQ_VARIANT=0" SHAPES=gpt2b,gpt2 timeout -k 10 400 bash tools/gpu_attn_probe.sh > gpurun_out/g2dq_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; grep -o '"tag[^}]*' gpurun_out/attn_probe.jsonl | head -20; [ $rc -eq 0 ] || exit $rc
for kv in KOP_DQ_VARIANT=10 KOP_DQ_VARIANT=9 KOP_DQ_VARIANT=10 KOP_DQ_VARIANT=9; do
  env $kv timeout -k 10 200 python bench.py --model gpt2_small --seq 1024 --mbs 32 --steps 20 --warmup 5 > gpurun_out/g2dq_$kv.log 2>&1
  rc=$?; echo "$kv rc=$rc $(grep -oE '"value": [0-9.]*|"ms_per_step": [0-9.]*' gpurun_out/g2dq_$kv.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
