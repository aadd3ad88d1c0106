#!/bin/bash
# Weight gradients on a side stream (KOP_WGRAD_STREAM): GPU training tests with it on, then alternating
# Llama-3-8B and GPT-2-small benches with it off / on inside one box session.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
KOP_WGRAD_STREAM=1 timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/wg_tests.log 2>&1
rc=$?; echo "wgrad-stream train tests rc=$rc"; tail -2 gpurun_out/wg_tests.log; [ $rc -eq 0 ] || exit $rc
i=0
for run in "0 llama" "1 llama" "0 gpt2" "1 gpt2" "0 llama" "1 llama" "0 gpt2" "1 gpt2"; do
  set -- $run
  i=$((i + 1))
  if [ $2 = llama ]; then args="--steps 8 --warmup 3"; else args="--model gpt2_small --seq 1024 --mbs 32 --steps 20 --warmup 5"; fi
  KOP_WGRAD_STREAM=$1 timeout -k 10 300 python bench.py $args > gpurun_out/wg_$i.log 2>&1
  rc=$?; echo "[$i] wgrad_stream=$1 $2 rc=$rc $(grep -oE '"value": [0-9.]*|"ms_per_step": [0-9.]*' gpurun_out/wg_$i.log | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
done
