#!/bin/bash
# Continuous-batching serving benchmark (Llama-3-8B, 256 requests, prompts 256-2048 tokens, 128 new tokens each).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for slots in 64 128; do
  timeout -k 10 500 python tools/bench_serve.py --requests 256 --slots $slots --prompt 256,2048 --new 128 > gpurun_out/serve_bench_$slots.log 2>&1
  rc=$?; echo "slots $slots rc=$rc $(grep '"bench"' gpurun_out/serve_bench_$slots.log)"; [ $rc -eq 0 ] || exit $rc
done
