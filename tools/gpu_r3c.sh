#!/bin/bash
# Round 3, session C: weight-gradient GEMM forms at the GPT-2-small / Llama-3-8B training shapes (split-K probe).
source "$(dirname "$0")/gpu_lib.sh"
step wgrad_splitk 600 python tools/bench_wgrad_splitk.py && cat gpurun_out/wgrad_splitk.log | grep '^{' > gpurun_out/wgrad_splitk.jsonl
