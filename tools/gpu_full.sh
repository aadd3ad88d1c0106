#!/bin/bash
# GPU session: build, the whole GPU test suite, smoke(), GPT-2-small benches (BASELINE config #3),
# Llama-3-8B bench and its rocprofv3 kernel statistics.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a gpurun_out/steps.log; tail -4 gpurun_out/$name.log; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
step build 600 python __graft_entry__.py && \
step tests_gpu 900 python -m pytest tests -m gpu -q && \
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" && \
step gpt2_mbs16 300 python bench.py --model gpt2_small --seq 1024 --mbs 16 --steps 20 --warmup 5 && \
step gpt2_mbs32 300 python bench.py --model gpt2_small --seq 1024 --mbs 32 --steps 20 --warmup 5 && \
step bench 400 python bench.py --steps 10 --warmup 3 && \
step prof_v5 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/v5 -o l8b --output-format csv -- python3 bench.py --steps 3 --warmup 2
