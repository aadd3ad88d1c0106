#!/bin/bash
# End-of-round GPU check of the in-tree build: GPU test suite, smoke(), GPT-2-small and Llama-3-8B benches.
set -o pipefail
mkdir -p gpurun_out/final
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/final/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 gpurun_out/final/$name.log; [ $rc -eq 0 ]; }
step tests_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider && \
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" && \
step gpt2_mbs32 300 python bench.py --model gpt2_small --seq 1024 --mbs 32 --steps 20 --warmup 5 && \
step bench 500 python bench.py
