#!/bin/bash
# Quick check after a kernel change: the kernel numerics tests, the GPT-2-small and Llama-3-8B benches,
# then the whole GPU suite and smoke(). Every GPU step has its own time limit; the chain stops at the
# first failure.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a gpurun_out/steps.log; tail -4 gpurun_out/$name.log; return $rc; }
step kernels 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread && \
step gpt2 300 python bench.py --model gpt2_small --seq 1024 --mbs 32 --steps 20 --warmup 5 && \
step bench 400 python bench.py --steps 10 --warmup 3 && \
step tests_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
