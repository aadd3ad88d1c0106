#!/bin/bash
# End-of-session check of the committed tree on one MI355X with the in-tree prebuilt extension (as the driver
# runs it): the whole GPU suite, smoke(), the Llama-3-8B and GPT-2-small benches, then a rocprofv3 kernel trace of
# the Llama-3-8B step.
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a gpurun_out/steps.log; tail -3 gpurun_out/$name.log | cut -c1-600; return $rc; }
step tests_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" && \
step bench 400 python bench.py --steps 10 --warmup 3 && \
step gpt2 300 python bench.py --model gpt2_small --seq 1024 --mbs 32 --steps 20 --warmup 5 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
step prof_l8b 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/l8b -o l8b --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1
