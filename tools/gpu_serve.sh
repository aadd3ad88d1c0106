#!/bin/bash
# Serving path on one MI355X: decode-attention numerics + generator consistency tests, the Llama-3-8B decode
# benchmark, then a rocprofv3 kernel-stats pass of a short decode run.
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -6 gpurun_out/$name.log | cut -c1-400; return $rc; }
step serve_tests 300 python -u -m pytest tests/test_serve.py -x -v --timeout 120 --timeout-method thread && \
step decode_bench 400 python tools/bench_decode.py --batch 1,16,64,128 --prompt 2048 --steps 32 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
step decode_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/decode -o decode --output-format csv -- \
  python3 tools/bench_decode.py --batch 64 --prompt 2048 --steps 8
