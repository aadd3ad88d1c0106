#!/bin/bash
# GPT-2-small bench with the working-tree kernels (_C) and a baseline revision's kernels (_Cab, built by
# tools/build_ab.py), alternating in ONE box session, then a rocprofv3 kernel trace of the new build.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "norm or bias" > gpurun_out/g2k_tests.log 2>&1
rc=$?; echo "norm tests rc=$rc"; tail -1 gpurun_out/g2k_tests.log; [ $rc -eq 0 ] || exit $rc
for m in _C _Cab _C _Cab; do
  KOP_EXT_MODULE=$m timeout -k 10 200 python bench.py --model gpt2_small --seq 1024 --mbs 32 --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/g2k_$m.log 2>&1
  rc=$?; echo "$m rc=$rc $(grep -oE '"value": [0-9.]*|"ms_per_step": [0-9.]*' gpurun_out/g2k_$m.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/gpt2 -o gpt2 --output-format csv -- \
  python3 bench.py --model gpt2_small --seq 1024 --mbs 32 --steps 3 --warmup 2 > gpurun_out/prof_gpt2.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
