#!/bin/bash
# GPU session: build, kernel fuzz + training GPU tests, GEMM layout timings, bench with/without optimizer
# overlap, rocprofv3 kernel stats of the bench. A failing test (rc 1) does not stop the session; any other
# non-zero status (timeout, abort, fault) does.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a gpurun_out/steps.log; tail -8 gpurun_out/$name.log; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
step build 600 python __graft_entry__.py && \
step fuzz 600 python -m pytest tests/test_kernels_fuzz_gpu.py tests/test_train_gpu.py -q && \
step layouts 300 python tools/bench_gemm_layouts.py && \
step bench_ovl0 400 python bench.py --steps 10 --warmup 3 --overlap-opt 0 && \
step bench_ovl1 400 python bench.py --steps 10 --warmup 3 --overlap-opt 1 && \
step prof_v4 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/v4 -o l8b --output-format csv -- python3 bench.py --steps 3 --warmup 2
