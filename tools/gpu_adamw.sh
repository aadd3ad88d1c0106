#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a gpurun_out/steps.log; tail -3 gpurun_out/$name.log; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
step build 600 python __graft_entry__.py && \
step b_ovl0 300 python bench.py --steps 10 --warmup 3 --overlap-opt 0 && \
step b_ovl1 300 python bench.py --steps 10 --warmup 3 --overlap-opt 1 && \
KOP_ADAMW_WGS=64 step b_w64 300 python bench.py --steps 10 --warmup 3 --overlap-opt 1 && \
KOP_ADAMW_WGS=128 step b_w128 300 python bench.py --steps 10 --warmup 3 --overlap-opt 1 && \
KOP_ADAMW_WGS=256 step b_w256 300 python bench.py --steps 10 --warmup 3 --overlap-opt 1
