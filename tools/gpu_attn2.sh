#!/bin/bash
# Attention kernel session: numerics of every forward / dQ variant, micro-bench of each, PMC counters.
# Variants (env): 4 = 4-wave kernels, 8 = 8-wave lockstep, 9 = 8-wave with staggered halves.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a gpurun_out/steps.log; tail -6 gpurun_out/$name.log; return $rc; }
step build 600 python __graft_entry__.py && \
KOP_FWD_VARIANT=8 KOP_DQ_VARIANT=8 step t_v8 300 python -m pytest tests/test_kernels_gpu.py -x -q -k flash && \
KOP_FWD_VARIANT=9 KOP_DQ_VARIANT=9 step t_v9 300 python -m pytest tests/test_kernels_gpu.py -x -q -k flash && \
KOP_FWD_VARIANT=4 KOP_DQ_VARIANT=4 step b_v4 300 python tools/bench_kernels.py --only attn && \
KOP_FWD_VARIANT=8 KOP_DQ_VARIANT=8 step b_v8 300 python tools/bench_kernels.py --only attn --no-sdpa && \
KOP_FWD_VARIANT=9 KOP_DQ_VARIANT=9 step b_v9 300 python tools/bench_kernels.py --only attn --no-sdpa && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
KOP_FWD_VARIANT=9 KOP_DQ_VARIANT=9 step kt_v9 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_v9 -o kt --output-format csv -- python3 tools/bench_kernels.py --only attn --iters 3 --no-sdpa && \
step list_counters 120 rocprofv3 -L && \
KOP_FWD_VARIANT=9 KOP_DQ_VARIANT=9 step pmc1 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU -d gpurun_out/pmc1 -o pmc1 --output-format csv -- python3 tools/bench_kernels.py --only attn --iters 2 --no-sdpa && \
KOP_FWD_VARIANT=9 KOP_DQ_VARIANT=9 step pmc2 400 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_INSTS_SALU SQ_WAVES -d gpurun_out/pmc2 -o pmc2 --output-format csv -- python3 tools/bench_kernels.py --only attn --iters 2 --no-sdpa
