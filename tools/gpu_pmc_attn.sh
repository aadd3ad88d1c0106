#!/bin/bash
# PMC passes over the attention micro-benchmark (one rocprofv3 run per counter set, each under its own
# time limit): MFMA busy cycles, VALU / LDS / MFMA instruction counts, LDS bank conflicts and wait cycles
# per kernel. Summaries land in gpurun_out/pmc/.
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc "$@" -d gpurun_out/pmc/$tag -o $tag --output-format csv \
    -- python3 tools/bench_kernels.py --only attn --iters 3 --no-sdpa > gpurun_out/pmc/$tag.log 2>&1
  local rc=$?; echo "pmc $tag rc=$rc"; return $rc
}
run busy SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS && \
run lds SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_ANY && \
run grbm GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD
