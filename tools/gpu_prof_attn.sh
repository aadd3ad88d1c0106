#!/bin/bash
# Per-kernel times of the attention passes (rocprofv3 kernel trace of tools/attn_probe.py), one run per
# KOP_DQ_VARIANT listed in $DQV (10: dK/dV kernel stores dS + dQ from dS; 9: dQ recomputes S and dP).
set -o pipefail
mkdir -p gpurun_out/profattn
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ${DQV:-10 9}; do
  KOP_DQ_VARIANT=$v timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/profattn/v$v -o attn --output-format csv -- \
    python3 tools/attn_probe.py --shapes ${SHAPES:-llama} --causal 1 --iters 10 > gpurun_out/profattn/v$v.log 2>&1
  rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
