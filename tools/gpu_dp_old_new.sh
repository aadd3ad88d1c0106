#!/bin/bash
# DP rehearsal A/B: this tree vs the pre-session tree (_old, a git worktree of 0bc4819 with its own build),
# 4 ranks on one MI355X, allreduce and zero1, twice each.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
port=29800
for rep in 1 2; do
  for tree in new old; do
    for mode in allreduce zero1; do
      port=$((port + 1))
      dir=.; [ $tree = old ] && dir=_old
      (cd $dir && timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
        --master-port $port tools/dp_rehearsal.py --mode $mode > $GRAFT_REPO_ROOT/gpurun_out/dpon_${tree}_${mode}_$port.log 2>&1)
      echo "$tree $mode rc=$? $(grep -o '"rel_update_error": [0-9.e-]*' gpurun_out/dpon_${tree}_${mode}_$port.log)"
    done
  done
done
