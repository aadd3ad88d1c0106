#!/bin/bash
# Shared helpers of the GPU session scripts (sourced): every GPU step runs under its own time limit, writes its
# log under gpurun_out/, and returns its exit status so a session chains steps with && and stops at the first
# failure (no retries).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
_root="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$_root"
step() {
  local name=$1 lim=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log
  tail -4 "gpurun_out/$name.log" | cut -c1-800
  return $rc
}
# one rocprofv3 counter pass over a short program (counters of one pass must fit the hardware blocks)
pmc() {
  local tag=$1; shift
  local counters=$1; shift
  echo "=== pmc $tag $(date +%T)"
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc $counters -d gpurun_out/pmc/$tag -o $tag \
    --output-format csv -- "$@" > gpurun_out/pmc_$tag.log 2>&1
  local rc=$?
  echo "pmc $tag rc=$rc" | tee -a gpurun_out/steps.log
  return $rc
}
