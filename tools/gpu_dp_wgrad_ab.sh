#!/bin/bash
# ZeRO-1 rehearsal (4 gloo ranks on one MI355X) with the weight-gradient side stream forced off / on.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
port=29720
for cfg in "0 4" "1 4" "0 1" "1 1" "0 4"; do
  set -- $cfg
  port=$((port + 1))
  KOP_WGRAD_STREAM=$1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port $port tools/dp_rehearsal.py --mode zero1 --accum $2 > gpurun_out/dpw_$1_$2_$port.log 2>&1
  echo "wgrad_stream=$1 accum$2 rc=$? $(grep -o '"rel_update_error": [0-9.e-]*' gpurun_out/dpw_$1_$2_$port.log)"
done
