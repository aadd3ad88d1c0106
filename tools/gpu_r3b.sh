#!/bin/bash
# Round 3, session B: the weight-gradient side stream in MULTI-rank jobs (the in-place-accumulation fix), under a
# forced side-stream lag, in the one-GPU data- / tensor-parallel rehearsals (ranks share cuda:0 over gloo); the
# bench.py communication fields on GPU ranks; a Llama-3-8B bench.
source "$(dirname "$0")/gpu_lib.sh"
export KOP_WGRAD_STREAM=1 KOP_WGRAD_STREAM_MULTI=1 KOP_SIDE_LAG_CYCLES=200000
port=29760
rehearse() {  # nproc script args...
  local n=$1; shift; port=$((port + 1))
  step "reh_$port" 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $port "$@" && grep -h rehearsal gpurun_out/reh_$port.log | tee -a gpurun_out/rehearsals.jsonl
}
rehearse 2 tools/dp_rehearsal.py --mode zero1 && \
rehearse 4 tools/dp_rehearsal.py --mode zero1 --accum 4 && \
rehearse 4 tools/dp_rehearsal.py --mode allreduce && \
rehearse 2 tools/dp_rehearsal.py --mode allreduce --accum 2 --grad-dtype fp32 && \
rehearse 2 tools/dp_rehearsal.py --mode zero1 --model tiny_gpt2 --accum 2 && \
rehearse 4 tools/dp_rehearsal.py --mode zero1 --model tiny_gpt2 --accum 4 && \
rehearse 2 tools/tp_rehearsal.py --tp 2 --mode zero1 --out /tmp/kop_tp_a && \
rehearse 4 tools/tp_rehearsal.py --tp 2 --mode zero1 --sp 1 --out /tmp/kop_tp_b && \
unset KOP_SIDE_LAG_CYCLES KOP_WGRAD_STREAM KOP_WGRAD_STREAM_MULTI && \
KOP_DIST_BACKEND=gloo KOP_DEVICE_INDEX=0 step bench_dp2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29792 bench.py --gpus 2 --steps 2 --warmup 1 --model llama3_1b_proxy --seq 2048 && \
step bench_l8b 400 python bench.py --steps 10 --warmup 3
