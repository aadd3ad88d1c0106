#!/bin/bash
# Llama-3-70B shapes on ONE MI355X: 4 of its 80 layers at tp 2 (two ranks share the card over gloo, launched by
# torchrun as the driver launches bench.py), with per-block recompute -- the hidden 8192 / 64 heads / 8 KV heads /
# FFN 28672 block through the HIP kernels at its TP-2 shard shapes, plus the replicated 128256 x 8192
# embedding and LM head. Throughput is meaningless (shared card, gloo copies through the host).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
KOP_DIST_BACKEND=gloo KOP_DEVICE_INDEX=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29695 bench.py --gpus 2 --tp 2 --model llama3_70b --layers 4 --recompute 1 --sp 1 \
  --seq 8192 --mbs 1 --accum 1 --steps 2 --warmup 1 --gemm-tuning off > gpurun_out/tp70b.log 2>&1
rc=$?; echo "70b tp2 rc=$rc"; grep metric gpurun_out/tp70b.log | cut -c1-900; tail -3 gpurun_out/tp70b.log | cut -c1-300; exit $rc
