#!/bin/bash
# Data-parallel rehearsal on the one-GPU box: 2 and 4 ranks on cuda:0 over gloo, launched by torchrun like the
# driver launches bench.py; each rank runs the real GPU step (overlapped optimizer, ZeRO-1 gathers as gates).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
port=29560
for cfg in "2 zero1 1 bf16" "2 allreduce 1 bf16" "4 zero1 1 bf16" "4 allreduce 1 bf16" "2 zero1 2 bf16" \
           "4 zero1 4 bf16" "4 zero1 4 fp32" "2 allreduce 2 fp32"; do
  set -- $cfg
  port=$((port + 1))
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 \
    --master-port $port tools/dp_rehearsal.py --mode $2 --accum $3 --grad-dtype $4 > gpurun_out/dp_$1_$2_a$3_$4.log 2>&1
  rc=$?; echo "dp$1 $2 accum$3 $4 rc=$rc $(grep rehearsal gpurun_out/dp_$1_$2_a$3_$4.log)"; [ $rc -eq 0 ] || exit $rc
done
# Llama-3 1B proxy (vocab 128256, hidden 2048) with the production 512 MiB buckets
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29590 tools/dp_rehearsal.py --mode zero1 --model llama3_1b_proxy --seq 2048 --mbs 1 --bucket-mb 512 \
  > gpurun_out/dp_2_zero1_1b.log 2>&1
rc=$?; echo "dp2 zero1 1b rc=$rc $(grep rehearsal gpurun_out/dp_2_zero1_1b.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29591 tools/dp_rehearsal.py --mode allreduce --model llama3_1b_proxy --seq 2048 --mbs 1 --bucket-mb 512 \
  > gpurun_out/dp_2_allreduce_1b.log 2>&1
rc=$?; echo "dp2 allreduce 1b rc=$rc $(grep rehearsal gpurun_out/dp_2_allreduce_1b.log)"; [ $rc -eq 0 ] || exit $rc
# bench.py itself, launched exactly as the driver launches it, 2 ranks sharing the card (throughput meaningless)
KOP_DIST_BACKEND=gloo KOP_DEVICE_INDEX=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29592 bench.py --gpus 2 --steps 2 --warmup 1 --model llama3_1b_proxy --seq 2048 \
  > gpurun_out/dp_bench_2.log 2>&1
rc=$?; echo "bench dp2 rc=$rc $(grep metric gpurun_out/dp_bench_2.log | cut -c1-200)"; exit $rc
