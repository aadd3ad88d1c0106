#!/bin/bash
# Tensor-parallel rehearsal on the one-GPU box (ranks share cuda:0 over gloo), launched by torchrun like the
# driver launches bench.py: tp2, tp2 x dp2 (ZeRO-1), tp4; then bench.py --tp 2 on the Llama-3 1B proxy
# (throughput meaningless: the ranks share one card and gloo copies through the host).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
port=29660
for cfg in "2 2 zero1" "4 2 zero1" "4 2 allreduce" "4 4 zero1 --model llama3_1b_proxy --mbs 1" "2 2 zero1 --sp 1" \
           "4 2 zero1 --sp 1" "4 2 allreduce --sp 1"; do
  set -- $cfg; extra="${*:4}"
  port=$((port + 1))
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 \
    --master-port $port tools/tp_rehearsal.py --tp $2 --mode $3 $extra --out /tmp/kop_tp_$port > gpurun_out/tp_$1_$2_$3_$port.log 2>&1
  rc=$?; echo "world$1 tp$2 $3 $extra rc=$rc $(grep rehearsal gpurun_out/tp_$1_$2_$3_$port.log)"; [ $rc -eq 0 ] || exit $rc
done
KOP_DIST_BACKEND=gloo KOP_DEVICE_INDEX=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29690 bench.py --gpus 2 --tp 2 --steps 2 --warmup 1 --model llama3_1b_proxy \
  --seq 2048 > gpurun_out/tp_bench_2.log 2>&1
rc=$?; echo "bench tp2 rc=$rc $(grep metric gpurun_out/tp_bench_2.log | cut -c1-300)"; [ $rc -eq 0 ] || exit $rc
KOP_DIST_BACKEND=gloo KOP_DEVICE_INDEX=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29691 bench.py --gpus 2 --tp 2 --sp 1 --steps 2 --warmup 1 --model llama3_1b_proxy \
  --seq 2048 > gpurun_out/tp_bench_2_sp.log 2>&1
rc=$?; echo "bench tp2 sp rc=$rc $(grep metric gpurun_out/tp_bench_2_sp.log | cut -c1-300)"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_tp70b_rehearsal.sh
