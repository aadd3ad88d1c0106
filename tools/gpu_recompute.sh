#!/bin/bash
# Activation recompute: GPU numerics test, then Llama-3-8B at seq 8192 without / with recompute and at 32768
# (recompute on; one sequence per micro-batch) inside one box session.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k recompute > gpurun_out/rc_tests.log 2>&1
rc=$?; echo "recompute tests rc=$rc"; tail -2 gpurun_out/rc_tests.log; [ $rc -eq 0 ] || exit $rc
i=0
for a in "--recompute 0" "--recompute 1" "--seq 32768 --accum 1 --recompute 1" "--seq 16384 --accum 2 --recompute 1"; do
  i=$((i + 1))
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 $a > gpurun_out/rc_$i.log 2>&1
  rc=$?; echo "[$i] $a rc=$rc $(grep -oE '"value": [0-9.]*|"ms_per_step": [0-9.]*|"peak_mem_gb_rank0": [0-9.]*|"tflops_per_gpu": [0-9.]*' gpurun_out/rc_$i.log | tr '\n' ' ')"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/rc_$i.log; exit $rc; }
done
