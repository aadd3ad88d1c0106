#!/bin/bash
# FP8 projection GEMMs: GPU tests, then Llama-3-8B bf16 vs --fp8 alternating inside one box session.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/fp8_tests.log 2>&1
rc=$?; echo "fp8 tests rc=$rc"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/fp8_tests.log | head -12; [ $rc -eq 0 ] || exit $rc
i=0
for a in "--fp8 0" "--fp8 1" "--fp8 0" "--fp8 1"; do
  i=$((i + 1))
  timeout -k 10 400 python bench.py --steps 8 --warmup 3 $a > gpurun_out/f8_$i.log 2>&1
  rc=$?; echo "[$i] $a rc=$rc $(grep -oE '"value": [0-9.]*|"ms_per_step": [0-9.]*|"peak_mem_gb_rank0": [0-9.]*|"last_loss": [0-9.]*' gpurun_out/f8_$i.log | tr '\n' ' ')"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/f8_$i.log; exit $rc; }
done
