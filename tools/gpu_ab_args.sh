#!/bin/bash
# A/B of bench.py argument sets inside ONE box session; sets separated by ';' in ARGSETS.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
IFS=';' read -ra SETS <<< "${ARGSETS:---mbs 1;--mbs 2;--mbs 1 --accum 2;--mbs 1}"
i=0
for a in "${SETS[@]}"; do
  i=$((i + 1))
  timeout -k 10 400 python bench.py --steps 8 --warmup 3 $a > gpurun_out/aa_$i.log 2>&1
  rc=$?; echo "[$i] $a rc=$rc $(grep -oE '"value": [0-9.]*|"ms_per_step": [0-9.]*|"peak_mem_gb_rank0": [0-9.]*' gpurun_out/aa_$i.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
