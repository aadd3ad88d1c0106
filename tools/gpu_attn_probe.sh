#!/bin/bash
# Attention probe on one MI355X: every variant listed in $VARIANTS ("ENV=val ENV2=val;..." separated by ';',
# "base" for defaults), alternating twice, inside one box session.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
VARIANTS=${VARIANTS:-base}
SHAPES=${SHAPES:-llama,guide}
out=gpurun_out/attn_probe.jsonl
: > $out
for rep in 1 2; do
  IFS=';' read -ra VS <<< "$VARIANTS"
  for v in "${VS[@]}"; do
    if [ "$v" = "base" ]; then envs=""; else envs="$v"; fi
    env $envs KOP_PROBE_TAG="$v" timeout -k 10 120 python tools/attn_probe.py --shapes $SHAPES >> $out 2>gpurun_out/attn_probe.err
    rc=$?; [ $rc -eq 0 ] || { echo "variant '$v' rc=$rc"; tail -5 gpurun_out/attn_probe.err; exit $rc; }
  done
done
cat $out
