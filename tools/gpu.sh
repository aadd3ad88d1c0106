#!/bin/bash
# GPU sessions on a one-GPU MI355X box, one entry point:
#   /usr/local/graft/bin/gpurun --timeout N -- bash tools/gpu.sh <session> [<session> ...]
# Sessions run in order and stop at the first failing step (every step has its own time limit, no retries).
# Logs land in gpurun_out/<step>.log; the summaries worth keeping are copied into profiles/.
#
#   check        GPU test suite, smoke(), Llama-3-8B and GPT-2-small benches (what the driver runs at round end)
#   tests        the GPU test suite only (SEL=<pytest selection> narrows it)
#   bench        Llama-3-8B bench (ARGSETS="--a;ENV=1 --b" runs several env / argument sets back to back: same-box A/B)
#   gpt2         GPT-2-small bench (ARGSETS as above)
#   prof-l8b     rocprofv3 kernel trace + stats of the Llama-3-8B step
#   prof-gpt2    rocprofv3 kernel trace + stats of the GPT-2-small step
#   pmc-attn     PMC counter passes (one rocprofv3 run each) over the attention micro-benchmark
#   attn-probe   attention TF/s per shape; VARIANTS="ENV=a;ENV=b;base" alternates env variants twice
#   attn-prof    rocprofv3 kernel trace of the attention probe per VARIANTS entry (per-kernel times), then PMC passes
#                over the first entry
#   rccl1        one-rank RCCL self-test (KOP_RCCL_SELFTEST=1): the bench's data-parallel collectives through RCCL
#                under torchrun on one GPU -- 1B proxy (ZeRO-1, all-reduce) and Llama-3-8B (ZeRO-1)
#   dp           one-GPU data-parallel rehearsals (2 / 4 gloo ranks sharing cuda:0) + bench.py --gpus 2 under torchrun
#   tp           one-GPU tensor (+ sequence) parallel rehearsals + bench.py --tp 2 [--sp 1] + 4 Llama-3-70B layers
#   wgrad-lag    weight-gradient and optimizer streams under a forced lag: GPU tests, then DP / TP rehearsals
#   wgrad-splitk weight-gradient GEMM forms at the training shapes (tools/bench_wgrad_splitk.py)
#   tune         TunableOp tuning of the training GEMMs, then heuristic vs tuned bench
#   tune-decode  TunableOp tuning of the decode GEMMs, then the decode benchmark
#   serve        serving tests, decode benchmark, continuous-batching benchmark
#   fp8          FP8 GPU tests and the opt-in --fp8 Llama-3-8B bench
#   roofline     every library GEMM of the Llama-3-8B step, in-step vs isolated, with power / clock samples
source "$(dirname "$0")/gpu_lib.sh"
mkdir -p gpurun_out/prof gpurun_out/pmc

L8B="${L8B:-python bench.py --steps 10 --warmup 3}"
G2="python bench.py --model gpt2_small --seq 1024 --mbs 64 --accum 2 --steps 20 --warmup 5"
port=29700

torchrun_n() {  # name limit nproc args...
  local name=$1 lim=$2 n=$3; shift 3; port=$((port + 1))
  step "$name" "$lim" python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
    --master-port $port "$@"
}

argsets() {  # tag base-command: one bench per ';'-separated ARGSETS entry (default: the base command once);
  # an entry's leading NAME=value words are environment settings, the rest bench arguments
  local tag=$1 base=$2 i=0 a tok
  IFS=';' read -ra SETS <<< "${ARGSETS:-}"
  [ ${#SETS[@]} -eq 0 ] && SETS=("")
  for a in "${SETS[@]}"; do
    i=$((i + 1))
    local envs=() args=()
    for tok in $a; do
      if [ ${#args[@]} -eq 0 ] && [[ $tok == *=* && $tok != -* ]]; then envs+=("$tok"); else args+=("$tok"); fi
    done
    step "${tag}_$i" 400 env "${envs[@]}" $base "${args[@]}" || return $?
    grep -h '"metric"' "gpurun_out/${tag}_$i.log" | sed "s|^|[$a] |" | tee -a "gpurun_out/$tag.jsonl"
  done
}

s_tests() {
  step tests_gpu 900 python -u -m pytest ${SEL:-tests} -m gpu -x -v --timeout 240 --timeout-method thread
}
s_smoke() { step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; }
s_bench() { argsets l8b "$L8B"; }
s_gpt2() { argsets gpt2 "$G2"; }
s_check() { s_tests && s_smoke && step bench 400 $L8B && step gpt2 300 $G2; }

s_prof_l8b() {
  step prof_l8b 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/l8b -o l8b --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1
}
s_prof_gpt2() {
  step prof_gpt2 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/gpt2 -o gpt2 --output-format csv -- \
    python3 bench.py --model gpt2_small --seq 1024 --mbs 64 --accum 2 --steps 3 --warmup 2
}

s_pmc_attn() {
  local prog="python3 tools/bench_kernels.py --only attn --iters 3 --no-sdpa"
  pmc busy "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS" $prog && \
  pmc inst "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_ANY" $prog && \
  pmc grbm "GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" $prog && \
  python tools/pmc_summary.py $(find gpurun_out/pmc -name '*counter_collection.csv') > gpurun_out/pmc_summary.txt
}

s_attn_probe() {
  local out=gpurun_out/attn_probe.jsonl v envs rep rc
  : > $out
  IFS=';' read -ra VS <<< "${VARIANTS:-base}"
  for rep in 1 2; do
    for v in "${VS[@]}"; do
      [ "$v" = "base" ] && envs="" || envs="$v"
      env $envs KOP_PROBE_TAG="$v" timeout -k 10 120 python tools/attn_probe.py --shapes "${SHAPES:-llama,guide}" \
        >> $out 2> gpurun_out/attn_probe.err
      rc=$?; [ $rc -eq 0 ] || { echo "variant '$v' rc=$rc"; tail -5 gpurun_out/attn_probe.err; return $rc; }
    done
  done
  cat $out
}

s_attn_prof() {
  local v envs i=0 prog="python3 tools/attn_probe.py --shapes ${SHAPES:-llama} --causal 1 --iters 6"
  IFS=';' read -ra VS <<< "${VARIANTS:-base}"
  for v in "${VS[@]}"; do
    i=$((i + 1)); [ "$v" = "base" ] && envs="" || envs="$v"
    (export $envs; step attn_prof_$i 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/attn_$i -o attn_$i \
      --output-format csv -- $prog) || return $?
  done
  v="${VS[0]}"; [ "$v" = "base" ] && envs="" || envs="$v"
  (export $envs
   pmc abusy "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS" $prog && \
   pmc ainst "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_ANY" $prog && \
   pmc agrbm "GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" $prog) && \
  python tools/pmc_summary.py $(find gpurun_out/pmc -name '*counter_collection.csv') > gpurun_out/pmc_attn_summary.txt
}

rehearse() {  # nproc script args...: the rehearsal's JSON line is appended to gpurun_out/rehearsals.jsonl
  local n=$1; shift
  torchrun_n "reh_$((port + 1))" 300 "$n" "$@" && grep -h rehearsal "gpurun_out/reh_$port.log" | tee -a gpurun_out/rehearsals.jsonl
}

s_rccl1() {
  export KOP_RCCL_SELFTEST=1
  torchrun_n rccl1_zero1 300 1 bench.py --gpus 1 --steps 3 --warmup 1 --model llama3_1b_proxy --seq 2048 && \
  torchrun_n rccl1_allreduce 300 1 bench.py --gpus 1 --steps 3 --warmup 1 --model llama3_1b_proxy --seq 2048 \
    --dp allreduce && \
  torchrun_n rccl1_l8b 400 1 bench.py --gpus 1 --steps 5 --warmup 2 && \
  grep -h '"metric"' gpurun_out/rccl1_*.log | tee gpurun_out/rccl1.jsonl
  local rc=$?; unset KOP_RCCL_SELFTEST; return $rc
}

s_dp() {
  rehearse 2 tools/dp_rehearsal.py --mode zero1 && \
  rehearse 2 tools/dp_rehearsal.py --mode allreduce && \
  rehearse 4 tools/dp_rehearsal.py --mode zero1 --accum 4 && \
  rehearse 4 tools/dp_rehearsal.py --mode zero1 --accum 4 --grad-dtype fp32 && \
  rehearse 2 tools/dp_rehearsal.py --mode allreduce --accum 2 --grad-dtype fp32 && \
  rehearse 2 tools/dp_rehearsal.py --mode zero1 --model llama3_1b_proxy --seq 2048 --mbs 1 --bucket-mb 512 && \
  KOP_DIST_BACKEND=gloo KOP_DEVICE_INDEX=0 torchrun_n bench_dp2 300 2 bench.py --gpus 2 --steps 2 --warmup 1 \
    --model llama3_1b_proxy --seq 2048
}

s_tp() {
  rehearse 2 tools/tp_rehearsal.py --tp 2 --mode zero1 --out /tmp/kop_tp_a && \
  rehearse 4 tools/tp_rehearsal.py --tp 2 --mode zero1 --out /tmp/kop_tp_b && \
  rehearse 4 tools/tp_rehearsal.py --tp 2 --mode allreduce --sp 1 --out /tmp/kop_tp_c && \
  rehearse 4 tools/tp_rehearsal.py --tp 4 --mode zero1 --model llama3_1b_proxy --mbs 1 --out /tmp/kop_tp_d && \
  KOP_DIST_BACKEND=gloo KOP_DEVICE_INDEX=0 torchrun_n bench_tp2 300 2 bench.py --gpus 2 --tp 2 --steps 2 --warmup 1 \
    --model llama3_1b_proxy --seq 2048 && \
  KOP_DIST_BACKEND=gloo KOP_DEVICE_INDEX=0 torchrun_n bench_tp2_sp 300 2 bench.py --gpus 2 --tp 2 --sp 1 --steps 2 \
    --warmup 1 --model llama3_1b_proxy --seq 2048 && \
  KOP_DIST_BACKEND=gloo KOP_DEVICE_INDEX=0 torchrun_n tp70b 600 2 bench.py --gpus 2 --tp 2 --model llama3_70b --layers 4 \
    --recompute 1 --sp 1 --seq 8192 --mbs 1 --accum 1 --steps 2 --warmup 1 --gemm-tuning off
}

s_wgrad_lag() {
  step wgrad_tests 600 python -u -m pytest tests/test_wgrad_stream_gpu.py tests/test_stream_lag_gpu.py -x -v --timeout 200 \
    --timeout-method thread && (
    export KOP_WGRAD_STREAM=1 KOP_SIDE_LAG_CYCLES=200000 KOP_OPTIM_LAG_CYCLES=200000
    rehearse 2 tools/dp_rehearsal.py --mode zero1 && \
    rehearse 4 tools/dp_rehearsal.py --mode zero1 --accum 4 && \
    rehearse 4 tools/dp_rehearsal.py --mode allreduce && \
    rehearse 2 tools/dp_rehearsal.py --mode zero1 --model tiny_gpt2 --accum 2 && \
    rehearse 4 tools/tp_rehearsal.py --tp 2 --mode zero1 --sp 1 --out /tmp/kop_tp_lag
  )
}

s_wgrad_splitk() {
  step wgrad_splitk 600 python tools/bench_wgrad_splitk.py ${SPLITK_ARGS:-} && \
    grep -h '^{' gpurun_out/wgrad_splitk.log > gpurun_out/wgrad_splitk.jsonl
}

s_tune() {
  PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=0 KOP_TUNE_MS=100 KOP_TUNE_ITERS=30 step tune 700 python tools/tune_gemms.py && \
  cp kubeoperator_amd/tuning/tunableop_results_gfx950.csv gpurun_out/ && \
  step bench_tune_off 600 $L8B --gemm-tuning off && \
  step bench_tune_use 600 $L8B --gemm-tuning use
}

s_tune_decode() {
  KOP_TUNE_MS=60 KOP_TUNE_ITERS=20 step tune_decode 900 python tools/bench_decode.py --batch 1,16,64,128 --prompt 128 \
    --steps 2 --graph 0 --gemm-tuning tune --gemm-results gpurun_out/tunableop_results_gfx950_decode.csv && \
  step decode_tuned 400 python tools/bench_decode.py --batch 1,16,64,128 --prompt 2048 --steps 32 --graph 0,1 \
    --gemm-tuning use --gemm-results gpurun_out/tunableop_results_gfx950_decode.csv
}

s_serve() {
  step serve_tests 300 python -u -m pytest tests/test_serve.py -x -v --timeout 120 --timeout-method thread && \
  step decode 400 python tools/bench_decode.py --batch 1,16,64,128 --prompt 2048 --steps 32 --graph 0,1 && \
  step serve_bench 500 python tools/bench_serve.py --requests 256 --slots 128 --prompt 256,2048 --new 128
}

s_fp8() {
  step fp8_tests 300 python -u -m pytest tests/test_fp8_gpu.py -x -v --timeout 120 --timeout-method thread && \
  step fp8_bench 400 $L8B --fp8 1
}

s_roofline() {
  step gemm_roofline 900 python tools/gemm_roofline.py --out gpurun_out/gemm_roofline.jsonl
}

[ $# -gt 0 ] || { sed -n '2,23p' tools/gpu.sh; exit 2; }
for s in "$@"; do
  fn="s_${s//-/_}"
  declare -F "$fn" > /dev/null || { echo "unknown session: $s"; exit 2; }
  echo "##### session $s $(date +%T)"
  "$fn" || exit $?
done
