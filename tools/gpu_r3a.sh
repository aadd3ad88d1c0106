#!/bin/bash
# Round 3, session A: side-stream fix under forced lag, bench-shape numerics, smoke, GPT-2 side-stream A/B,
# fresh attention PMC counters.
source "$(dirname "$0")/gpu_lib.sh"
mkdir -p gpurun_out/pmc
G2="python bench.py --model gpt2_small --seq 1024 --mbs 32 --steps 20 --warmup 5"
step wgrad 600 python -u -m pytest tests/test_wgrad_stream_gpu.py -x -v --timeout 200 --timeout-method thread && \
step shapes 900 python -u -m pytest tests/test_bench_shapes_gpu.py -x -v --timeout 400 --timeout-method thread && \
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" && \
step g2_auto1 300 $G2 --wgrad-stream auto && \
step g2_off1 300 $G2 --wgrad-stream off && \
step g2_auto2 300 $G2 --wgrad-stream auto && \
step g2_off2 300 $G2 --wgrad-stream off && \
pmc busy "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS" \
  python3 tools/bench_kernels.py --only attn --iters 3 --no-sdpa && \
pmc inst "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_ANY" \
  python3 tools/bench_kernels.py --only attn --iters 3 --no-sdpa && \
pmc grbm "GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
  python3 tools/bench_kernels.py --only attn --iters 3 --no-sdpa
