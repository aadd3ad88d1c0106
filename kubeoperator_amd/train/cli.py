"""Training entry point of the bundled chart: ``torchrun --nproc-per-node=8 -m kubeoperator_amd.train.cli``.

Logs one JSON line per ``--log-every`` steps on rank 0 (step, loss, grad norm, lr, step time, tokens/s,
TFLOP/s per GPU), optionally also as Prometheus gauges on ``--metrics-port`` (``train.metrics``); checkpoints every ``--ckpt-every`` steps and resumes from the newest complete
checkpoint with ``--resume`` (elastic restarts via ``torchrun --max-restarts`` then continue where the
failed attempt left off).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def build_parser() -> argparse.ArgumentParser:
    """The CLI's arguments (also what the training chart's rendered Job args are checked against)."""
    ap = argparse.ArgumentParser(prog="kubeoperator_amd.train.cli")
    ap.add_argument("--model", default="llama3_8b")
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--mbs", type=int, default=1)
    ap.add_argument("--accum", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5, help="LR warmup steps")
    ap.add_argument("--lr", type=float, default=3e-4)
    ap.add_argument("--dp", default="auto", choices=["auto", "allreduce", "zero1"],
                    help="auto: ZeRO-1 when WORLD_SIZE > 1")
    ap.add_argument("--bucket-mb", type=int, default=512)
    ap.add_argument("--data", default="synthetic", help="'synthetic' or a flat uint16 token file")
    ap.add_argument("--ckpt-dir", default="")
    ap.add_argument("--ckpt-every", type=int, default=0)
    ap.add_argument("--resume", action="store_true")
    ap.add_argument("--log-every", type=int, default=1)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--gemm-tuning", default="use", choices=["off", "use", "tune"])
    ap.add_argument("--overlap-opt", type=int, default=1, choices=[0, 1])
    ap.add_argument("--fp8", type=int, default=0, choices=[0, 1],
                    help="E4M3 forward + data-gradient GEMMs of the Llama block projections (opt-in; reported "
                         "as dtype fp8-mixed)")
    ap.add_argument("--recompute", type=int, default=0, choices=[0, 1],
                    help="per-block activation recompute: only block inputs stay saved (long sequences, e.g. "
                         "Llama-3-8B at --seq 32768 on one GPU; ~1/3 more FLOPs)")
    ap.add_argument("--wgrad-stream", default="auto", choices=["auto", "on", "off"],
                    help="weight-gradient GEMMs on a second HIP stream beside the data-gradient chain (auto: models "
                         "narrower than 2048, +8 %% on GPT-2-small)")
    ap.add_argument("--grad-dtype", default="bf16", choices=["bf16", "fp32"],
                    help="gradient buffer precision (fp32: accumulation and DP reduction in fp32)")
    ap.add_argument("--cuda-graph", type=int, default=0, choices=[0, 1],
                    help="replay micro-batches as captured HIP graphs (one GPU; small micro-batches)")
    ap.add_argument("--sp", type=int, default=0, choices=[0, 1],
                    help="sequence parallelism with --tp > 1: norms, residual stream and LM head on 1/tp of the rows")
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel degree (Llama): TP groups of consecutive ranks, data parallelism across them")
    ap.add_argument("--metrics-port", type=int, default=0, help="rank 0 serves Prometheus metrics here (0: off)")
    ap.add_argument("--inject-fault", default="",
                    help="fault injection 'RANK:STEP': that rank dies abruptly after finishing STEP (before its "
                         "checkpoint) on the first attempt only (TORCHELASTIC_RESTART_COUNT 0), to exercise "
                         "torchrun --max-restarts + --resume")
    return ap


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    fault = None
    if a.inject_fault:
        fr, _, fs = a.inject_fault.partition(":")
        fault = (int(fr), int(fs))

    import torch

    from ..parallel.dist import all_reduce_max, init_distributed, shutdown
    from . import checkpoint
    from .data import SyntheticTokens, TokenFileDataset
    from .trainer import TrainConfig, Trainer, lr_at

    info = init_distributed(a.device)
    if a.dp == "auto":
        a.dp = "zero1" if info.world > 1 else "allreduce"
    from . import gemm_tuning

    gemm_tuning.setup(a.gemm_tuning, rank=info.rank)
    tc = TrainConfig(model=a.model, micro_batch=a.mbs, seq_len=a.seq, grad_accum=a.accum, lr=a.lr,
                     warmup_steps=a.warmup, total_steps=a.steps, dp_mode=a.dp, bucket_mb=a.bucket_mb, overlap_optimizer=bool(a.overlap_opt),
                     cuda_graph=bool(a.cuda_graph), grad_dtype=a.grad_dtype,
                     wgrad_stream=a.wgrad_stream, recompute=bool(a.recompute), fp8=bool(a.fp8), tp=a.tp, sp=bool(a.sp))
    tr = Trainer(tc, info)
    dpi = tr.dp_info  # the TP ranks of a group read the same tokens
    if a.resume and a.ckpt_dir:
        s = checkpoint.load(tr, a.ckpt_dir, info)
        if s is not None and info.is_main:
            print(json.dumps({"event": "resumed", "step": s}), flush=True)
    if a.data == "synthetic":
        data = SyntheticTokens(tr.cfg.vocab_size, a.mbs, a.seq, info.device, seed=tc.seed + tr.step, rank=dpi.rank)
    else:
        data = TokenFileDataset(a.data, a.mbs, a.seq, info.device, seed=tc.seed, rank=dpi.rank, world=dpi.world,
                                start_batch=tr.step * a.accum)
    cuda = info.device.type == "cuda"
    flops_tok = tr.cfg.flops_per_token(a.seq)
    metrics = None
    if a.metrics_port and info.is_main:
        from .metrics import TrainMetrics

        metrics = TrainMetrics(a.metrics_port, {"model": a.model, "world": str(info.world), "dp": a.dp})
    comm_seen = 0
    while tr.step < a.steps:
        t0 = time.perf_counter()
        loss = tr.train_step(data.batches(a.accum))
        if tr.step % a.log_every == 0:
            if cuda:
                torch.cuda.synchronize()
            dt = all_reduce_max(time.perf_counter() - t0, info)
            toks = tr.job_tokens_per_step / dt
            if info.is_main:
                rec = {"step": tr.step, "loss": round(float(loss), 4),
                       "grad_norm": round(float(tr.opt.last_grad_norm), 4),
                       "lr": lr_at(tr.step - 1, tc), "step_s": round(dt, 4), "tokens_per_s": round(toks, 1),
                       "tflops_per_gpu": round(flops_tok * toks / info.world / 1e12, 1)}
                print(json.dumps(rec), flush=True)
                if metrics is not None:
                    metrics.observe(step=rec["step"], loss=rec["loss"], grad_norm=rec["grad_norm"], lr=rec["lr"],
                                    step_s=dt, tokens_per_s=toks, tflops=rec["tflops_per_gpu"],
                                    comm_bytes_delta=tr.dp.comm_bytes - comm_seen)
                    comm_seen = tr.dp.comm_bytes
        if (fault is not None and (info.rank, tr.step) == fault
                and os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") == "0"):
            print(json.dumps({"event": "injected_fault", "rank": info.rank, "step": tr.step}), flush=True)
            os._exit(17)  # no cleanup, no barrier: a crashed worker as the elastic agent sees it
        if a.ckpt_dir and a.ckpt_every and tr.step % a.ckpt_every == 0:
            checkpoint.save(tr, a.ckpt_dir, info)
    if metrics is not None:
        metrics.close()
    shutdown(info)
    return 0


if __name__ == "__main__":
    sys.exit(main())
