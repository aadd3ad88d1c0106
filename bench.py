"""Headline benchmark: training tokens/sec of the bundled Llama-3-8B PyTorch-ROCm chart on N MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 launched by torchrun,
one rank per GPU over RCCL. W untimed warmup steps, then EXACTLY K timed optimizer steps bracketed by a
barrier + device synchronize on both sides; the MAX step time over ranks is used; rank 0 prints one JSON
line. ``value`` is the whole-job throughput (sum over ranks = N x per-rank tokens / max time).

Every timed step is a complete training step: ``--accum`` micro-batches of forward through all 32 layers,
cross-entropy over the full 128,256 vocabulary and backward (gradients accumulated in the flat bf16 buffer),
bucketed RCCL gradient collectives overlapped with the last backward (N > 1; ZeRO-1 by default), gradient
clipping and the fused AdamW update of all 8.03 B parameters. Weights are random-init, tokens synthetic (no
network / datasets).

Launch: under torchrun (WORLD_SIZE set) every process is one rank. ``--gpus N > 1`` WITHOUT torchrun starts the
N ranks itself: ``python -m torch.distributed.run`` as a CHILD process (before this process imports torch or
touches a GPU; never an exec), whose rank 0 prints the JSON line; the exit code is the child's. A collective that
hangs fails the run after ``--comm-timeout`` seconds (RCCL watchdog abort) instead of burning the lease.

Communication evidence in the JSON (N > 1): ``backend``, ``rccl_world`` (``dist.get_world_size()``),
``grad_comm_bytes_per_step`` / ``param_gather_bytes_per_step`` (bytes each rank hands to the gradient
reduce-scatter or all-reduce / the ZeRO-1 all-gather per optimizer step) and ``exposed_comm_ms`` (per step, max
over ranks): the compute stream's stall between backward's last kernel and the completion of the last gradient
collective, plus its stalls on ZeRO-1 all-gather gates in the next forward -- CUDA-event timed on the GPU.
``runtime`` records torch / HIP / RCCL versions and every ``NCCL_*`` / ``RCCL_*`` / ``HSA_*`` / ``TORCH_NCCL_*`` /
``HIP_*`` variable in effect; ``gpu_telemetry_rank0`` the board power and shader clock sampled over the timed
steps (sysfs, read-only; per rank in ``ranks``); ``cpu_affinity_rank0`` the CPUs rank 0 was pinned to (N > 1: each rank is bound to
its GPU's NUMA-local CPUs and sizes its thread pool to them, ``parallel/dist.py`` ``bind_rank_cpus``, with the reason
of any fallback). ``ranks`` (N > 1): one record per rank -- its pinning, its exposed waits (``finish_wait_ms``: the
compute stream's stall for the last gradient collective; ``gate_wait_ms``: its stalls on ZeRO-1 all-gather gates) and
its bucket timeline (``parallel/ddp.py`` ``timeline_summary``: when the buckets' gradients were ready, relative to
backward's last kernel, and each collective's duration from RCCL's own events -- no extra stream). ``streams``: the
HIP streams the rank issues work on against ``GPU_MAX_HW_QUEUES``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _self_launch(n: int) -> int:
    """N ranks on this node via torchrun in a child process; stdout / stderr pass straight through (rank 0's
    JSON line included). Nothing here imports torch's CUDA runtime or touches a GPU."""
    import subprocess

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL peer buffers)
    # an even share of the CPUs this job may use per rank (each rank re-sizes its pool to the CPUs it is pinned to,
    # parallel/dist.py bind_rank_cpus): a fixed count per rank oversubscribes a small CPU share N-fold
    env.setdefault("OMP_NUM_THREADS", str(max(1, len(os.sched_getaffinity(0)) // n)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] --gpus {n} without torchrun: launching {n} ranks ({' '.join(cmd[1:6])} ...)", file=sys.stderr,
          flush=True)
    return subprocess.call(cmd, env=env)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama3_8b")
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--mbs", type=int, default=1, help="micro-batch (sequences) per rank")
    ap.add_argument("--accum", type=int, default=4,
                    help="gradient-accumulation micro-batches per optimizer step (default 4: 32k tokens per GPU per "
                         "step, 256k at 8 GPUs -- still far below the ~4M-token global batches Llama-3 pretraining "
                         "uses; one step per 8k-token micro-batch would be dominated by the 28 B/param update)")
    ap.add_argument("--dp", default="auto", choices=["auto", "allreduce", "zero1"],
                    help="auto: ZeRO-1 when WORLD_SIZE > 1 (reduce-scatter + sharded AdamW + all-gather: the same "
                         "bytes on xGMI as an all-reduce, 1/N of the optimizer's HBM traffic), else plain")
    ap.add_argument("--bucket-mb", type=int, default=512)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--gemm-tuning", default="use", choices=["off", "use", "tune"],
                    help="hipBLASLt solution selection: committed TunableOp winners (use), heuristic (off), re-tune")
    ap.add_argument("--overlap-opt", type=int, default=1, choices=[0, 1],
                    help="run AdamW on its own stream, gated per bucket into the next forward (1) or serially (0)")
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
                    help="replay each micro-batch's forward + backward as a captured HIP graph (one GPU only; pays "
                         "off when small micro-batches are bound by host-side launch overhead)")
    ap.add_argument("--sp", type=int, default=0, choices=[0, 1],
                    help="sequence parallelism with --tp > 1: norms, residual stream and LM head on 1/tp of the rows")
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel degree (Llama; TP groups of consecutive ranks, DP across them). The "
                         "headline runs tp 1: Llama-3-8B and its fp32 optimizer state fit one MI355X")
    ap.add_argument("--layers", type=int, default=0,
                    help="override the model's layer count (shape rehearsals of big models on one GPU; recorded in "
                         "the JSON config; never used for the headline)")
    ap.add_argument("--comm-timeout", type=int, default=300,
                    help="seconds before a hung collective aborts the run (RCCL watchdog; non-zero exit)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _self_launch(args.gpus)
    # a collective timeout tears the process group down and aborts the rank (non-zero exit, torchrun stops the rest)
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    # RCCL's own start / end events per collective: the bucket timeline reads them (Work._get_duration) instead of
    # a stream of its own waiting on every collective
    os.environ.setdefault("TORCH_NCCL_ENABLE_TIMING", "1")

    import torch

    from kubeoperator_amd.parallel.dist import (all_reduce_max, barrier, bind_rank_cpus, collectives_on,
                                                gather_objects, init_distributed, runtime_env, shutdown)
    from kubeoperator_amd.models import get_config
    from kubeoperator_amd.train import SyntheticTokens, TrainConfig, Trainer

    info = init_distributed(args.device, timeout_s=args.comm_timeout)
    affinity = bind_rank_cpus(info)  # multi-rank GPU jobs: each rank on the CPUs of its GPU's NUMA node
    if args.dp == "auto":
        args.dp = "zero1" if collectives_on(info) else "allreduce"
    from kubeoperator_amd.train import gemm_tuning

    tuning = gemm_tuning.setup(args.gemm_tuning, rank=info.rank)
    world = info.world
    if world != args.gpus:
        # launched by torchrun with another rank count than --gpus: never report a different job than was asked for
        if info.is_main:
            print(f"[bench] error: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        shutdown(info)
        return 2
    tc = TrainConfig(model=args.model, micro_batch=args.mbs, seq_len=args.seq, grad_accum=args.accum,
                     dp_mode=args.dp, bucket_mb=args.bucket_mb, warmup_steps=10, total_steps=1000,
                     overlap_optimizer=bool(args.overlap_opt),
                     transposed_weights=os.environ.get("KOP_TRANSPOSED_W", "1") != "0",
                     cuda_graph=bool(args.cuda_graph), grad_dtype=args.grad_dtype,
                     wgrad_stream=args.wgrad_stream, recompute=bool(args.recompute), fp8=bool(args.fp8), tp=args.tp, sp=bool(args.sp),
                     model_overrides={"n_layers": args.layers} if args.layers else {})
    trainer = Trainer(tc, info)
    dp_world = trainer.dp_info.world
    data = SyntheticTokens(trainer.cfg.vocab_size, args.mbs, args.seq, info.device, seed=tc.seed,
                           rank=trainer.dp_info.rank)
    cuda = info.device.type == "cuda"

    def sync():
        if cuda:
            torch.cuda.synchronize()

    loss = None
    for _ in range(args.warmup):
        loss = trainer.train_step(data.batches(args.accum))
    sync()
    barrier(info)
    sync()
    timing = cuda and collectives_on(info)
    if timing:  # exposed-communication events (a handful per step, no host synchronisation)
        trainer.dp.finish_waits, trainer.store.gate_waits = [], []
        # per-bucket timeline (ready events + RCCL's own durations); KOP_BENCH_TIMELINE=0 turns it off (A/B)
        trainer.dp.timeline = [] if os.environ.get("KOP_BENCH_TIMELINE", "1") != "0" else None
    comm0, gather0 = trainer.dp.comm_bytes, trainer.dp.gather_bytes
    # board power and shader clock of this rank's GPU over the timed steps (sysfs, read-only; the clock the
    # power cap leaves differs by a few % between boxes: train/gpu_telemetry.py)
    sampler = None
    if cuda and os.environ.get("KOP_BENCH_TELEMETRY", "1") != "0":  # 0: no sampler thread (A/B)
        from kubeoperator_amd.train.gpu_telemetry import PowerClockSampler

        sampler = PowerClockSampler(info.device.index or 0, period=0.5).start()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = trainer.train_step(data.batches(args.accum))
    sync()
    barrier(info)
    sync()
    elapsed = time.perf_counter() - t0
    telemetry = sampler.stop() if sampler is not None else None
    elapsed = all_reduce_max(elapsed, info)
    exposed_ms = None
    ranks = None
    if timing:
        trainer.store.await_all()  # the next step's gates: their waits belong to the timed steps' collectives
        sync()
        fin = sum(a.elapsed_time(b) for a, b in trainer.dp.finish_waits) / args.steps
        gate = sum(a.elapsed_time(b) for a, b in trainer.store.gate_waits) / args.steps
        exposed_ms = all_reduce_max(fin + gate, info)
        # per rank: what it was pinned to, its bucket timeline and its two exposed-wait components (all ranks' records
        # land in rank 0's JSON line, so a slow rank or a late bucket is attributable)
        from kubeoperator_amd.parallel.ddp import timeline_summary

        rec = {"rank": info.rank, "affinity": affinity, "gpu_telemetry": telemetry,
               "finish_wait_ms": round(fin, 3), "gate_wait_ms": round(gate, 3),
               "gate_waits_per_step": len(trainer.store.gate_waits) // max(1, args.steps),
               "buckets": timeline_summary(trainer.dp.timeline) if trainer.dp.timeline is not None else None}
        ranks = gather_objects(rec, info)
        trainer.dp.finish_waits = trainer.store.gate_waits = trainer.dp.timeline = None
    streams = stream_inventory(trainer, collectives_on(info)) if cuda else None
    comm_step = (trainer.dp.comm_bytes - comm0) // max(1, args.steps)
    gather_step = (trainer.dp.gather_bytes - gather0) // max(1, args.steps)
    gemm_tuning.finish(tuning, info.rank)
    last_loss = float(loss.item()) if loss is not None else float("nan")
    tokens = trainer.job_tokens_per_step * args.steps
    value = tokens / elapsed
    ms = elapsed / args.steps * 1000.0
    cfg = trainer.cfg
    flops_tok = cfg.flops_per_token(args.seq)
    mem_gb = torch.cuda.max_memory_allocated() / 1e9 if cuda else 0.0
    reserved_gb = torch.cuda.max_memory_reserved() / 1e9 if cuda else 0.0
    if info.is_main:
        model_name = {"llama3_8b": "Llama-3-8B", "gpt2_small": "GPT-2-small",
                      "llama3_70b": "Llama-3-70B"}.get(args.model, args.model)
        if args.layers:
            model_name += f" ({args.layers} of {get_config(args.model).n_layers} layers)"
        out = {
            "metric": "tokens/sec of bundled Llama-3-8B pod" if args.model == "llama3_8b" and not args.layers
            else f"tokens/sec of bundled {model_name} pod",
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp8-mixed (E4M3 projection GEMMs, bf16 elsewhere)" if args.fp8 else "bf16",
            "data": "synthetic (random token ids generated on device; random-init weights)",
            "config": {
                "model": model_name,
                "params": cfg.num_params(),
                "global_batch": args.mbs * args.accum * dp_world,
                "micro_batch_per_gpu": args.mbs,
                "grad_accum": args.accum,
                "seq_len": args.seq,
                "parallelism": (f"tp{args.tp}-" if args.tp > 1 else "") + ("sp-" if args.sp and args.tp > 1 else "")
                + f"dp{dp_world}"
                + ("-zero1" if args.dp == "zero1" and (dp_world > 1 or collectives_on(info)) else ""),
                "optimizer": "fused AdamW (fp32 master/moments), grad clip 1.0",
                "optimizer_overlap": bool(args.overlap_opt),
                "hip_graph": bool(args.cuda_graph),
                "grad_dtype": args.grad_dtype,
                "wgrad_stream": trainer.store.wgrad_stream,
                "recompute": bool(args.recompute),
            },
            "tflops_per_gpu": round(flops_tok * value / world / 1e12, 1),
            "last_loss": round(last_loss, 4),
            "peak_mem_gb_rank0": round(mem_gb, 1),
            "peak_reserved_gb_rank0": round(reserved_gb, 1),
            "setup_s": round(trainer.setup_seconds, 1),
            "gemm_selection": tuning,
            "backend": info.backend,
            "rccl_world": _dist_world(),
            "grad_comm_bytes_per_step": int(comm_step),
            "param_gather_bytes_per_step": int(gather_step),
            "exposed_comm_ms": round(exposed_ms, 3) if exposed_ms is not None else None,
            "cpu_affinity_rank0": affinity,
            "gpu_telemetry_rank0": telemetry,
            "streams": streams,
            "ranks": ranks,
            "runtime": runtime_env(),
        }
        print(json.dumps(out), flush=True)
    dump = os.environ.get("KOP_BENCH_DUMP_PARAMS")  # tests: the final parameters, layout order, no padding
    if dump and info.is_main:
        torch.save(torch.cat([p.detach().reshape(-1).float().cpu() for _, p in trainer.store.named_params()]), dump)
    shutdown(info)
    return 0


def stream_inventory(trainer, rccl: bool) -> dict:
    """The HIP streams this rank issues work on, against the hardware queues a process gets (GPU_MAX_HW_QUEUES,
    HIP's default 4): more streams than queues share queues, and work queued behind another stream's barrier
    packets then waits for it. Warns on stderr when they do not fit."""
    names = ["compute"]
    if getattr(trainer.opt, "overlap", False):
        names.append("optimizer")
    if trainer.store.wgrad_stream:
        names.append("wgrad")
    if rccl:
        names.append("rccl")
    queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    fits = len(names) <= queues
    if not fits:
        print(f"[bench] warning: {len(names)} streams ({', '.join(names)}) > GPU_MAX_HW_QUEUES={queues}",
              file=sys.stderr, flush=True)
    return {"in_use": names, "hw_queues": queues, "fits": fits}


def _dist_world() -> int:
    import torch.distributed as dist

    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


if __name__ == "__main__":
    sys.exit(main())
