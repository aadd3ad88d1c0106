"""Host-side (Python) cost of the training step: cProfile over ``--steps`` optimizer steps of bench.py's trainer, with
the autograd engine on the calling thread (``torch.autograd.set_multithreading_enabled(False)``) so the backward's
Python -- the custom Functions' backward methods, the weight-gradient sinks, the side-stream groups -- is profiled
too (by default it runs on the engine's device thread, which cProfile does not see).

A launch blocks when the stream's queue is full (the host far ahead of the GPU), so time inside a launch call is not
all host cost; the host-only wall (``--no-sync`` steps timed without device synchronisation) against the device
step time says which side bounds the step.

usage: python tools/host_profile.py --model gpt2_small --seq 1024 --mbs 32 --accum 4 [--steps 4] [--top 40]
"""
from __future__ import annotations

import argparse
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2_small")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--mbs", type=int, default=32)
    ap.add_argument("--accum", type=int, default=4)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    import torch

    from kubeoperator_amd.parallel.dist import init_distributed
    from kubeoperator_amd.train import SyntheticTokens, TrainConfig, Trainer, gemm_tuning

    info = init_distributed("auto")
    gemm_tuning.setup("use", rank=0)
    tr = Trainer(TrainConfig(model=a.model, micro_batch=a.mbs, seq_len=a.seq, grad_accum=a.accum, warmup_steps=10,
                             total_steps=1000), info)
    data = SyntheticTokens(tr.cfg.vocab_size, a.mbs, a.seq, info.device, seed=1)
    for _ in range(a.warmup):
        tr.train_step(data.batches(a.accum))
    torch.cuda.synchronize()
    # device time per step
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.train_step(data.batches(a.accum))
    torch.cuda.synchronize()
    dev_ms = (time.perf_counter() - t0) / a.steps * 1e3
    # the host's own time per step: the same steps issued while the device runs a long sleep first, so no launch
    # finds a full queue before the host is done (the sleep is sized to cover the host's issue time)
    torch.autograd.set_multithreading_enabled(False)
    torch.cuda._sleep(int(1.0e9))  # ~0.5 s of GPU cycles queued ahead of the step
    t0 = time.perf_counter()
    tr.train_step(data.batches(a.accum))
    host_ms = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    prof = cProfile.Profile()
    torch.cuda._sleep(int(1.0e9))
    prof.enable()
    tr.train_step(data.batches(a.accum))
    prof.disable()
    torch.cuda.synchronize()
    print(f"device step {dev_ms:.2f} ms; host issue time of one step (device busy ahead of it) {host_ms:.2f} ms, "
          f"{host_ms / dev_ms * 100:.0f} % of the device step")
    st = pstats.Stats(prof)
    st.sort_stats("tottime").print_stats(a.top)
    st.sort_stats("cumulative").print_stats("kubeoperator_amd", a.top)


if __name__ == "__main__":
    main()
