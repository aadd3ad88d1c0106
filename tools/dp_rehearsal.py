"""Data-parallel rehearsal on ONE GPU: several ranks share cuda:0 over gloo (RCCL refuses two ranks on one
device) and run the real GPU training step -- HIP kernels, flat bucketed gradients, the optimizer on its own
stream and, for ZeRO-1, the per-bucket in-place all-gather issued on that stream as the next forward's gate.
Rank 0 then trains one process on the global batch and checks the parameters match.

Launch it the way the driver launches bench.py (the launcher process never touches the GPU):
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 \
      tools/dp_rehearsal.py --mode zero1
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def global_batch(vocab, world, step, mbs, seq):
    g = torch.Generator().manual_seed(100 + step)  # step = optimizer step * accum + micro-batch
    ids = torch.randint(0, vocab, (mbs * world, seq + 1), generator=g)
    return ids[:, :-1].contiguous(), ids[:, 1:].contiguous()


def flat(tr):
    return torch.cat([p.detach().reshape(-1).float().cpu() for _, p in tr.store.named_params()])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="zero1", choices=["zero1", "allreduce"])
    ap.add_argument("--model", default="tiny_llama")
    ap.add_argument("--seq", type=int, default=256)
    ap.add_argument("--mbs", type=int, default=2)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--accum", type=int, default=1, help="gradient-accumulation micro-batches per step")
    ap.add_argument("--bucket-mb", type=int, default=1)
    ap.add_argument("--grad-dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--lr", type=float, default=1e-1, help="large, so a missing or double update is visible")
    ap.add_argument("--eps", type=float, default=1.0,
                    help="Adam eps >> |grad|: the update is ~linear in the gradient instead of +-lr per element, so "
                         "reduction-order noise cannot flip the sign of near-zero-gradient updates")
    a = ap.parse_args()
    os.environ.setdefault("KOP_DIST_BACKEND", "gloo")
    os.environ.setdefault("KOP_DEVICE_INDEX", "0")
    from kubeoperator_amd.parallel.dist import DistInfo, init_distributed, shutdown
    from kubeoperator_amd.train import TrainConfig, Trainer

    info = init_distributed("cuda" if torch.cuda.is_available() else "cpu")
    world, rank = info.world, info.rank
    kw = dict(model=a.model, seq_len=a.seq, warmup_steps=1, total_steps=10, bucket_mb=a.bucket_mb,
              overlap_optimizer=True, lr=a.lr, eps=a.eps, grad_dtype=a.grad_dtype)
    tr = Trainer(TrainConfig(micro_batch=a.mbs, grad_accum=a.accum, dp_mode=a.mode, **kw), info)
    init = flat(tr)
    sl = slice(a.mbs * rank, a.mbs * (rank + 1))
    for step in range(a.steps):
        mb = [global_batch(tr.cfg.vocab_size, world, step * a.accum + i, a.mbs, a.seq) for i in range(a.accum)]
        tr.train_step([(ids[sl].to(info.device), tgt[sl].to(info.device)) for ids, tgt in mb])
    tr.store.await_all()
    if info.device.type == "cuda":
        torch.cuda.synchronize()
    got = flat(tr)
    shutdown(info)
    if rank != 0:
        return 0
    one = Trainer(TrainConfig(micro_batch=a.mbs * world, grad_accum=a.accum, **kw), DistInfo(0, 0, 1, "none", info.device))
    for step in range(a.steps):
        mb = [global_batch(one.cfg.vocab_size, world, step * a.accum + i, a.mbs, a.seq) for i in range(a.accum)]
        one.train_step([(ids.to(info.device), tgt.to(info.device)) for ids, tgt in mb])
    one.store.await_all()
    want = flat(one)
    # relative error of the whole update: a lost, doubled or stale bucket update makes it O(1); bf16
    # reduction-order noise keeps it at a few percent
    upd = (want - init).norm().item()
    rel = (got - want).norm().item() / max(upd, 1e-30)
    ok = rel < 0.05
    print(json.dumps({"rehearsal": f"dp{world}-{a.mode}", "accum": a.accum, "model": a.model, "rel_update_error": rel,
                      "update_norm": upd, "max_abs_param_diff": (got - want).abs().max().item(), "ok": ok,
                      "buckets": len(tr.store.buckets), "optimizer_overlap": tr.opt.overlap}), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
