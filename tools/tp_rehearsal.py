"""Tensor-parallel rehearsal on ONE GPU: the ranks of a TP (x DP) job share cuda:0 over gloo (RCCL refuses two
ranks on one device) and run the real GPU step -- HIP kernels on each rank's heads / FFN slice, TP all-reduces
in forward and backward, flat bucketed DP collectives, the optimizer on its own stream. Every rank starts from
the same full weights (``Trainer.load_full_weights``); rank 0 then trains one process holding the whole model on
the global batch and compares every rank's shards with the matching slices (shards travel through a file).

  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 \
      tools/tp_rehearsal.py --tp 2
"""
import argparse
import json
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def global_batch(vocab, dp, step, mbs, seq):
    g = torch.Generator().manual_seed(100 + step)
    ids = torch.randint(0, vocab, (mbs * dp, seq + 1), generator=g)
    return ids[:, :-1].contiguous(), ids[:, 1:].contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=2)
    ap.add_argument("--mode", default="zero1", choices=["zero1", "allreduce"])
    ap.add_argument("--sp", type=int, default=0, choices=[0, 1], help="sequence parallelism on top of TP")
    ap.add_argument("--model", default="tiny_llama")
    ap.add_argument("--seq", type=int, default=256)
    ap.add_argument("--mbs", type=int, default=2)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(tempfile.gettempdir(), "kop_tp_rehearsal"))
    a = ap.parse_args()
    os.environ.setdefault("KOP_DIST_BACKEND", "gloo")
    os.environ.setdefault("KOP_DEVICE_INDEX", "0")
    from kubeoperator_amd.parallel.dist import DistInfo, barrier, init_distributed, shutdown
    from kubeoperator_amd.parallel.tensor import shard_llama_weight
    from kubeoperator_amd.train import TrainConfig, Trainer

    info = init_distributed("cuda" if torch.cuda.is_available() else "cpu")
    kw = dict(model=a.model, seq_len=a.seq, warmup_steps=1, total_steps=10, bucket_mb=1, lr=1e-1, eps=1.0)
    one_info = DistInfo(0, 0, 1, "none", info.device)
    full = {n: p.detach().clone() for n, p in Trainer(TrainConfig(**kw), one_info).store.named_params()}
    tr = Trainer(TrainConfig(micro_batch=a.mbs, dp_mode=a.mode, tp=a.tp, sp=bool(a.sp), **kw), info)
    tr.load_full_weights(full)
    dp, dpr = tr.dp_info.world, tr.dp_info.rank
    sl = slice(a.mbs * dpr, a.mbs * (dpr + 1))
    for step in range(a.steps):
        ids, tgt = global_batch(tr.cfg.vocab_size, dp, step, a.mbs, a.seq)
        tr.train_step([(ids[sl].to(info.device), tgt[sl].to(info.device))])
    tr.store.await_all()
    if info.device.type == "cuda":
        torch.cuda.synchronize()
    os.makedirs(a.out, exist_ok=True)
    torch.save({n: p.detach().float().cpu() for n, p in tr.store.named_params()},
               os.path.join(a.out, f"rank{info.rank}.pt"))
    barrier(info)
    shutdown(info)
    if info.rank != 0:
        return 0
    one = Trainer(TrainConfig(micro_batch=a.mbs * dp, **kw), one_info)
    one.load_full_weights(full)
    for step in range(a.steps):
        ids, tgt = global_batch(one.cfg.vocab_size, dp, step, a.mbs, a.seq)
        one.train_step([(ids.to(info.device), tgt.to(info.device))])
    one.store.await_all()
    want = {n: p.detach().float().cpu() for n, p in one.store.named_params()}
    num = den = 0.0
    for r in range(info.world):
        got = torch.load(os.path.join(a.out, f"rank{r}.pt"), weights_only=True)
        t = r % a.tp
        for n, g in got.items():
            w = shard_llama_weight(n, want[n], one.cfg, a.tp, t)
            w0 = shard_llama_weight(n, full[n].float().cpu(), one.cfg, a.tp, t)
            num += float((g - w).pow(2).sum())
            den += float((w - w0).pow(2).sum())
    rel = (num / max(den, 1e-30)) ** 0.5
    ok = rel < 0.05
    print(json.dumps({"rehearsal": f"tp{a.tp}-" + ("sp-" if a.sp else "") + f"dp{dp}-{a.mode}", "model": a.model, "rel_update_error": rel,
                      "ok": ok, "buckets": len(tr.store.buckets), "optimizer_overlap": tr.opt.overlap}), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
