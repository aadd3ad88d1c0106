"""Per-parameter gradient comparison of one Llama micro-batch with the transposed-companion norms on vs off
(``KOP_NORM_T``): prints one JSON line per parameter with the relative difference of its gradient. A wiring
mistake shows up as one parameter family far above bf16 noise.
Usage: python tools/norm_t_check.py [--model llama3_1b_proxy] [--layers 2] [--seq 2048]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def grads(on, a):
    from kubeoperator_amd.ops import functional
    from kubeoperator_amd.parallel.dist import DistInfo
    from kubeoperator_amd.train import TrainConfig, Trainer

    functional._NORM_T = on
    tr = Trainer(TrainConfig(model=a.model, micro_batch=1, seq_len=a.seq, grad_accum=1, bucket_mb=64,
                             grad_clip=0.0, model_overrides={"n_layers": a.layers}),
                 DistInfo(0, 0, 1, "none", torch.device("cuda", 0)))
    gen = torch.Generator().manual_seed(5)
    ids = torch.randint(0, tr.cfg.vocab_size, (1, a.seq + 1), generator=gen)
    tr.store.begin_microbatch(0)
    loss = tr.model(ids[:, :-1].cuda(), ids[:, 1:].cuda())
    print(json.dumps({"norm_t": on, "loss": loss.item()}), flush=True)
    loss.backward()
    tr.store.join_side()
    torch.cuda.synchronize()
    return {n: p.main_grad.float().clone() for n, p in tr.store.named_params()}


def kernels(T=2048, H=2048):
    """The companion kernels against the plain ones on the same inputs: fraction of bf16 outputs that differ."""
    from kubeoperator_amd.ops.functional import _lib

    lib = _lib()
    g = torch.Generator(device="cuda").manual_seed(1)
    x, r, dy, dr = (torch.randn(T, H, device="cuda", generator=g).bfloat16() for _ in range(4))
    w = (1 + 0.1 * torch.randn(H, device="cuda", generator=g)).bfloat16()
    y0, s0, rstd0, _ = lib.norm_fwd(x, r, w, None, 1e-5, False)
    y1, s1, rstd1, yt = lib.rms_norm_fwd_t(x, r, w, 1e-5)
    dw0, dw1 = torch.zeros_like(w), torch.zeros_like(w)
    dx0 = lib.norm_bwd(dy, s0, w, rstd0, None, dr, dw0, None, False, False)
    dx1, dxt = lib.rms_norm_bwd_t(dy, s0, w, rstd0, dr, dw1, False)
    for name, a0, a1 in (("y", y0, y1), ("s", s0, s1), ("rstd", rstd0, rstd1), ("dx", dx0, dx1), ("dw", dw0, dw1)):
        print(json.dumps({"kernel": name, "frac_differ": (a0 != a1).float().mean().item(),
                          "max_rel": ((a0.float() - a1.float()).abs().max() / a0.float().abs().max()).item()}),
              flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3_1b_proxy")
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--seq", type=int, default=2048)
    a = ap.parse_args()
    kernels()
    off = grads(False, a)
    off2 = grads(False, a)
    for n in off:  # run-to-run reproducibility of the plain path
        d = ((off2[n] - off[n]).norm() / off[n].norm().clamp_min(1e-30)).item()
        if d:
            print(json.dumps({"param": n, "rerun_rel": d}), flush=True)
    on = grads(True, a)
    for n in off:
        d = ((on[n] - off[n]).norm() / off[n].norm().clamp_min(1e-30)).item()
        print(json.dumps({"param": n, "rel": round(d, 6), "norm": round(off[n].norm().item(), 6)}), flush=True)


if __name__ == "__main__":
    main()
