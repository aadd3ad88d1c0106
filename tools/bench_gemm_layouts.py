"""Time the Llama-3-8B training GEMMs per operand layout on one GPU (hipBLASLt through torch.mm).

For each projection (tokens T = 8192): forward y = x w^T, data gradient dx = dy w, and the weight gradient
dW = dy^T x in three forms -- the strided "NT" call autograd makes, the same product after materialising
dy^T and x^T (both operands then K-contiguous, "TN"), the transposes alone (PyTorch strided copy and the HIP kernel), and the HIP-transpose path end to end -- so the cheapest
weight-gradient layout can be picked from measurement.

Usage: python tools/bench_gemm_layouts.py [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tokens", type=int, default=8192)
    a = ap.parse_args()
    T = a.tokens
    dev = "cuda"
    rows = []
    for name, (n, k) in SHAPES.items():
        x = torch.randn(T, k, device=dev, dtype=torch.bfloat16)
        w = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(T, n, device=dev, dtype=torch.bfloat16)
        dw = torch.empty(n, k, device=dev, dtype=torch.bfloat16)
        dyt = dy.t().contiguous()
        xt = x.t().contiguous()
        flop = 2.0 * T * n * k
        r = {"name": name, "N": n, "K": k, "T": T}
        r["fwd_ms"] = timed(lambda: torch.mm(x, w.t()), a.iters)
        r["dx_ms"] = timed(lambda: torch.mm(dy, w), a.iters)
        r["dw_nt_ms"] = timed(lambda: torch.mm(dy.t(), x, out=dw), a.iters)
        r["dw_tn_gemm_ms"] = timed(lambda: torch.mm(dyt, xt.t(), out=dw), a.iters)
        r["transpose_ms"] = timed(lambda: (dyt.copy_(dy.t()), xt.copy_(x.t())), a.iters)
        r["dw_addmm_nt_ms"] = timed(lambda: dw.addmm_(dy.t(), x), a.iters)
        from kubeoperator_amd.ops.functional import _dw_into, transpose
        r["hip_transpose_ms"] = timed(lambda: (transpose(dy), transpose(x)), a.iters)
        r["hip_transpose_TBps"] = round(2 * (dy.numel() + x.numel()) * 2 / (r["hip_transpose_ms"] * 1e-3) / 1e12, 2)
        r["dw_tn_hip_total_ms"] = timed(lambda: _dw_into(dy, x, dw, False), a.iters)
        for key in ("fwd_ms", "dx_ms", "dw_nt_ms", "dw_tn_gemm_ms", "dw_addmm_nt_ms"):
            r[key.replace("_ms", "_tflops")] = round(flop / (r[key] * 1e-3) / 1e12, 1)
        r["dw_tn_total_ms"] = r["dw_tn_gemm_ms"] + r["transpose_ms"]
        rows.append(r)
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
        del x, w, dy, dw, dyt, xt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
