"""Micro-benchmarks of the gfx950 kernels at Llama-3-8B training shapes (one GPU).

Prints one JSON line per kernel: time, achieved TFLOP/s or TB/s. Compares flash attention with
PyTorch SDPA on the same random data (reference point only; the framework never calls SDPA on GPU).
Usage: python tools/bench_kernels.py [--seq 8192] [--only attn]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


ITERS = [None]


def timeit(fn, iters=20, warmup=3):
    if ITERS[0] is not None:
        iters, warmup = ITERS[0], 1
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def emit(**kw):
    print(json.dumps(kw), flush=True)


def bench_attn(B, S, Hq, Hkv, D, causal=True, sdpa=True):
    from kubeoperator_amd.ops import load

    lib = load()
    dev = "cuda"
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
    a, c = Hq * D, (Hq + Hkv) * D
    q, k, v = qkv[:, :a], qkv[:, a:c], qkv[:, c:]
    o = torch.empty(B * S, Hq * D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * Hq * S, device=dev, dtype=torch.float32)
    scale = 1 / math.sqrt(D)
    flops_fwd = 4 * B * Hq * S * S * D * (0.5 if causal else 1.0)
    t = timeit(lambda: lib.flash_attn_fwd(q, k, v, o, lse, B, S, Hq, Hkv, D, scale, causal))
    emit(kernel="flash_attn_fwd", B=B, S=S, Hq=Hq, Hkv=Hkv, D=D, ms=round(t, 4), tflops=round(flops_fwd / t / 1e9, 1))
    do = torch.randn_like(o)
    dqkv = torch.empty_like(qkv)
    ws = torch.empty(lib.flash_attn_bwd_workspace(B, S, Hq, D), dtype=torch.uint8, device=dev)
    t = timeit(lambda: lib.flash_attn_bwd(q, k, v, o, do, lse, dqkv[:, :a], dqkv[:, a:c], dqkv[:, c:], ws, B, S, Hq,
                                          Hkv, D, scale, causal), iters=10)
    emit(kernel="flash_attn_bwd", B=B, S=S, Hq=Hq, Hkv=Hkv, D=D, ms=round(t, 4),
         tflops=round(2.5 * flops_fwd / t / 1e9, 1))
    # reference point: torch SDPA (aotriton / CK inside PyTorch-ROCm)
    if not sdpa:
        return
    try:
        qh = q.reshape(B, S, Hq, D).transpose(1, 2).contiguous()
        kh = k.reshape(B, S, Hkv, D).transpose(1, 2).repeat_interleave(Hq // Hkv, 1).contiguous()
        vh = v.reshape(B, S, Hkv, D).transpose(1, 2).repeat_interleave(Hq // Hkv, 1).contiguous()
        f = lambda: torch.nn.functional.scaled_dot_product_attention(qh, kh, vh, is_causal=causal)
        t = timeit(f)
        emit(kernel="torch_sdpa_fwd(reference)", S=S, ms=round(t, 4), tflops=round(flops_fwd / t / 1e9, 1))
        qh.requires_grad_(True)
        kh.requires_grad_(True)
        vh.requires_grad_(True)
        out = torch.nn.functional.scaled_dot_product_attention(qh, kh, vh, is_causal=causal)
        g = torch.randn_like(out)
        t = timeit(lambda: torch.autograd.grad(out, (qh, kh, vh), g, retain_graph=True), iters=10)
        emit(kernel="torch_sdpa_bwd(reference)", S=S, ms=round(t, 4), tflops=round(2.5 * flops_fwd / t / 1e9, 1))
    except Exception as ex:  # pragma: no cover
        emit(kernel="torch_sdpa", error=str(ex)[:200])


def bench_gemm(T=8192):
    dev = "cuda"
    shapes = {"qkv": (T, 4096, 6144), "o": (T, 4096, 4096), "gate_up": (T, 4096, 28672), "down": (T, 14336, 4096),
              "lm_head": (T, 4096, 128256)}
    for name, (M, K, N) in shapes.items():
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: torch.mm(a, w.t()), iters=10)
        emit(kernel=f"gemm_{name}_fwd", M=M, K=K, N=N, ms=round(t, 4), tflops=round(2 * M * N * K / t / 1e9, 1))
        dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: torch.mm(dy.t(), a), iters=10)
        emit(kernel=f"gemm_{name}_wgrad", ms=round(t, 4), tflops=round(2 * M * N * K / t / 1e9, 1))
        t = timeit(lambda: torch.mm(dy, w), iters=10)
        emit(kernel=f"gemm_{name}_dgrad", ms=round(t, 4), tflops=round(2 * M * N * K / t / 1e9, 1))
        del a, w, dy


def bench_mem(T=8192):
    from kubeoperator_amd.ops import load
    from kubeoperator_amd.ops.reference import rope_cache

    lib = load()
    dev = "cuda"
    H = 4096
    x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
    r = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
    w = torch.ones(H, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: lib.norm_fwd(x, r, w, None, 1e-5, False))
    emit(kernel="rmsnorm_fwd_residual", ms=round(t, 4), tbps=round(4 * T * H * 2 / t / 1e9, 2))
    y, s, rstd, _ = lib.norm_fwd(x, r, w, None, 1e-5, False)
    dw = torch.empty_like(w)
    t = timeit(lambda: lib.norm_bwd(x, s, w, rstd, None, r, dw, None, False, False))
    emit(kernel="rmsnorm_bwd_residual", ms=round(t, 4), tbps=round(4 * T * H * 2 / t / 1e9, 2))
    qkv = torch.randn(T, 6144, device=dev, dtype=torch.bfloat16)
    cos, sin = rope_cache(8192, 128, 500000.0, device=dev)
    t = timeit(lambda: lib.rope_(qkv, cos, sin, None, 8192, 40, 128, False))
    emit(kernel="rope", ms=round(t, 4), tbps=round(2 * T * 5120 * 2 / t / 1e9, 2))
    gu = torch.randn(T, 2 * 14336, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: lib.swiglu_fwd(gu))
    emit(kernel="swiglu_fwd", ms=round(t, 4), tbps=round(3 * T * 14336 * 2 / t / 1e9, 2))
    dh = torch.randn(T, 14336, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: lib.swiglu_bwd(gu, dh))
    emit(kernel="swiglu_bwd", ms=round(t, 4), tbps=round(5 * T * 14336 * 2 / t / 1e9, 2))
    logits = torch.randn(T, 128256, device=dev, dtype=torch.bfloat16)
    tgt = torch.randint(0, 128256, (T,), device=dev)
    t = timeit(lambda: lib.cross_entropy_fwd_(logits, tgt, -100, True, 1.0), iters=5)
    emit(kernel="cross_entropy_fwd_grad", ms=round(t, 4), tbps=round(3 * T * 128256 * 2 / t / 1e9, 2))
    del logits
    n = 512 * 1024 * 1024
    p = torch.zeros(n, device=dev, dtype=torch.bfloat16)
    g = torch.zeros(n, device=dev, dtype=torch.bfloat16)
    mw = torch.zeros(n, device=dev)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    t = timeit(lambda: lib.adamw_(p, g, mw, m, v, 1e-4, 0.9, 0.95, 1e-8, 0.1, 1, 1.0, None), iters=5)
    emit(kernel="adamw", n=n, ms=round(t, 4), tbps=round(28 * n / t / 1e9, 2))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--only", default="all")
    ap.add_argument("--iters", type=int, default=None)
    ap.add_argument("--no-sdpa", action="store_true")
    a = ap.parse_args()
    ITERS[0] = a.iters
    emit(device=torch.cuda.get_device_name(0), arch=torch.cuda.get_device_properties(0).gcnArchName)
    if a.only in ("all", "attn"):
        bench_attn(1, a.seq, 32, 8, 128, sdpa=not a.no_sdpa)
        bench_attn(4, 1024, 12, 12, 64, sdpa=not a.no_sdpa)
    if a.only in ("all", "mem"):
        bench_mem()
    if a.only in ("all", "gemm"):
        bench_gemm()
