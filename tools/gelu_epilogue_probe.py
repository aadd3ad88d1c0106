"""GPT-2 c_fc + GELU: the library's fused bias + GELU epilogue (``torch._addmm_activation(use_gelu=True)``, hipBLASLt
GELU_BIAS) against the bias GEMM followed by the HIP GELU kernel (csrc/elementwise.hip), at the bench shape.

The training step also needs the pre-activation for the GELU backward. torch exposes no auxiliary-output epilogue, so
the fused forward would have to be paired with a recomputed pre-activation GEMM in backward -- the third row prices
that. Usage: python tools/gelu_epilogue_probe.py [--tokens 32768]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=50, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    a = ap.parse_args()
    from kubeoperator_amd.ops import load

    lib = load()
    T, K, N = a.tokens, 768, 3072
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(T, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (0.02 * torch.randn(N, K, device="cuda", generator=g)).to(torch.bfloat16)
    b = (0.02 * torch.randn(N, device="cuda", generator=g)).to(torch.bfloat16)
    ref = lib.gelu_fwd(torch.addmm(b, x, w.t()))
    fused = torch._addmm_activation(b, x, w.t(), use_gelu=True)
    err = ((fused.float() - ref.float()).norm() / ref.float().norm()).item()
    t_sep = timeit(lambda: lib.gelu_fwd(torch.addmm(b, x, w.t())))
    t_gemm = timeit(lambda: torch.addmm(b, x, w.t()))
    t_fused = timeit(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=True))
    print(json.dumps({"shape": [T, K, N], "addmm_us": round(t_gemm, 1), "addmm_plus_gelu_kernel_us": round(t_sep, 1),
                      "gelu_kernel_us": round(t_sep - t_gemm, 1), "fused_epilogue_us": round(t_fused, 1),
                      "fused_plus_recompute_us": round(t_fused + t_gemm, 1), "fused_vs_reference_rel_err": err}),
          flush=True)


if __name__ == "__main__":
    main()
