"""Forward / data-gradient GEMMs of the Llama-3-8B block with the activation operand given TRANSPOSED (A^T stored
[K, M], M contiguous) against the row-major form: if hipBLASLt runs them at the same speed, the producers that
already write the transposed copy (SwiGLU y^T / dgu^T, RMSNorm y^T) could skip the row-major one.
Prints one JSON line per (GEMM, layout). Usage: python tools/bench_gemm_at.py [--tuning use|off]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

T = 8192
GEMMS = [  # name, K (reduction), N (output columns)
    ("w_down fwd: h . Wd^T", 14336, 4096),
    ("qkv fwd: y . Wqkv^T", 4096, 6144),
    ("gate_up fwd: y . Wgu^T", 4096, 28672),
    ("gate_up dX: dgu . Wgu", 28672, 4096),
    ("qkv dX: dqkv . Wqkv", 6144, 4096),
]


def timeit(fn, iters=20):
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
    ap.add_argument("--tuning", default="use")
    a = ap.parse_args()
    from kubeoperator_amd.train import gemm_tuning

    gemm_tuning.setup(a.tuning, rank=0)
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, K, N in GEMMS:
        x = torch.randn(T, K, device="cuda", generator=g).bfloat16()
        xt = x.t().contiguous()
        w = torch.randn(N, K, device="cuda", generator=g).bfloat16()  # the operand as the step passes it: B = w.t()
        fl = 2.0 * T * K * N
        ref = torch.mm(x, w.t())
        for layout, fn in (("A row-major", lambda: torch.mm(x, w.t())), ("A transposed", lambda: torch.mm(xt.t(), w.t()))):
            ms = timeit(fn)
            err = ((fn().float() - ref.float()).abs().max() / ref.float().abs().max()).item()
            print(json.dumps({"gemm": name, "layout": layout, "ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1),
                              "rel_err": round(err, 5)}), flush=True)
        del x, xt, w, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
