"""Weight-gradient GEMMs of the Llama-3-8B step: overwrite (micro-batch 1, ``mm out=``) vs accumulate
(micro-batches 2..N, ``addmm_`` beta=1) with the committed TunableOp winners -- does accumulation pick a
slower hipBLASLt solution? Usage: python tools/bench_accum_gemm.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kubeoperator_amd.train import gemm_tuning  # noqa: E402

# (out rows, out cols) of dW = dY^T X with T = 8192 tokens, as the step issues it: TN after the transposes
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def timed(fn, iters=20):
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
    print(gemm_tuning.setup("use"), file=sys.stderr)
    T = 8192
    for name, (o, i) in SHAPES.items():
        dyt = torch.randn(o, T, device="cuda", dtype=torch.bfloat16)   # dY^T, K-contiguous
        xt = torch.randn(i, T, device="cuda", dtype=torch.bfloat16)    # X^T, K-contiguous
        c = torch.zeros(o, i, device="cuda", dtype=torch.bfloat16)
        c32 = torch.zeros(o, i, device="cuda", dtype=torch.float32)
        fl = 2 * o * i * T
        t0 = timed(lambda: torch.mm(dyt, xt.t(), out=c))
        t1 = timed(lambda: c.addmm_(dyt, xt.t()))
        rec = {"shape": name, "mm_ms": round(t0, 4), "addmm_ms": round(t1, 4), "mm_tflops": round(fl / t0 / 1e9),
               "addmm_tflops": round(fl / t1 / 1e9)}
        try:
            t2 = timed(lambda: torch.ops.aten.addmm.dtype_out(c32, dyt, xt.t(), torch.float32, beta=1, alpha=1, out=c32))
            rec.update(addmm_fp32out_ms=round(t2, 4), addmm_fp32out_tflops=round(fl / t2 / 1e9))
        except RuntimeError as e:
            rec.update(addmm_fp32out=str(e)[:80])
        print(json.dumps(rec), flush=True)
        del dyt, xt, c, c32


if __name__ == "__main__":
    main()
