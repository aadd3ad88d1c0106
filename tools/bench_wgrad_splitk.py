"""Weight-gradient GEMM dW = dY^T X (reduction over the T token rows) at the training shapes: the current
forms (NT: strided operands; TN: both operands transposed to K-contiguous first) against split-K over the
token dimension (batched GEMM over T/s-row chunks into fp32 partials, then summed into the bf16 gradient).

Narrow outputs (GPT-2-small: 768 x 768 ... 3072 x 768 at T = 32768) give hipBLASLt only a few dozen output
tiles for 256 CUs; the chunks multiply the tiles. Prints one JSON line per (shape, variant).
Usage: python tools/bench_wgrad_splitk.py [--shapes gpt2,llama]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {
    "gpt2": [(32768, 2304, 768, "qkv"), (32768, 768, 768, "proj"), (32768, 3072, 768, "fc"), (32768, 768, 3072, "out"),
             (32768, 50304, 768, "lm_head")],
    "llama": [(8192, 6144, 4096, "wqkv"), (8192, 4096, 4096, "wo"), (8192, 28672, 4096, "w_gate_up"),
              (8192, 4096, 14336, "w_down"), (8192, 128256, 4096, "lm_head")],
}


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
    ap.add_argument("--shapes", default="gpt2,llama")
    ap.add_argument("--splits", default="2,4,8,16")
    a = ap.parse_args()
    from kubeoperator_amd.ops.functional import transpose
    from kubeoperator_amd.train import gemm_tuning

    gemm_tuning.setup("use", rank=0)
    for group in a.shapes.split(","):
        for T, N, K, name in SHAPES[group]:
            g = torch.Generator(device="cuda").manual_seed(0)
            dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16, generator=g)
            x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16, generator=g)
            out = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
            ref = (dy.float().t() @ x.float())
            fl = 2.0 * T * N * K

            def report(variant, ms, res):
                err = ((res.float() - ref).abs().max() / ref.abs().max()).item()
                print(json.dumps({"shape": name, "T": T, "N": N, "K": K, "variant": variant, "ms": round(ms, 4),
                                  "tflops": round(fl / ms / 1e9, 1), "rel_err": round(err, 5)}), flush=True)

            report("nt", timeit(lambda: torch.mm(dy.t(), x, out=out)), out)
            report("nt_acc", timeit(lambda: out.addmm_(dy.t(), x)), torch.mm(dy.t(), x))
            report("tn(+2 transposes)", timeit(lambda: torch.mm(transpose(dy), transpose(x).t(), out=out)), out)
            for s in [int(v) for v in a.splits.split(",")]:
                if T % s:
                    continue
                c = T // s

                def split(s=s, c=c):
                    part = torch.bmm(dy.view(s, c, N).transpose(1, 2), x.view(s, c, K), out_dtype=torch.float32)
                    out.copy_(part.sum(0))  # fp32 sum, rounded once into the bf16 gradient

                report(f"splitk{s}", timeit(split), out)

                def split_only(s=s, c=c):
                    return torch.bmm(dy.view(s, c, N).transpose(1, 2), x.view(s, c, K), out_dtype=torch.float32)

                report(f"splitk{s}_bmm_only", timeit(split_only), split_only().sum(0))
            del dy, x, out, ref
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
