"""Attention probe: forward / backward TFLOP/s of the HIP flash-attention kernels at several shapes, causal and
not, in one process (A/B of kernel variants selected by environment variables happens across invocations in
one box session). Usage: python tools/attn_probe.py [--shapes llama,guide,gpt2]"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"llama": (1, 8192, 32, 8, 128), "llama4k": (2, 4096, 32, 8, 128), "guide": (16, 2048, 64, 8, 128),
          "gpt2": (4, 1024, 12, 12, 64), "gpt2b": (32, 1024, 12, 12, 64), "s1k": (8, 1024, 32, 8, 128), "s2k": (4, 2048, 32, 8, 128),
          "s512": (16, 512, 32, 8, 128)}


def timeit(fn, iters, warmup=3):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="llama,guide")
    ap.add_argument("--causal", default="1,0")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tag", default=os.environ.get("KOP_PROBE_TAG", ""))
    ap.add_argument("--sdpa", action="store_true", help="also time torch SDPA (the ROCm build's flash kernels) on the shape")
    a = ap.parse_args()
    from kubeoperator_amd.ops import load

    lib = load()
    for name in a.shapes.split(","):
        B, S, Hq, Hkv, D = SHAPES[name]
        g = torch.Generator(device="cuda").manual_seed(0)
        qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16, generator=g)
        x, c = Hq * D, (Hq + Hkv) * D
        q, k, v = qkv[:, :x], qkv[:, x:c], qkv[:, c:]
        o = torch.empty(B * S, Hq * D, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(B * Hq * S, device="cuda", dtype=torch.float32)
        do = torch.randn_like(o)
        dqkv = torch.empty_like(qkv)
        ws = torch.empty(lib.flash_attn_bwd_workspace(B, S, Hq, D), dtype=torch.uint8, device="cuda")
        ot = torch.empty(Hq * D, B * S, device="cuda", dtype=torch.bfloat16)  # O^T companion (the training step's form)
        sc = 1 / math.sqrt(D)
        for causal in [bool(int(x)) for x in a.causal.split(",")]:
            fl = 4 * B * Hq * S * S * D * (0.5 if causal else 1.0)
            tf = timeit(lambda: lib.flash_attn_fwd(q, k, v, o, lse, B, S, Hq, Hkv, D, sc, causal), a.iters)
            tft = timeit(lambda: lib.flash_attn_fwd_t(q, k, v, o, ot, lse, B, S, Hq, Hkv, D, sc, causal), a.iters)
            tb = timeit(lambda: lib.flash_attn_bwd(q, k, v, o, do, lse, dqkv[:, :x], dqkv[:, x:c], dqkv[:, c:], ws,
                                                   B, S, Hq, Hkv, D, sc, causal), max(3, a.iters // 2))
            print(json.dumps({"tag": a.tag, "shape": name, "causal": causal, "fwd_ms": round(tf, 4),
                              "fwd_tflops": round(fl / tf / 1e9, 1), "fwd_ot_ms": round(tft, 4), "bwd_ms": round(tb, 4),
                              "bwd_tflops": round(2.5 * fl / tb / 1e9, 1)}), flush=True)
            if a.sdpa:
                import torch.nn.functional as F

                rep = Hq // Hkv
                qh = q.reshape(B, S, Hq, D).transpose(1, 2).contiguous().requires_grad_(True)
                kh = k.reshape(B, S, Hkv, D).transpose(1, 2).repeat_interleave(rep, 1).contiguous().requires_grad_(True)
                vh = v.reshape(B, S, Hkv, D).transpose(1, 2).repeat_interleave(rep, 1).contiguous().requires_grad_(True)
                dh = do.reshape(B, S, Hq, D).transpose(1, 2).contiguous()
                ts = timeit(lambda: F.scaled_dot_product_attention(qh, kh, vh, is_causal=causal), a.iters)
                out = F.scaled_dot_product_attention(qh, kh, vh, is_causal=causal)
                tsb = timeit(lambda: torch.autograd.grad(out, (qh, kh, vh), dh, retain_graph=True), max(3, a.iters // 2))
                print(json.dumps({"tag": "torch_sdpa", "shape": name, "causal": causal, "fwd_ms": round(ts, 4),
                                  "fwd_tflops": round(fl / ts / 1e9, 1), "bwd_ms": round(tsb, 4),
                                  "bwd_tflops": round(2.5 * fl / tsb / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
