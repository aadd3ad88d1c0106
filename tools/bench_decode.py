"""Serving benchmark on one MI355X: Llama-3-8B (random init, bf16) KV-cache generation -- prefill of a batch of
prompts, then timed greedy decode steps (one token per sequence per step through all 32 layers, the split-K
decode-attention kernel over the cache and the LM head). Prints one JSON line per configuration.

  python tools/bench_decode.py --batch 64 --prompt 2048 --steps 32
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3_8b")
    ap.add_argument("--batch", default="1,16,64")
    ap.add_argument("--prompt", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--graph", default="0,1", help="decode steps eager (0) and/or as replayed HIP graphs (1)")
    ap.add_argument("--gemm-tuning", default="use", choices=["off", "use", "tune"],
                    help="TunableOp winners for the decode GEMM shapes (small M = batch): read, or re-tune into --gemm-results")
    ap.add_argument("--gemm-results", default="")
    ap.add_argument("--fp8", default="0", help="0 and/or 1: E4M3 block-projection weights (opt-in serving mode)")
    a = ap.parse_args()
    from kubeoperator_amd.models import build_model, get_config
    from kubeoperator_amd.ops import load
    from kubeoperator_amd.serve import LlamaGenerator
    from kubeoperator_amd.train import gemm_tuning

    load()
    tuning = gemm_tuning.setup(a.gemm_tuning, path=a.gemm_results or gemm_tuning.results_path("gfx950_decode"))
    cfg = get_config(a.model)
    with torch.device("meta"):
        m = build_model(cfg)
    m = m.to_empty(device="cuda").to(torch.bfloat16)
    g = torch.Generator(device="cuda").manual_seed(0)
    with torch.no_grad():
        for n, p in m.named_parameters():
            p.fill_(1.0) if "norm" in n else p.normal_(0.0, 0.02, generator=g)
    wbytes = sum(p.numel() * p.element_size() for p in m.parameters())
    runs = [(int(x), int(gr), int(f)) for f in a.fp8.split(",") for x in a.batch.split(",") for gr in a.graph.split(",")]
    for B, graph, f8 in runs:
        gen = LlamaGenerator(m, max_batch=B, max_seq=a.prompt + a.steps + 3, graph=bool(graph), fp8=bool(f8))
        ids = torch.randint(0, cfg.vocab_size, (B, a.prompt), device="cuda")
        gen.prefill(ids)  # untimed: first-call library / workspace setup (the timed prefill rewrites the same rows)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        logits = gen.prefill(ids)
        torch.cuda.synchronize()
        t_pre = time.perf_counter() - t0
        nxt = logits.argmax(-1)
        for _ in range(2):  # warm-up decode steps
            nxt = gen.decode(nxt).argmax(-1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            nxt = gen.decode(nxt).argmax(-1)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        ctx = a.prompt + 2 + a.steps / 2  # mean cached length over the timed steps
        kv_bytes = B * ctx * cfg.n_layers * 2 * cfg.n_kv_heads * cfg.head_dim * 2
        print(json.dumps({"bench": "decode", "model": a.model, "batch": B, "prompt": a.prompt, "hip_graph": bool(graph), "weights": "e4m3 projections" if f8 else "bf16",
                          "prefill_tokens_per_s": round(B * a.prompt / t_pre, 1), "decode_ms_per_step": round(dt * 1e3, 3),
                          "decode_tokens_per_s": round(B / dt, 1),
                          "hbm_gb_per_step": round((wbytes + kv_bytes) / 1e9, 2),
                          "effective_tb_per_s": round((wbytes + kv_bytes) / dt / 1e12, 2),
                          "kv_cache_gb": round(gen.cache.bytes() / 1e9, 2), "gemm_selection": tuning}), flush=True)
        gen.drop_fp8()
        del gen
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
