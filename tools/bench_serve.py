"""Continuous-batching serving benchmark on one MI355X: N concurrent requests (random prompt lengths, fixed
number of new tokens each) through ``serve.server.ContinuousBatcher`` on Llama-3-8B (random init, bf16).
Reports generated tokens/s over the whole run (prefills included) and the decode-step count.

  python tools/bench_serve.py --requests 256 --slots 64 --prompt 256,2048 --new 128
"""
import argparse
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3_8b")
    ap.add_argument("--requests", type=int, default=256)
    ap.add_argument("--slots", type=int, default=64)
    ap.add_argument("--prompt", default="256,2048", help="min,max prompt tokens (uniform)")
    ap.add_argument("--new", type=int, default=128)
    ap.add_argument("--fp8", type=int, default=0)
    a = ap.parse_args()
    from kubeoperator_amd.ops import load
    from kubeoperator_amd.serve import LlamaGenerator
    from kubeoperator_amd.serve.server import ContinuousBatcher, load_model
    from kubeoperator_amd.train import gemm_tuning

    load()
    tuning = gemm_tuning.setup("use", path=gemm_tuning.results_path("gfx950_decode"))
    m = load_model(a.model, "cuda")
    lo, hi = (int(x) for x in a.prompt.split(","))
    g = torch.Generator().manual_seed(0)
    lens = torch.randint(lo, hi + 1, (a.requests,), generator=g).tolist()
    prompts = [torch.randint(0, m.cfg.vocab_size, (n,), generator=g).tolist() for n in lens]
    b = ContinuousBatcher(LlamaGenerator(m, max_batch=a.slots, max_seq=hi + a.new + 128, fp8=bool(a.fp8)))
    b.generate([prompts[0][:128]], 2)  # warm-up (library handles)
    steps0 = b.steps
    out = [None] * a.requests
    t0 = time.perf_counter()

    def run(i):
        out[i] = b.generate([prompts[i]], a.new)[0]

    th = [threading.Thread(target=run, args=(i,)) for i in range(a.requests)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    b.close()
    gen_tok = sum(len(o) for o in out)
    print(json.dumps({"bench": "serve", "model": a.model, "requests": a.requests, "slots": a.slots,
                      "prompt_tokens": sum(lens), "new_tokens_per_request": a.new, "seconds": round(dt, 2),
                      "generated_tokens_per_s": round(gen_tok / dt, 1),
                      "total_tokens_per_s": round((gen_tok + sum(lens)) / dt, 1),
                      "decode_steps": b.steps - steps0, "fp8_weights": bool(a.fp8), "gemm_selection": tuning}),
          flush=True)


if __name__ == "__main__":
    main()
