"""HTTP front end of the generator: the serving pod's entry point.

  python -m kubeoperator_amd.serve.server --model llama3_8b --max-batch 64 --max-seq 8192 --port 8000 [--ckpt DIR]

``POST /v1/generate`` ``{"tokens": [[id, ...], ...], "max_new_tokens": N}`` -> ``{"tokens": [[...]], "ms": ...}``:
the prompts of one request (equal lengths) are prefilled together and decoded greedily as one batch; requests
are served one at a time on the GPU (a lock around the generator). ``GET /v1/model`` describes the loaded model,
``GET /healthz`` answers readiness probes. Token ids in, token ids out: the chart ships no tokenizer files.
Weights are random-init unless ``--ckpt`` names a training checkpoint directory (the trainer's flat layout;
loaded with ``torch.load(weights_only=True)``).
"""
from __future__ import annotations

import argparse
import threading
import time

import torch
from pydantic import BaseModel

from ..models import build_model, get_config
from .generate import LlamaGenerator


class GenerateRequest(BaseModel):
    tokens: list[list[int]]
    max_new_tokens: int = 16


def create_app(model, max_batch: int, max_seq: int, graph: bool = False, fp8: bool = False):
    from fastapi import FastAPI, HTTPException

    gen = LlamaGenerator(model, max_batch=max_batch, max_seq=max_seq, graph=graph, fp8=fp8)
    lock = threading.Lock()
    app = FastAPI(title="KubeOperator-AMD serving", docs_url="/docs")

    @app.get("/healthz")
    def healthz():
        return {"ok": True}

    @app.get("/v1/model")
    def info():
        c = model.cfg
        return {"model": c.name, "params": c.num_params(), "max_batch": max_batch, "max_seq": max_seq,
                "kv_cache_gb": round(gen.cache.bytes() / 1e9, 3), "hip_graph": gen.graph, "fp8_weights": fp8}

    @app.post("/v1/generate")
    def generate(req: GenerateRequest):
        if not req.tokens or len({len(t) for t in req.tokens}) != 1:
            raise HTTPException(400, "tokens: a non-empty batch of equal-length prompts")
        B, S = len(req.tokens), len(req.tokens[0])
        if B > max_batch or S < 1 or S + req.max_new_tokens > max_seq or req.max_new_tokens < 1:
            raise HTTPException(400, f"batch <= {max_batch}, 1 <= prompt and prompt + max_new_tokens <= {max_seq}")
        vocab = model.cfg.vocab_size
        if any(t < 0 or t >= vocab for row in req.tokens for t in row):
            raise HTTPException(400, f"token ids must be in [0, {vocab})")
        ids = torch.tensor(req.tokens, dtype=torch.long, device=gen.device)
        with lock:
            t0 = time.perf_counter()
            out = gen.generate(ids, req.max_new_tokens)
            new = out[:, S:].tolist()
            ms = (time.perf_counter() - t0) * 1e3
        return {"tokens": new, "ms": round(ms, 3)}

    return app


def load_model(name: str, device: str, ckpt: str = ""):
    cfg = get_config(name)
    with torch.device("meta"):
        m = build_model(cfg)
    m = m.to_empty(device=device).to(torch.bfloat16)
    if ckpt:
        from ..train import checkpoint

        step = checkpoint.latest_step(ckpt)
        sd = torch.load(f"{ckpt}/step_{step}/rank_0.pt", map_location=device, weights_only=True)
        flat, lay = sd["params"], sd["layout"]
        named = dict(m.named_parameters())
        with torch.no_grad():
            for n, off, k in zip(lay["names"], lay["offsets"], lay["numels"]):
                named[n].copy_(flat[off:off + k].view_as(named[n]))
    else:
        g = torch.Generator(device=device).manual_seed(0)
        with torch.no_grad():
            for n, p in m.named_parameters():
                p.fill_(1.0) if "norm" in n else p.normal_(0.0, cfg.init_std, generator=g)
    return m


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3_8b")
    ap.add_argument("--max-batch", type=int, default=64)
    ap.add_argument("--max-seq", type=int, default=8192)
    ap.add_argument("--graph", type=int, default=0, choices=[0, 1])
    ap.add_argument("--fp8", type=int, default=0, choices=[0, 1])
    ap.add_argument("--ckpt", default="")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    a = ap.parse_args(argv)
    import uvicorn

    dev = "cuda" if torch.cuda.is_available() else "cpu"
    app = create_app(load_model(a.model, dev, a.ckpt), a.max_batch, a.max_seq, bool(a.graph), bool(a.fp8))
    uvicorn.run(app, host=a.host, port=a.port, log_level="warning")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
