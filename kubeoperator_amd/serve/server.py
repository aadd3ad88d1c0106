"""HTTP front end of the generator: the serving pod's entry point.

  python -m kubeoperator_amd.serve.server --model llama3_8b --max-batch 64 --max-seq 8192 --port 8000 [--ckpt DIR]

``POST /v1/generate`` ``{"tokens": [[id, ...], ...], "max_new_tokens": N}`` -> ``{"tokens": [[...]], "ms": ...}``:
greedy continuation of every prompt. Continuous batching (``ContinuousBatcher``): every prompt of every
concurrent request takes a free sequence slot of the KV cache as soon as one is free (its own prefill), and one
decode step advances all active slots together -- prompts of any length, joining and leaving between steps, so
the decode GEMMs and the decode-attention kernel see the whole live batch (ragged cache lengths). ``GET /v1/model`` describes the loaded model,
``GET /healthz`` answers readiness probes. Token ids in, token ids out: the chart ships no tokenizer files.
Weights are random-init unless ``--ckpt`` names a training checkpoint directory (the trainer's flat layout;
loaded with ``torch.load(weights_only=True)``).
"""
from __future__ import annotations

import argparse
import queue
import threading
import time

import torch
from pydantic import BaseModel

from ..models import build_model, get_config
from .generate import LlamaGenerator


class GenerateRequest(BaseModel):
    tokens: list[list[int]]
    max_new_tokens: int = 16


class _Seq:
    def __init__(self, prompt: list[int], max_new: int):
        self.prompt, self.max_new = prompt, max_new
        self.out: list[int] = []
        self.done = threading.Event()
        self.error: Exception | None = None


class ContinuousBatcher:
    """One scheduler thread owns the generator: admits queued sequences into free cache slots (prefill), then
    runs one decode step over every active slot; a sequence leaves its slot once it has its tokens."""

    def __init__(self, gen: LlamaGenerator):
        self.gen = gen
        self.q: queue.Queue = queue.Queue()
        self.slots: list[_Seq | None] = [None] * gen.cache.batch
        self.next_tok = [0] * gen.cache.batch
        self.steps = 0
        self._stop = False
        self._thread = threading.Thread(target=self._loop, name="kop-serve-batcher", daemon=True)
        self._thread.start()

    def generate(self, prompts: list[list[int]], max_new: int) -> list[list[int]]:
        seqs = [_Seq(p, max_new) for p in prompts]
        for sq in seqs:
            self.q.put(sq)
        for sq in seqs:
            sq.done.wait()
            if sq.error is not None:
                raise sq.error
        return [sq.out for sq in seqs]

    def close(self) -> None:
        self._stop = True
        self.q.put(None)
        self._thread.join(10)

    def _finish(self, slot: int) -> None:
        sq = self.slots[slot]
        self.slots[slot] = None
        self.gen.cache.release(slot)
        sq.done.set()

    def _admit(self, seqs: list) -> None:
        """Prefill newly admitted sequences into free slots, one batched prefill per padded length (prompts
        right-padded to 128-token multiples, so sequences of similar lengths share the prefill GEMMs)."""
        groups: dict[int, list] = {}
        for sq in seqs:
            slot = self.slots.index(None)
            self.slots[slot] = sq
            n = len(sq.prompt)
            padded = -(-n // 128) * 128
            groups.setdefault(padded if padded <= self.gen.cache.max_seq else n, []).append((slot, sq))
        for S, members in groups.items():
            try:
                ids = torch.zeros(len(members), S, dtype=torch.long)
                for r, (_, sq) in enumerate(members):
                    ids[r, :len(sq.prompt)] = torch.tensor(sq.prompt, dtype=torch.long)
                logits = self.gen.prefill(ids.to(self.gen.device), slots=[sl for sl, _ in members],
                                          lengths=[len(sq.prompt) for _, sq in members])
                nxt = logits.argmax(-1).tolist()
            except Exception as e:  # a bad request fails alone
                for slot, sq in members:
                    sq.error = e
                    self._finish(slot)
                continue
            for (slot, sq), t in zip(members, nxt):
                sq.out.append(t)
                self.next_tok[slot] = t
                if len(sq.out) >= sq.max_new:
                    self._finish(slot)

    def _loop(self) -> None:
        while not self._stop:
            # admit queued sequences into the free slots; block on the queue only when nothing is running
            new = []
            free = self.slots.count(None)
            while len(new) < free:
                running = any(s is not None for s in self.slots) or new
                try:
                    item = self.q.get_nowait() if running else self.q.get(timeout=0.5)
                except queue.Empty:
                    break
                if item is None:  # close()
                    break
                new.append(item)
            if new:
                self._admit(new)
            active = [s is not None for s in self.slots]
            if not any(active):
                continue
            n = max(i for i, a in enumerate(active) if a) + 1  # rows [0, n) cover every active slot
            try:
                tok = torch.tensor(self.next_tok[:n], dtype=torch.long, device=self.gen.device)
                nxt = self.gen.decode(tok, active=active[:n]).argmax(-1).tolist()
            except Exception as e:  # fail the running sequences, keep serving
                for i in range(n):
                    if self.slots[i] is not None:
                        self.slots[i].error = e
                        self._finish(i)
                continue
            self.steps += 1
            for i in range(n):
                sq = self.slots[i]
                if sq is None:
                    continue
                sq.out.append(nxt[i])
                self.next_tok[i] = nxt[i]
                if len(sq.out) >= sq.max_new:
                    self._finish(i)


def create_app(model, max_batch: int, max_seq: int, graph: bool = False, fp8: bool = False):
    from fastapi import FastAPI, HTTPException

    gen = LlamaGenerator(model, max_batch=max_batch, max_seq=max_seq, graph=graph, fp8=fp8)
    batcher = ContinuousBatcher(gen)
    app = FastAPI(title="KubeOperator-AMD serving", docs_url="/docs")
    app.state.batcher = batcher

    @app.get("/healthz")
    def healthz():
        return {"ok": True}

    @app.get("/v1/model")
    def info():
        c = model.cfg
        return {"model": c.name, "params": c.num_params(), "max_batch": max_batch, "max_seq": max_seq,
                "active": sum(x is not None for x in batcher.slots), "decode_steps": batcher.steps,
                "kv_cache_gb": round(gen.cache.bytes() / 1e9, 3), "hip_graph": gen.graph, "fp8_weights": fp8}

    @app.post("/v1/generate")
    def generate(req: GenerateRequest):
        if not req.tokens:
            raise HTTPException(400, "tokens: a non-empty list of prompts")
        S = max(len(t) for t in req.tokens)
        if min(len(t) for t in req.tokens) < 1 or S + req.max_new_tokens > max_seq or req.max_new_tokens < 1:
            raise HTTPException(400, f"1 <= prompt length and prompt + max_new_tokens <= {max_seq}")
        vocab = model.cfg.vocab_size
        if any(t < 0 or t >= vocab for row in req.tokens for t in row):
            raise HTTPException(400, f"token ids must be in [0, {vocab})")
        t0 = time.perf_counter()
        new = batcher.generate(req.tokens, req.max_new_tokens)
        return {"tokens": new, "ms": round((time.perf_counter() - t0) * 1e3, 3)}

    return app


def load_model(name: str, device: str, ckpt: str = ""):
    cfg = get_config(name)
    with torch.device("meta"):
        m = build_model(cfg)
    m = m.to_empty(device=device).to(torch.bfloat16)
    if ckpt:
        from ..train import checkpoint

        import os

        step = checkpoint.latest_step(ckpt)
        if step is None:
            tp_trees = [d for d in os.listdir(ckpt) if d.startswith("tp")] if os.path.isdir(ckpt) else []
            if tp_trees:
                raise ValueError(f"{ckpt} holds tensor-parallel checkpoint trees ({', '.join(sorted(tp_trees))}): "
                                 "the server loads single-GPU (tp 1) checkpoints")
            raise ValueError(f"{ckpt} holds no complete checkpoint (no 'latest' marker)")
        sd = torch.load(f"{ckpt}/step_{step}/rank_0.pt", map_location=device, weights_only=True)
        if int(sd.get("tp", 1)) != 1:
            raise ValueError(f"checkpoint {ckpt} step {step} is a tensor-parallel shard (tp {sd['tp']})")
        mc = sd.get("model_config") or {}
        want = cfg.to_dict()
        diff = {k: (mc[k], want[k]) for k in ("arch", "vocab_size", "hidden", "n_layers", "n_heads", "n_kv_heads",
                                              "ffn_hidden", "tie_embeddings") if k in mc and mc[k] != want[k]}
        if diff:
            raise ValueError(f"checkpoint model_config differs from --model {name}: {diff}")
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


def build_parser() -> argparse.ArgumentParser:
    """The server's arguments (also what the serving chart's rendered args are checked against)."""
    ap = argparse.ArgumentParser(prog="kubeoperator_amd.serve.server")
    ap.add_argument("--model", default="llama3_8b")
    ap.add_argument("--max-batch", type=int, default=64)
    ap.add_argument("--max-seq", type=int, default=8192)
    ap.add_argument("--graph", type=int, default=0, choices=[0, 1])
    ap.add_argument("--fp8", type=int, default=0, choices=[0, 1])
    ap.add_argument("--ckpt", default="")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    return ap


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    import uvicorn

    dev = "cuda" if torch.cuda.is_available() else "cpu"
    app = create_app(load_model(a.model, dev, a.ckpt), a.max_batch, a.max_seq, bool(a.graph), bool(a.fp8))
    uvicorn.run(app, host=a.host, port=a.port, log_level="warning")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
