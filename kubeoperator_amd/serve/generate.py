"""KV-cache generation for the Llama family on the gfx950 kernels (serving / evaluation of a trained chart).

Prefill runs the prompt through the training forward's kernels (fused residual + RMSNorm, one QKV GEMM, RoPE
in place, the flash-attention forward, SwiGLU MLP) and writes each layer's rotated K and V into a
preallocated cache; every decode step then pushes one token per sequence through the same projections with
RoPE at the sequence's position and the split-K decode-attention kernel (``csrc/decode_attn.hip``) over the
cache. MI355X-first sizing: the cache is one contiguous [B, Hkv, Smax, D] bf16 tensor per layer for K and for
V (each (sequence, KV head) a contiguous slab the decode kernel streams) (Llama-3-8B: 128 KiB per token across its 32 layers, so 288 GB of HBM minus 16 GB of weights holds ~2M
cached tokens, e.g. 256 sequences x 8k context), allocated once, never reshaped or copied between steps.

Weights are the model's own parameters (views into a trainer's flat store, or any loaded Llama module); the
generator adds no autograd state (``torch.no_grad``). On CPU every op falls back to its PyTorch reference.
"""
from __future__ import annotations

import math
import os

import torch

from ..models.llama import Llama
from ..ops import functional as kf
from ..ops import reference as ref


class KVCache:
    def __init__(self, n_layers: int, batch: int, max_seq: int, n_kv_heads: int, head_dim: int, device,
                 dtype=torch.bfloat16):
        shape = (batch, n_kv_heads, max_seq, head_dim)
        self.k = [torch.zeros(shape, dtype=dtype, device=device) for _ in range(n_layers)]
        self.v = [torch.zeros(shape, dtype=dtype, device=device) for _ in range(n_layers)]
        self.lens = torch.zeros(batch, dtype=torch.int32, device=device)
        self.host_lens = [0] * batch  # host mirror of lens: sizes the decode kernel's split grid without a sync
        self.batch, self.max_seq = batch, max_seq

    @property
    def max_len(self) -> int:
        return max(self.host_lens)

    def release(self, slot: int) -> None:
        """Free a sequence slot (continuous batching): its next prefill overwrites the stale rows."""
        self.host_lens[slot] = 0
        self.lens[slot] = 0

    def bytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.k + self.v)


class LlamaGenerator:
    """``graph``: replay each decode step as one captured HIP graph (``torch.cuda.CUDAGraph`` is a hipGraph on
    ROCm) -- a decode step is ~400 small launches whose host-side cost dominates at small batch. The graph's
    decode-attention grid then covers the whole cache (splits past a sequence's length exit at once)."""

    def __init__(self, model: Llama, max_batch: int, max_seq: int, graph: bool = False, fp8: bool = False):
        """``fp8``: E4M3 copies of the four block projections (per-tensor scale) are attached to the model's
        weights (``w.w8``, read by ``ops.functional`` linear / swiglu_mlp): decode steps then read half the weight
        bytes. Serving-only models: a trainer would pick the copies up too (``drop_fp8`` removes them)."""
        if not isinstance(model, Llama) or model.tp.enabled:
            raise ValueError("the generator serves single-GPU Llama models")
        self.model = model
        if fp8:
            from ..ops import fp8 as f8

            with torch.no_grad():
                for blk in model.layers:
                    for w in (blk.wqkv, blk.wo, blk.w_gate_up, blk.w_down):
                        w.w8, w.w8_scale = f8.quantize(w.detach())
        c = model.cfg
        self.cfg = c
        self.device = model.tok_emb.device
        self.cache = KVCache(c.n_layers, max_batch, max_seq, c.n_kv_heads, c.head_dim, self.device)
        self.cos, self.sin = ref.rope_cache(max_seq, c.head_dim, c.rope_theta, device=self.device)
        self.scale = 1.0 / math.sqrt(c.head_dim)
        self.graph = graph and self.device.type == "cuda"
        self._graphs: dict = {}  # batch -> (graph, static token input, static logits output)
        # decode projections of <= GEMV_ROWS token rows through the HIP GEMV (csrc/gemv.hip); KOP_DECODE_GEMV=0: GEMMs
        self._gemv = self.device.type == "cuda" and os.environ.get("KOP_DECODE_GEMV", "1") != "0"

    def drop_fp8(self) -> None:
        for blk in self.model.layers:
            for w in (blk.wqkv, blk.wo, blk.w_gate_up, blk.w_down):
                for a in ("w8", "w8_scale"):
                    if hasattr(w, a):
                        delattr(w, a)

    def _head(self):
        return self.model.tok_emb if self.cfg.tie_embeddings else self.model.lm_head

    # rows routed to the GEMV: Llama-3-8B decode at batch 1 runs 4.35 vs 4.77 ms per step (+9.6 %), but at
    # batch 4 / 8 the library GEMM is 15-20 % faster (profiles/r3_decode_gemv_ab.jsonl); the kernel takes up to 8
    GEMV_ROWS = 1

    def _gemv_ok(self, x, w) -> bool:
        return (self._gemv and x.shape[0] <= self.GEMV_ROWS and x.shape[-1] % 1024 == 0
                and w.dtype == torch.bfloat16 and not hasattr(w, "w8"))

    def _lin(self, x, w):
        """x . w^T: a decode step reads every weight once, so for a few token rows the HIP GEMV (weight rows
        streamed at HBM rate) replaces the library GEMM's small-M tiles; FP8 weights and larger batches keep
        ``kf.linear``."""
        if self._gemv_ok(x, w):
            from ..ops import load

            return load().gemv(x, w)
        return kf.linear(x, w)

    def _mlp(self, blk, y2):
        if self._gemv_ok(y2, blk.w_gate_up) and self._gemv_ok(y2, blk.w_down):
            return self._lin(kf.swiglu(self._lin(y2, blk.w_gate_up)), blk.w_down)
        return kf.swiglu_mlp(y2, blk.w_gate_up, blk.w_down)

    @torch.no_grad()
    def prefill(self, ids: torch.Tensor, slot: int = 0, lengths: list | None = None,
                slots: list | None = None) -> torch.Tensor:
        """Prompts ``ids`` [B, S] into cache rows [slot, slot + B) (or the listed ``slots``) -> logits of each
        prompt's last position [B, vocab] (fp32). ``lengths``: real lengths of right-padded rows (default S):
        causal attention keeps every real position independent of the padding after it."""
        c, m = self.cfg, self.model
        B, S = ids.shape
        slots = list(range(slot, slot + B)) if slots is None else list(slots)
        lengths = [S] * B if lengths is None else list(lengths)
        if len(slots) != B or len(lengths) != B or max(slots) >= self.cache.batch or S > self.cache.max_seq:
            raise ValueError("prompt batch / length exceeds the cache")
        contiguous = slots == list(range(slots[0], slots[0] + B))
        rows = slice(slots[0], slots[0] + B) if contiguous else torch.tensor(slots, device=self.device)
        if ids.is_cuda and S % 128 and S + 128 - S % 128 <= self.cache.max_seq:
            # right-pad to the HIP flash forward's 128-row tiles: causal attention keeps the real positions
            # independent of the padding, whose cache rows lie past lens and are overwritten by decode steps
            ids = torch.cat([ids, ids.new_zeros(B, 128 - S % 128)], dim=1)
            S = ids.shape[1]
        Hq, Hkv, D = c.n_heads, c.n_kv_heads, c.head_dim
        a, kc = Hq * D, (Hq + Hkv) * D
        x = kf.embedding(ids.reshape(-1), m.tok_emb)
        pending = None
        for i, blk in enumerate(m.layers):
            if pending is None:
                y, x1 = kf.rms_norm(x, blk.attn_norm, c.norm_eps), x
            else:
                y, x1 = kf.rms_norm(x, blk.attn_norm, c.norm_eps, residual=pending)
            qkv = kf.linear(y, blk.wqkv)
            if qkv.is_cuda:
                from ..ops import load

                load().rope_(qkv, self.cos, self.sin, None, S, Hq + Hkv, D, False)
            else:
                qkv = ref.rope_ref(qkv, self.cos, self.sin, S, Hq + Hkv, D)
            q, k, v = qkv[:, :a], qkv[:, a:kc], qkv[:, kc:]
            kh, vh = k.reshape(B, S, Hkv, D).transpose(1, 2), v.reshape(B, S, Hkv, D).transpose(1, 2)
            if contiguous:  # a slice of the cache: copy in place
                self.cache.k[i][rows, :, :S].copy_(kh)
                self.cache.v[i][rows, :, :S].copy_(vh)
            else:  # index tensor: advanced indexing returns a COPY, so write through index_put_ (assignment)
                self.cache.k[i][rows, :, :S] = kh
                self.cache.v[i][rows, :, :S] = vh
            if q.is_cuda and S % 128 == 0:  # the HIP flash forward's tile constraint
                o, _ = kf.flash_attention(q, k, v, B, S, Hq, Hkv, D, causal=True, scale=self.scale)
            else:
                o, _ = ref.attention_ref(q, k, v, B, S, Hq, Hkv, D, True, self.scale)
            y2, x = kf.rms_norm(x1, blk.mlp_norm, c.norm_eps, residual=self._lin(o, blk.wo))
            pending = self._mlp(blk, y2)
        y, _ = kf.rms_norm(x, m.final_norm, c.norm_eps, residual=pending)
        lt = torch.tensor(lengths, dtype=torch.int32)
        self.cache.lens[rows] = lt.to(self.device)
        for r, n in zip(slots, lengths):
            self.cache.host_lens[r] = int(n)
        last = y.view(B, S, -1)[torch.arange(B, device=y.device), (lt.long() - 1).to(y.device)]
        return torch.mm(last, self._head().t()).float()

    @torch.no_grad()
    def decode(self, tok: torch.Tensor, active: list | None = None) -> torch.Tensor:
        """One new token per sequence ``tok`` [B] (cache rows [0, B)) at position lens[b] -> next-token logits
        [B, vocab] (fp32). ``active`` (host list of bools, continuous batching): only those rows advance; the
        others compute throw-away rows of the same batched GEMMs."""
        B = tok.shape[0]
        rows = range(B) if active is None else [r for r in range(B) if active[r]]
        if max((self.cache.host_lens[r] for r in rows), default=0) + 1 > self.cache.max_seq:
            raise ValueError("KV cache is full")
        max_len = max(self.cache.host_lens[:B]) + 1
        if active is not None:
            act = torch.tensor([bool(x) for x in active[:B]], dtype=torch.int32).to(self.device, non_blocking=True)
            out = self._decode(tok, max_len, act)
        elif not self.graph:
            out = self._decode(tok, max_len)
        else:
            if B not in self._graphs:
                self._capture(B, tok)
            g, static_tok, static_out = self._graphs[B]
            static_tok.copy_(tok)
            g.replay()
            out = static_out.clone()
        for r in rows:
            self.cache.host_lens[r] += 1
        return out

    def _capture(self, B: int, tok: torch.Tensor) -> None:
        static_tok = tok.clone()
        lens0 = self.cache.lens.clone()
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):  # warm-up outside capture (library handles, workspaces); state restored below
            self._decode(static_tok, self.cache.max_seq)
        torch.cuda.current_stream().wait_stream(s)
        self.cache.lens.copy_(lens0)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            static_out = self._decode(static_tok, self.cache.max_seq)
        self.cache.lens.copy_(lens0)  # capture does not run the kernels, but keep the state exact either way
        self._graphs[B] = (g, static_tok, static_out)

    def _decode(self, tok: torch.Tensor, max_len: int, active: torch.Tensor | None = None) -> torch.Tensor:
        """Device-side body of a decode step (no host reads: capturable); ``max_len`` sizes the split grid."""
        c, m = self.cfg, self.model
        B = tok.shape[0]
        Hq, Hkv, D = c.n_heads, c.n_kv_heads, c.head_dim
        a, kc = Hq * D, (Hq + Hkv) * D
        pos = self.cache.lens[:B].clone()
        rows = self._rows(B)
        pl = pos.long()
        lens = pos + 1
        x = kf.embedding(tok.reshape(-1), m.tok_emb)
        pending = None
        for i, blk in enumerate(m.layers):
            if pending is None:
                y, x1 = kf.rms_norm(x, blk.attn_norm, c.norm_eps), x
            else:
                y, x1 = kf.rms_norm(x, blk.attn_norm, c.norm_eps, residual=pending)
            qkv = self._lin(y, blk.wqkv)
            if qkv.is_cuda:  # one kernel: RoPE at pos on Q / K + K / V rows appended to the cache
                from ..ops import load

                load().decode_rope_append_(qkv, self.cos, self.sin, pos, self.cache.k[i], self.cache.v[i], Hq)
            else:
                kf.rope_positions_(qkv, self.cos, self.sin, pos, Hq + Hkv, D)
                self.cache.k[i][rows, :, pl] = qkv[:, a:kc].reshape(B, Hkv, D)
                self.cache.v[i][rows, :, pl] = qkv[:, kc:].reshape(B, Hkv, D)
            o = kf.decode_attention(qkv[:, :a], self.cache.k[i][:B], self.cache.v[i][:B], lens, max_len, self.scale)
            y2, x = kf.rms_norm(x1, blk.mlp_norm, c.norm_eps, residual=self._lin(o, blk.wo))
            pending = self._mlp(blk, y2)
        y, _ = kf.rms_norm(x, m.final_norm, c.norm_eps, residual=pending)
        self.cache.lens[:B] = lens if active is None else pos + active
        return self._lin(y, self._head()).float() if self._gemv_ok(y, self._head()) else \
            torch.mm(y, self._head().t()).float()

    def _rows(self, B: int) -> torch.Tensor:
        key = ("rows", B)
        if key not in self._graphs:
            self._graphs[key] = torch.arange(B, device=self.device)
        return self._graphs[key]

    @torch.no_grad()
    def generate(self, ids: torch.Tensor, max_new_tokens: int) -> torch.Tensor:
        """Greedy continuation: [B, S] prompt -> [B, S + max_new_tokens] tokens."""
        out = [ids]
        logits = self.prefill(ids)
        for _ in range(max_new_tokens):
            nxt = logits.argmax(-1)
            out.append(nxt.unsqueeze(1).to(ids.dtype))
            if len(out) - 1 == max_new_tokens:
                break
            logits = self.decode(nxt)
        return torch.cat(out, dim=1)
