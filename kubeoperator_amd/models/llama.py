"""Llama-3 decoder (the bundled chart's headline model), built on the gfx950 kernels.

Token activations are kept 2-D ``[B*S, hidden]`` end to end so every projection is one hipBLASLt GEMM and
every elementwise/normalisation kernel streams contiguous rows. Per block:

    y1, x1 = rmsnorm(x + pending)        fused residual-add + RMSNorm (one kernel)
    qkv    = y1 @ Wqkv^T                 fused Q|K|V projection, [T, (Hq + 2 Hkv) * 128]
    a      = flash_attn(rope(qkv))       RoPE in place on the Q/K columns, attention reads the strided
                                         Q/K/V column views directly (no split / transpose copies)
    y2, x2 = rmsnorm(x1 + a @ Wo^T)
    m      = swiglu(y2 @ Wgu^T) @ Wd^T   fused gate|up projection, SwiGLU kernel
    -> (x2, m)                           the residual add of m is fused into the next block's norm

With ``recompute`` each block keeps only its inputs for backward and re-runs its forward there (one more
forward pass, ~1/3 more FLOPs): what lets one MI355X train Llama-3-8B at 32k-token sequences.

With tensor parallelism (``tp``, ``parallel.tensor``) each block holds its TP rank's heads of Wqkv / Wo and
its slice of the FFN (gate|up rows, down columns); the two row-split projections end in a TP all-reduce.

The LM head and the cross-entropy are one autograd node whose logits buffer is overwritten by its own
gradient (``ops.cross_entropy_lmhead``). Weight gradients are written straight into the flat gradient
buffer (see ``parallel.flat``).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
from torch.utils.checkpoint import checkpoint

from ..ops import functional as kf
from ..ops.reference import rope_cache
from ..parallel.flat import ParamSpec
from ..parallel.tensor import TPContext, check_llama_tp, reduce_from_tp, sp_gather, sp_rows, sp_scatter
from .config import ModelConfig


class LlamaBlock(nn.Module):
    def __init__(self, cfg: ModelConfig, tp: TPContext | None = None):
        super().__init__()
        self.tp = tp or TPContext()
        t = self.tp.size
        H, D = cfg.hidden, cfg.head_dim
        self.cfg = cfg
        self.hq, self.hkv, self.ffn = cfg.n_heads // t, cfg.n_kv_heads // t, cfg.ffn_hidden // t  # this rank's
        self.attn_norm = nn.Parameter(torch.empty(H))
        self.wqkv = nn.Parameter(torch.empty((self.hq + 2 * self.hkv) * D, H))
        self.wo = nn.Parameter(torch.empty(H, self.hq * D))
        self.mlp_norm = nn.Parameter(torch.empty(H))
        self.w_gate_up = nn.Parameter(torch.empty(2 * self.ffn, H))
        self.w_down = nn.Parameter(torch.empty(H, self.ffn))

    def forward(self, x, pending, cos, sin, B, S, box_in=None, box_out=None):
        """``box_in`` / ``box_out`` (``kf.TBox``, set by ``Llama.forward`` when the transposed companions are on):
        the norms write y^T / dx^T for the weight gradients of the projections around them."""
        c, tp = self.cfg, self.tp
        if box_out is not None:
            return self._forward_t(x, pending, cos, sin, B, S, box_in, box_out)
        if pending is None:
            y, x1 = kf.rms_norm(x, self.attn_norm, c.norm_eps), x
        else:
            y, x1 = kf.rms_norm(x, self.attn_norm, c.norm_eps, residual=pending)
        if tp.seq_parallel:  # token-row shards: gathered into the column splits, reduce-scattered out of the rows
            qkv = kf.linear(sp_gather(y, tp), self.wqkv)
            a = kf.rope_attention(qkv, cos, sin, B, S, self.hq, self.hkv, c.head_dim, causal=True)
            y2, x2 = kf.rms_norm(x1, self.mlp_norm, c.norm_eps, residual=sp_scatter(kf.linear(a, self.wo), tp))
            return x2, sp_scatter(kf.swiglu_mlp(sp_gather(y2, tp), self.w_gate_up, self.w_down), tp)
        g = tp.group if tp.enabled else None  # column splits: input gradient summed over TP, overlapped
        qkv = kf.linear(y, self.wqkv, tp_group=g)
        a = kf.rope_attention(qkv, cos, sin, B, S, self.hq, self.hkv, c.head_dim, causal=True)
        a = reduce_from_tp(kf.linear(a, self.wo), tp)
        y2, x2 = kf.rms_norm(x1, self.mlp_norm, c.norm_eps, residual=a)
        return x2, reduce_from_tp(kf.swiglu_mlp(y2, self.w_gate_up, self.w_down, tp_group=g), tp)

    def _forward_t(self, x, pending, cos, sin, B, S, box_in, box_out):
        """One GPU rank, no TP: the forward norms hand y^T to the QKV / gate|up projections (``xt``), the backward
        norms hand dx^T to the Wo / W_down projections, the attention backward hands dQKV^T (fused with its
        inverse RoPE) to the QKV projection (``box``) and the attention forward hands O^T to Wo (``xt``): none of the
        block's weight-gradient GEMMs transposes an operand (csrc/norms.hip rms_fwd_t / rms_bwd_t,
        csrc/transpose.hip rope_t, csrc/flash_fwd.hip O^T tail)."""
        c = self.cfg
        if pending is None:
            (y, yt), x1 = kf.rms_norm(x, self.attn_norm, c.norm_eps, want_t=True), x
        else:
            y, x1, yt = kf.rms_norm(x, self.attn_norm, c.norm_eps, residual=pending, want_t=True, box=box_in)
        box_qkv = kf.TBox()
        qkv = kf.linear(y, self.wqkv, xt=yt, box=box_qkv)
        a, at = kf.rope_attention(qkv, cos, sin, B, S, self.hq, self.hkv, c.head_dim, causal=True, box=box_qkv,
                                  want_ot=True)
        box_wo = kf.TBox()
        a = kf.linear(a, self.wo, xt=at, box=box_wo)
        y2, x2, yt2 = kf.rms_norm(x1, self.mlp_norm, c.norm_eps, residual=a, want_t=True, box=box_wo)
        return x2, kf.swiglu_mlp(y2, self.w_gate_up, self.w_down, xt=yt2, box=box_out)


class Llama(nn.Module):
    def __init__(self, cfg: ModelConfig, tp: TPContext | None = None):
        super().__init__()
        assert cfg.arch == "llama"
        self.tp = tp or TPContext()
        check_llama_tp(cfg, self.tp.size)
        self.cfg = cfg
        self.tok_emb = nn.Parameter(torch.empty(cfg.vocab_size, cfg.hidden))
        self.layers = nn.ModuleList([LlamaBlock(cfg, self.tp) for _ in range(cfg.n_layers)])
        self.final_norm = nn.Parameter(torch.empty(cfg.hidden))
        if not cfg.tie_embeddings:
            self.lm_head = nn.Parameter(torch.empty(cfg.vocab_size, cfg.hidden))
        self._rope = {}
        self.recompute = False  # activation recompute per block (set by the trainer)

    # flat layout: reverse order of gradient readiness in backward; norms in the no-decay region
    def param_specs(self) -> list[ParamSpec]:
        c = self.cfg
        std = c.init_std
        out_std = std / math.sqrt(2 * c.n_layers)
        sh = self.tp.enabled  # block projections are TP shards
        specs = []
        if not c.tie_embeddings:
            specs.append(ParamSpec("lm_head", self.lm_head, True, 1, "normal", std))
        for i in reversed(range(c.n_layers)):
            L = self.layers[i]
            specs += [
                ParamSpec(f"layers.{i}.w_down", L.w_down, True, 1, "normal", out_std, sh),
                ParamSpec(f"layers.{i}.w_gate_up", L.w_gate_up, True, 1, "normal", std, sh),
                ParamSpec(f"layers.{i}.wo", L.wo, True, 1, "normal", out_std, sh),
                ParamSpec(f"layers.{i}.wqkv", L.wqkv, True, 1, "normal", std, sh),
            ]
        specs.append(ParamSpec("tok_emb", self.tok_emb, True, 2 if c.tie_embeddings else 1, "normal", std))
        specs.append(ParamSpec("final_norm", self.final_norm, False, 1, "ones"))
        for i in reversed(range(c.n_layers)):
            specs.append(ParamSpec(f"layers.{i}.mlp_norm", self.layers[i].mlp_norm, False, 1, "ones"))
            specs.append(ParamSpec(f"layers.{i}.attn_norm", self.layers[i].attn_norm, False, 1, "ones"))
        return specs

    def fp8_param_names(self) -> list[str]:
        """The block projections whose forward / data-gradient GEMMs may run in E4M3 (``--fp8``)."""
        return [f"layers.{i}.{n}" for i in range(self.cfg.n_layers) for n in ("wqkv", "wo", "w_gate_up", "w_down")]

    def rope_tables(self, S, device):
        key = (S, str(device))
        if key not in self._rope:
            self._rope[key] = rope_cache(S, self.cfg.head_dim, self.cfg.rope_theta, device=device)
        return self._rope[key]

    def _companions(self, x) -> bool:
        """Norm kernels with transposed outputs: one rank of the block projections (no TP), bf16 GEMMs (the FP8
        path transposes while casting), H 2048 / 4096 and T a multiple of 16 (``kf.norm_t_enabled``)."""
        return (x.is_cuda and torch.is_grad_enabled() and not self.tp.enabled and kf.norm_t_enabled()
                and getattr(self.layers[0].wqkv, "w8", None) is None and kf._t_ok(x))

    def forward(self, ids: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        B, S = ids.shape
        cos, sin = self.rope_tables(S, ids.device)
        ids, targets = ids.reshape(-1), targets.reshape(-1)
        if self.tp.seq_parallel:  # this rank's token rows: embedding, norms, LM head and loss on 1/tp of them
            rows = sp_rows(ids.numel(), self.tp)
            ids, targets = ids[rows], targets[rows]
        x = kf.embedding(ids, self.tok_emb)
        pending = None
        # transposed companions of the norms (see LlamaBlock._forward_t): one box per block for its MLP output
        boxes = [kf.TBox() for _ in self.layers] if self._companions(x) else [None] * len(self.layers)
        box_in = None
        for blk, box in zip(self.layers, boxes):
            if self.recompute and torch.is_grad_enabled():
                # keep only the block's inputs; its activations are rebuilt in backward (long sequences)
                x, pending = checkpoint(blk, x, pending, cos, sin, B, S, box_in, box, use_reentrant=False)
            else:
                x, pending = blk(x, pending, cos, sin, B, S, box_in, box)
            box_in = box
        y, _ = kf.rms_norm(x, self.final_norm, self.cfg.norm_eps, residual=pending, box=box_in)
        head = self.tok_emb if self.cfg.tie_embeddings else self.lm_head
        return kf.cross_entropy_lmhead(y, head, targets)
