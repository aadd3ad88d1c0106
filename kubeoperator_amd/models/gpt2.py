"""GPT-2 (BASELINE config #3, "GPT-2-small bf16 on 1 MI355X"), true architecture: learned positions, pre-LN
LayerNorm blocks with biases, GELU(tanh) MLP, tied input/output embeddings.

Same execution structure as :mod:`.llama`: 2-D token activations, fused residual-add + LayerNorm kernel,
fused QKV projection feeding the flash-attention kernel through strided column views (head_dim 64, no
RoPE), GELU kernel, fused LM-head + cross-entropy. The vocabulary is padded to 50,304 (a multiple of 128)
so LM-head GEMMs and the cross-entropy rows stay vector-aligned.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
from torch.utils.checkpoint import checkpoint

from ..ops import functional as kf
from ..parallel.flat import ParamSpec
from .config import ModelConfig


class GPT2Block(nn.Module):
    def __init__(self, cfg: ModelConfig):
        super().__init__()
        H, F = cfg.hidden, cfg.ffn_hidden
        self.cfg = cfg
        self.ln1_w = nn.Parameter(torch.empty(H))
        self.ln1_b = nn.Parameter(torch.empty(H))
        self.attn_w = nn.Parameter(torch.empty(3 * H, H))
        self.attn_b = nn.Parameter(torch.empty(3 * H))
        self.proj_w = nn.Parameter(torch.empty(H, H))
        self.proj_b = nn.Parameter(torch.empty(H))
        self.ln2_w = nn.Parameter(torch.empty(H))
        self.ln2_b = nn.Parameter(torch.empty(H))
        self.fc_w = nn.Parameter(torch.empty(F, H))
        self.fc_b = nn.Parameter(torch.empty(F))
        self.out_w = nn.Parameter(torch.empty(H, F))
        self.out_b = nn.Parameter(torch.empty(H))

    def forward(self, x, pending, B, S):
        c = self.cfg
        if pending is None:
            y, x1 = kf.layer_norm(x, self.ln1_w, self.ln1_b, c.norm_eps), x
        else:
            y, x1 = kf.layer_norm(x, self.ln1_w, self.ln1_b, c.norm_eps, residual=pending)
        qkv = kf.linear(y, self.attn_w, self.attn_b)
        a = kf.rope_attention(qkv, None, None, B, S, c.n_heads, c.n_heads, c.head_dim, causal=True, use_rope=False)
        a = kf.linear(a, self.proj_w, self.proj_b)
        y2, x2 = kf.layer_norm(x1, self.ln2_w, self.ln2_b, c.norm_eps, residual=a)
        h = kf.gelu(kf.linear(y2, self.fc_w, self.fc_b))
        return x2, kf.linear(h, self.out_w, self.out_b)


class GPT2(nn.Module):
    def __init__(self, cfg: ModelConfig):
        super().__init__()
        assert cfg.arch == "gpt2" and cfg.tie_embeddings
        self.cfg = cfg
        self.wte = nn.Parameter(torch.empty(cfg.vocab_size, cfg.hidden))
        self.wpe = nn.Parameter(torch.empty(cfg.max_seq_len, cfg.hidden))
        self.layers = nn.ModuleList([GPT2Block(cfg) for _ in range(cfg.n_layers)])
        self.lnf_w = nn.Parameter(torch.empty(cfg.hidden))
        self.lnf_b = nn.Parameter(torch.empty(cfg.hidden))
        self.recompute = False  # activation recompute per block (set by the trainer)

    def param_specs(self) -> list[ParamSpec]:
        c = self.cfg
        std = c.init_std
        out_std = std / math.sqrt(2 * c.n_layers)
        specs = [ParamSpec("wte", self.wte, True, 2, "normal", std)]
        for i in reversed(range(c.n_layers)):
            L = self.layers[i]
            specs += [
                ParamSpec(f"layers.{i}.out_w", L.out_w, True, 1, "normal", out_std),
                ParamSpec(f"layers.{i}.fc_w", L.fc_w, True, 1, "normal", std),
                ParamSpec(f"layers.{i}.proj_w", L.proj_w, True, 1, "normal", out_std),
                ParamSpec(f"layers.{i}.attn_w", L.attn_w, True, 1, "normal", std),
            ]
        specs.append(ParamSpec("wpe", self.wpe, True, 1, "normal", 0.01))
        specs += [ParamSpec("lnf_w", self.lnf_w, False, 1, "ones"), ParamSpec("lnf_b", self.lnf_b, False, 1, "zeros")]
        for i in reversed(range(c.n_layers)):
            L = self.layers[i]
            for nm, init in (("out_b", "zeros"), ("fc_b", "zeros"), ("ln2_w", "ones"), ("ln2_b", "zeros"),
                             ("proj_b", "zeros"), ("attn_b", "zeros"), ("ln1_w", "ones"), ("ln1_b", "zeros")):
                specs.append(ParamSpec(f"layers.{i}.{nm}", getattr(L, nm), False, 1, init))
        return specs

    def forward(self, ids: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        B, S = ids.shape
        pos = torch.arange(S, device=ids.device).repeat(B)
        x = kf.embedding(ids.reshape(-1), self.wte) + kf.embedding(pos, self.wpe)
        pending = None
        for blk in self.layers:
            if self.recompute and torch.is_grad_enabled():
                x, pending = checkpoint(blk, x, pending, B, S, use_reentrant=False)
            else:
                x, pending = blk(x, pending, B, S)
        y, _ = kf.layer_norm(x, self.lnf_w, self.lnf_b, self.cfg.norm_eps, residual=pending)
        return kf.cross_entropy_lmhead(y, self.wte, targets.reshape(-1))
