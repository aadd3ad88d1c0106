"""Plain-PyTorch fp32 references of every HIP kernel (numerics oracle + CPU plumbing path).

Each function mirrors the semantics of the corresponding gfx950 kernel exactly (layouts, fused residual,
rotate-half RoPE on the first ``nheads`` heads of a row, GQA head mapping, mean cross-entropy with
ignore_index), computing in fp32 and returning the input dtype.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def rms_norm_ref(x, w, eps=1e-5, residual=None):
    s = x if residual is None else (x.float() + residual.float()).to(x.dtype)
    sf = s.float()
    y = sf * torch.rsqrt(sf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(x.dtype), s


def layer_norm_ref(x, w, b, eps=1e-5, residual=None):
    s = x if residual is None else (x.float() + residual.float()).to(x.dtype)
    y = F.layer_norm(s.float(), (s.shape[-1],), w.float(), b.float(), eps)
    return y.to(x.dtype), s


def rope_cache(S: int, D: int, theta: float, device=None):
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, dtype=torch.float64, device=device) / D))
    t = torch.arange(S, dtype=torch.float64, device=device)
    ang = torch.outer(t, inv)
    return torch.cos(ang).float().contiguous(), torch.sin(ang).float().contiguous()


def rope_ref(x, cos, sin, S: int, nheads: int, D: int, inverse: bool = False, pos=None):
    """Rotate-half RoPE on the first ``nheads`` heads of each row of x [T, >= nheads*D]; returns new tensor."""
    T = x.shape[0]
    out = x.clone()
    p = pos.long() if pos is not None else torch.arange(T, device=x.device) % S
    c = cos[p].unsqueeze(1)  # [T,1,D/2]
    s = sin[p].unsqueeze(1) * (-1.0 if inverse else 1.0)
    h = x[:, : nheads * D].float().view(T, nheads, D)
    a, b = h[..., : D // 2], h[..., D // 2:]
    rot = torch.cat([a * c - b * s, b * c + a * s], dim=-1)
    out[:, : nheads * D] = rot.reshape(T, nheads * D).to(x.dtype)
    return out


def swiglu_ref(gu):
    g, u = gu.float().chunk(2, dim=-1)
    return (F.silu(g) * u).to(gu.dtype)


def gelu_ref(x):
    return F.gelu(x.float(), approximate="tanh").to(x.dtype)


def attention_ref(q, k, v, B, S, Hq, Hkv, D, causal=True, scale=None):
    """q [B*S, >=Hq*D], k/v [B*S, >=Hkv*D] row views -> o [B*S, Hq*D], lse [B, Hq, S] (natural log)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    qh = q[:, : Hq * D].float().reshape(B, S, Hq, D).transpose(1, 2)
    kh = k[:, : Hkv * D].float().reshape(B, S, Hkv, D).transpose(1, 2)
    vh = v[:, : Hkv * D].float().reshape(B, S, Hkv, D).transpose(1, 2)
    rep = Hq // Hkv
    kh = kh.repeat_interleave(rep, dim=1)
    vh = vh.repeat_interleave(rep, dim=1)
    s = torch.matmul(qh, kh.transpose(-1, -2)) * scale
    if causal:
        mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, vh).transpose(1, 2).reshape(B * S, Hq * D)
    return o.to(q.dtype), lse


def cross_entropy_ref(logits, targets, ignore_index=-100):
    return F.cross_entropy(logits.float(), targets, ignore_index=ignore_index)


def adamw_ref(master, m, v, g, lr, b1, b2, eps, wd, step, gscale=1.0):
    g = g.float() * gscale
    m.mul_(b1).add_(g, alpha=1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    master.mul_(1 - lr * wd)
    master.sub_(lr * (m / bc1) / ((v.sqrt() / math.sqrt(bc2)) + eps))
    return master


def decode_attention_ref(q, k_cache, v_cache, lens, scale):
    """One query row per sequence against its cache: q [B, Hq*D], caches [B, Hkv, Smax, D], lens [B] valid keys."""
    B, Hkv, _, D = k_cache.shape
    Hq = q.shape[1] // D
    out = torch.empty(B, Hq * D, dtype=q.dtype, device=q.device)
    for b in range(B):
        n = int(lens[b])
        qh = q[b].float().view(Hq, 1, D)
        kh = k_cache[b, :, :n].float().repeat_interleave(Hq // Hkv, dim=0)  # [Hq, n, D]
        vh = v_cache[b, :, :n].float().repeat_interleave(Hq // Hkv, dim=0)
        p = torch.softmax((qh @ kh.transpose(1, 2)) * scale, dim=-1)
        out[b] = (p @ vh).reshape(Hq * D).to(q.dtype)
    return out
