"""Tensor parallelism (Megatron-style column / row split of the Llama block projections) over RCCL.

Why and when on MI355X: one GPU holds Llama-3-8B with its fp32 optimizer state (288 GB of HBM), so the
headline chart runs pure data parallelism. TP is the lever for models whose weights + fp32 state do not fit
one GPU (Llama-3-70B: ~1.1 TB) or whose per-GPU micro-batch must stay small: the projections of every block
are split over ``tp`` GPUs of ONE node, where the 8 MI355X are fully connected by xGMI (7 links per GPU), so a
TP all-reduce of a [tokens, hidden] activation never leaves the node. Data parallelism runs across the TP
groups (``dp = world / tp``), with the usual bucketed reduce-scatter / all-gather (``parallel.ddp``).

Rank layout: TP groups are consecutive ranks (``[g*tp, (g+1)*tp)``: with one process per GPU these are
neighbouring GPUs of one node), DP groups are the ranks with the same TP rank (stride ``tp``).

Per block (``models.llama.LlamaBlock``), with ``f`` = identity forward / all-reduce backward and
``g`` = all-reduce forward / identity backward:

    y1 = rmsnorm(x)                          replicated
    a  = g(attn(f(y1) @ Wqkv_r^T) @ Wo_r^T)  column split of Q/K/V by heads, row split of Wo
    y2 = rmsnorm(x + a)                      replicated
    m  = g(swiglu(f(y2) @ Wgu_r^T) @ Wd_r^T) column split of gate|up, row split of Wd

Two all-reduces per block forward and two in backward. On the GPU the backward ones are issued
asynchronously from inside the column-split projections' backward (``ops.functional.linear`` /
``swiglu_mlp`` with ``tp_group``) right after their data-gradient GEMM, so they run on RCCL's stream under the
weight-gradient GEMM; the forward ones sit on the critical path. Norm weights, embeddings and the LM head are
replicated: their gradients come out identical on every TP rank (replicated inputs, all-reduced output
gradients), so they need no TP reduction; the gradient-norm sum counts each replicated bucket once (it is
weighted 1/tp before the sum over TP ranks, see ``ops.optim``).

Sequence parallelism (``--sp``, Megatron-SP): between the projections the residual stream, the norms and the
LM head + cross-entropy work on 1/tp of the token rows. ``f`` becomes an all-gather of the rows (reduce-scatter
in backward) and ``g`` a reduce-scatter (all-gather in backward): the same bytes on xGMI as the two all-reduces,
while norm / residual activations and the LM head's vocabulary GEMMs and cross-entropy shrink by tp (without SP
every TP rank computes the whole 128k-vocabulary head). Each rank's loss is the mean over its rows, so all
gradients come out tp x the job's; replicated parameters (norms, embeddings, LM head) then see only their rank's
rows and are reduced over the whole job (TP x DP) instead of the DP group (``parallel.ddp``).

The reference has no model code at all (TP "not required; optional later"); this is the
MI355X-native option for models past Llama-3-8B.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist
from torch.autograd import Function

from .dist import DistInfo


@dataclass
class TPContext:
    size: int = 1
    rank: int = 0
    group: object = None  # torch.distributed group of this rank's TP peers (None when size == 1)
    sp: bool = False  # sequence parallelism: the residual stream is split over the group by token rows

    @property
    def enabled(self) -> bool:
        return self.size > 1

    @property
    def seq_parallel(self) -> bool:
        return self.sp and self.size > 1


def make_groups(info: DistInfo, tp: int, sp: bool = False) -> tuple[DistInfo, TPContext]:
    """Split the job into TP groups of ``tp`` consecutive ranks and DP groups across them. Returns the
    data-parallel view of this rank (``DistInfo`` with the DP rank / size / group) and its TP context.
    Every rank creates every group, in the same order (``new_group`` is collective)."""
    if tp <= 1:
        return info, TPContext()
    world = info.world
    if world % tp != 0:
        raise ValueError(f"world size {world} is not a multiple of tp {tp}")
    tp_group = dp_group = None
    for g in range(world // tp):
        ranks = list(range(g * tp, (g + 1) * tp))
        grp = dist.new_group(ranks)
        if info.rank in ranks:
            tp_group = grp
    dp_ranks = None
    for t in range(tp):
        ranks = list(range(t, world, tp))
        grp = dist.new_group(ranks)
        if info.rank in ranks:
            dp_group, dp_ranks = grp, ranks
    dp_info = DistInfo(rank=info.rank // tp, local_rank=info.local_rank, world=world // tp, backend=info.backend,
                       device=info.device, group=dp_group, src=dp_ranks[0], global_rank=info.rank)
    return dp_info, TPContext(tp, info.rank % tp, tp_group, sp)


class _CopyToTP(Function):
    """f: identity in forward; the input gradient is summed over the TP group in backward."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        dist.all_reduce(g, group=ctx.group)
        return g, None


class _ReduceFromTP(Function):
    """g: partial outputs of a row-split projection summed over the TP group in forward (in place on the
    fresh GEMM output, which nothing else reads and no backward saved); the gradient passes through."""

    @staticmethod
    def forward(ctx, x, group):
        x = x.contiguous()
        dist.all_reduce(x, group=group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _GatherFromSP(Function):
    """Sequence parallelism, entering a column split: the token-row shards of the group are concatenated
    (all-gather along rows) in forward; the full-row gradient is reduce-scattered back to the shards."""

    @staticmethod
    def forward(ctx, x, group, n):
        ctx.group, ctx.n = group, n
        x = x.contiguous()
        out = torch.empty((x.shape[0] * n,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x, group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        out = torch.empty((g.shape[0] // ctx.n,) + tuple(g.shape[1:]), dtype=g.dtype, device=g.device)
        dist.reduce_scatter_tensor(out, g, group=ctx.group)
        return out, None, None


class _ScatterToSP(Function):
    """Sequence parallelism, leaving a row split: the partial full-row outputs are summed AND split by token
    rows (reduce-scatter) in forward; the shard gradients are all-gathered in backward."""

    @staticmethod
    def forward(ctx, x, group, n):
        ctx.group, ctx.n = group, n
        x = x.contiguous()
        out = torch.empty((x.shape[0] // n,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.reduce_scatter_tensor(out, x, group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        out = torch.empty((g.shape[0] * ctx.n,) + tuple(g.shape[1:]), dtype=g.dtype, device=g.device)
        dist.all_gather_into_tensor(out, g, group=ctx.group)
        return out, None, None


def sp_gather(x: torch.Tensor, tp: TPContext) -> torch.Tensor:
    return _GatherFromSP.apply(x, tp.group, tp.size)


def sp_scatter(x: torch.Tensor, tp: TPContext) -> torch.Tensor:
    return _ScatterToSP.apply(x, tp.group, tp.size)


def sp_rows(n_rows: int, tp: TPContext) -> slice:
    """This rank's token rows of a [n_rows, ...] activation under sequence parallelism."""
    if n_rows % tp.size != 0:
        raise ValueError(f"{n_rows} token rows do not split over tp {tp.size} (sequence parallelism)")
    k = n_rows // tp.size
    return slice(tp.rank * k, (tp.rank + 1) * k)


def copy_to_tp(x: torch.Tensor, tp: TPContext) -> torch.Tensor:
    return _CopyToTP.apply(x, tp.group) if tp.enabled else x


def reduce_from_tp(x: torch.Tensor, tp: TPContext) -> torch.Tensor:
    return _ReduceFromTP.apply(x, tp.group) if tp.enabled else x


# ---------------------------------------------------------------------------------------------------
# shard maps: which part of a full (tp = 1) Llama weight TP rank r owns -- weight conversion and tests
# ---------------------------------------------------------------------------------------------------
def shard_llama_weight(name: str, full: torch.Tensor, cfg, tp: int, r: int) -> torch.Tensor:
    """The slice of the full parameter ``name`` held by TP rank ``r`` (replicated parameters: the whole)."""
    if tp <= 1:
        return full
    leaf = name.rsplit(".", 1)[-1]
    D = cfg.head_dim
    if leaf == "wqkv":
        hq, hkv = cfg.n_heads // tp, cfg.n_kv_heads // tp
        q = full[: cfg.n_heads * D]
        k = full[cfg.n_heads * D: (cfg.n_heads + cfg.n_kv_heads) * D]
        v = full[(cfg.n_heads + cfg.n_kv_heads) * D:]
        return torch.cat([q[r * hq * D:(r + 1) * hq * D], k[r * hkv * D:(r + 1) * hkv * D],
                          v[r * hkv * D:(r + 1) * hkv * D]])
    if leaf == "wo":
        n = cfg.n_heads * D // tp
        return full[:, r * n:(r + 1) * n]
    if leaf == "w_gate_up":
        F = cfg.ffn_hidden
        n = F // tp
        return torch.cat([full[r * n:(r + 1) * n], full[F + r * n:F + (r + 1) * n]])
    if leaf == "w_down":
        n = cfg.ffn_hidden // tp
        return full[:, r * n:(r + 1) * n]
    return full


def check_llama_tp(cfg, tp: int) -> None:
    if tp <= 1:
        return
    if cfg.arch != "llama":
        raise ValueError("tensor parallelism is implemented for the Llama family")
    for what, n in (("n_heads", cfg.n_heads), ("n_kv_heads", cfg.n_kv_heads), ("ffn_hidden", cfg.ffn_hidden)):
        if n % tp != 0:
            raise ValueError(f"{what} = {n} is not divisible by tp = {tp}")
