"""Data parallelism over RCCL: bucketed gradient collectives overlapped with backward.

Two modes over the same flat/bucketed gradient layout (``parallel.flat``):

``allreduce`` (DDP)
    each bucket is all-reduced (SUM; the 1/world average is folded into the optimizer's fp32 grad scale)
    the moment backward has written its last gradient, from inside the backward pass, so ring traffic
    overlaps the remaining backward GEMMs. Every rank then runs the fused AdamW over all parameters.

``zero1`` (ZeRO stage 1: optimizer-state sharding)
    each bucket is reduce-scattered IN PLACE (rank r receives the reduced piece r of every bucket);
    rank r keeps fp32 master/exp_avg/exp_avg_sq only for its pieces (12 B/param / world instead of
    12 B/param) and runs AdamW only over them (1/world of the optimizer's HBM traffic); the updated
    bf16 pieces are all-gathered IN PLACE back into the flat parameter buffer. Same bytes on the wire
    as all-reduce (reduce-scatter + all-gather = one ring all-reduce), less optimizer time and memory.

Sizing for MI355X: 288 GB of HBM means no memory pressure on bucket size; point-to-point xGMI ring
collectives are per-link bound with a fixed per-call cost, so buckets default to 512 MiB (a few dozen
calls per step at Llama-3-8B instead of hundreds of 25 MB DDP buckets). Collectives run on RCCL's own
stream; ``ProcessGroupNCCL`` orders them after the producing GEMMs on the compute stream, and
``finish_grads`` makes the compute stream wait for all of them before the optimizer.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops.optim import Segment
from .dist import DistInfo, collectives_on
from .flat import Bucket, FlatParamStore


class DataParallel:
    """``info`` is the data-parallel view of this rank: the whole job, or under tensor parallelism the ranks
    with this rank's TP index (``info.group``; ``tp`` the ``parallel.tensor.TPContext``)."""

    def __init__(self, store: FlatParamStore, info: DistInfo, mode: str = "allreduce", tp=None):
        if mode not in ("allreduce", "zero1"):
            raise ValueError(f"unknown data-parallel mode {mode!r}")
        self.store = store
        self.info = info
        self.group = info.group
        self.tp = tp
        # sequence parallelism: replicated parameters saw only this rank's token rows, so their buckets are
        # reduced over the whole job (TP x DP ranks), the sharded ones over the DP group
        self.sp = tp is not None and tp.seq_parallel
        self.job_rank = info.global_rank if info.global_rank >= 0 else info.rank
        self.job_world = info.world * (tp.size if tp is not None else 1)
        self.mode = mode
        self.world = info.world
        self.rank = info.rank
        self.sync = True
        self._works = []
        self._gather_works = []
        self.comm_bytes = 0  # gradient bytes handed to collectives (per rank, cumulative)
        self.gather_bytes = 0  # ZeRO-1 all-gather output bytes (per rank, cumulative)
        self.finish_waits: list | None = None  # (event, event) around finish_grads (exposed comm timing)
        # bench: per optimizer step, every bucket's (index, grads-ready event on the compute stream, collective Work)
        # and backward's end. Passive: no stream of its own and no wait on the collective -- RCCL's own start / end
        # events (TORCH_NCCL_ENABLE_TIMING=1) give each collective's duration after the timed region
        # (``timeline_summary``). (An extra stream blocking on every collective could share a hardware queue with
        # the compute stream under GPU_MAX_HW_QUEUES=4 and hold backward kernels behind it.)
        self.timeline: list | None = None
        self._tl_cur: list = []
        store.on_ready = self._on_ready
        store.collectives_live = lambda: self.sync and (self.world > 1 or self.force or self.sp)
        self.overlapped = False  # set once the optimizer publishes ZeRO-1 gathers itself
        # one-rank RCCL self-test (parallel.dist.rccl_selftest): world-1 buckets still go through the collectives
        self.force = info.world == 1 and collectives_on(info)

    def _topo(self, b: Bucket):
        """(group, rank, world) the bucket's gradient collective and ZeRO-1 pieces run over."""
        if self.sp and not b.shard:
            return None, self.job_rank, self.job_world
        return self.group, self.rank, self.world

    # -------------------------------------------------------------------------------------------
    def broadcast_params(self) -> None:
        if self.world > 1 or self.force:
            dist.broadcast(self.store.params, src=self.info.src, group=self.group)

    def _on_ready(self, b: Bucket) -> None:
        group, rank, world = self._topo(b)
        if (world == 1 and not self.force) or not self.sync:
            return
        g = self.store.grads[b.start:b.end]
        self.comm_bytes += g.numel() * g.element_size()
        timed = self.timeline is not None and g.is_cuda and self.info.backend == "nccl"
        if timed:
            ready = torch.cuda.Event(enable_timing=True)
            ready.record()  # compute stream: the bucket's last gradient is written here
        if self.mode == "allreduce":
            self._works.append(dist.all_reduce(g, group=group, async_op=True))
        else:
            a, e = b.piece(rank, world)
            self._works.append(dist.reduce_scatter_tensor(self.store.grads[a:e], g, group=group, async_op=True))
        if timed:
            self._tl_cur.append((b.index, ready, self._works[-1]))

    def finish_grads(self) -> None:
        """Make the current (compute) stream wait for every outstanding gradient collective. With
        ``finish_waits`` set (bench.py, GPU), the wait is bracketed by two timing events on the compute stream:
        backward's last kernel has run at the first, the last collective has completed at the second."""
        timed = self.finish_waits is not None and self._works and self.store.params.is_cuda
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        for w in self._works:
            w.wait()
        if timed:
            e1.record()
            self.finish_waits.append((e0, e1))
            if self.timeline is not None and self._tl_cur:
                self.timeline.append({"bwd_end": e0, "buckets": list(self._tl_cur)})
        self._tl_cur.clear()
        self._works.clear()

    @property
    def grad_scale(self) -> float:
        # under SP every rank's loss is the mean over its 1/tp of the rows: the summed gradients are tp x the job's
        return 1.0 / (self.world * (self.tp.size if self.sp else 1))

    def optimizer_segments(self) -> list[Segment]:
        st = self.store
        wd_of = {True: None, False: 0.0}
        tp = self.tp is not None and self.tp.enabled
        segs = []
        for b in st.buckets:
            _, rank, world = self._topo(b)
            whole = self.mode == "allreduce" or world == 1
            a, e = (b.start, b.end) if whole else b.piece(rank, world)
            # a replicated bucket's piece held identically by every TP rank counts 1/tp in the grad norm
            dup = tp and not b.shard and (whole or not self.sp)
            segs.append(Segment(st.params[a:e], st.grads[a:e], wd_of[b.decay], b.index,
                                1.0 / self.tp.size if dup else 1.0))
        return segs

    def publish_segment(self, seg: Segment):
        """Optimizer-overlap hook, called on the optimizer stream right after a bucket's AdamW launch.
        ZeRO-1: start the bucket's in-place all-gather there and hand its work back as the bucket's gate."""
        if self.mode != "zero1":
            return None
        b = self.store.buckets[seg.bucket]
        group, rank, world = self._topo(b)
        if world == 1 and not self.force:
            return None
        self.overlapped = True
        a, e = b.piece(rank, world)
        return self._gather(b, a, e, group, async_op=True)

    def _gather(self, b: Bucket, a: int, e: int, group, async_op: bool):
        """In-place all-gather of the bucket's updated pieces (RCCL on GPU; gloo runs the same call on CPU).

        Through ``params.data``: the parameters are views of the flat buffer and share ITS autograd version
        counter, so a collective writing bucket Y through a plain view would bump the version of the bucket-X
        weights the current forward has already saved for backward (gloo completes CUDA gathers with a
        ``copy_`` at ``wait()``, i.e. mid-forward when the gate is resolved). The ordering that matters --
        bucket Y written before any kernel reads it -- is the gate's stream dependency, not autograd's."""
        pd = self.store.params.data
        self.gather_bytes += (b.end - b.start) * pd.element_size()
        return dist.all_gather_into_tensor(pd[b.start:b.end], pd[a:e], group=group, async_op=async_op)

    def norm_allreduce(self):
        """The grad-norm sum of squares is summed over the ranks holding distinct gradient pieces: the DP
        group under ZeRO-1, the TP group under tensor parallelism, the whole job with both."""
        tp = self.tp is not None and self.tp.enabled
        if self.mode == "zero1" and (self.world > 1 or self.sp or self.force):
            if tp:
                return lambda t: dist.all_reduce(t)  # every rank: DP pieces x TP shards
            return lambda t: dist.all_reduce(t, group=self.group)
        if tp:
            return lambda t: dist.all_reduce(t, group=self.tp.group)
        return None

    def after_step(self) -> None:
        """ZeRO-1: all-gather the updated bf16 parameter pieces back into every rank's flat buffer."""
        if self.mode != "zero1" or self.overlapped:
            return
        st = self.store
        for b in st.buckets:
            group, rank, world = self._topo(b)
            if world == 1 and not self.force:
                continue
            a, e = b.piece(rank, world)
            w = self._gather(b, a, e, group, async_op=True)
            if w is not None:
                self._gather_works.append(w)
        self.wait_params()

    def wait_params(self) -> None:
        for w in self._gather_works:
            w.wait()
        self._gather_works.clear()


def _duration_ms(work) -> float | None:
    """A finished collective's GPU time from RCCL's start / end events (``TORCH_NCCL_ENABLE_TIMING=1``), else None."""
    try:
        d = work._get_duration()
    except (RuntimeError, AttributeError, ValueError):
        return None
    return float(d) if d is not None and d >= 0 else None


def timeline_summary(steps: list[dict]) -> dict | None:
    """Per-rank gradient-collective timeline (bench JSON), from ``DataParallel.timeline`` after a synchronize.

    Times are ms relative to backward's last kernel on the compute stream (negative: before it), medians over the
    timed steps. Measured: when each bucket's gradients were ready (compute-stream events) and each collective's own
    duration (RCCL's events, ``Work._get_duration``). Derived: the collectives run one after another on RCCL's
    stream, so collective i starts at max(its bucket ready, collective i-1 done) and is done ``duration`` later --
    ``last_done_ms`` > 0 is communication exposed after backward, ``comm_ms`` the summed collective time. Without
    RCCL timing (durations unavailable) only the ready times are reported."""
    rows = []
    for st in steps:
        bk = st["buckets"]
        if not bk:
            continue
        ref = bk[0][1]  # the first ready event: everything below is recorded after it
        t = lambda ev: ref.elapsed_time(ev)  # noqa: E731
        end = t(st["bwd_end"])
        ready = [t(r) - end for _, r, _ in bk]
        row = {"n_buckets": len(bk), "first_ready_ms": min(ready), "last_ready_ms": max(ready)}
        durs = [_duration_ms(w) for _, _, w in bk]
        if all(d is not None for d in durs):
            done, prev = [], float("-inf")
            for rd, d in zip(ready, durs):
                prev = max(rd, prev) + d
                done.append(prev)
            row.update({"first_done_ms": min(done), "last_done_ms": max(done), "in_flight_ms": max(done) - min(ready),
                        "comm_ms": sum(durs), "max_collective_ms": max(durs)})
        rows.append(row)
    return summarize_rows(rows)


def summarize_rows(rows: list[dict]) -> dict | None:
    """Median of each field over the steps (pure; tests feed it numbers)."""
    if not rows:
        return None
    out = {}
    for k in rows[0]:
        v = sorted(r[k] for r in rows)
        m = v[len(v) // 2] if len(v) % 2 else 0.5 * (v[len(v) // 2 - 1] + v[len(v) // 2])
        out[k] = round(m, 3) if isinstance(m, float) else m
    out["steps"] = len(rows)
    return out
