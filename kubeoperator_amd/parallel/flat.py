"""Flat parameter / gradient storage with a communication-bucket layout.

Every trainable parameter of the model becomes a view into ONE contiguous bf16 buffer (``params``) and its
gradient a view into ONE contiguous bf16 (optionally fp32) buffer (``grads``, exposed as ``param.main_grad``). The layout is
decided once, MI355X-first:

* parameters are placed in the order their gradients become ready during backward (reverse forward
  order), so buckets close in the order backward produces them and each bucket's collective overlaps the
  rest of backward;
* weight-decayed and non-decayed parameters live in two contiguous regions (one fused-AdamW launch each);
* each bucket is padded so its length is a multiple of ``world * 128`` elements: a bucket splits into
  ``world`` equal, 256-byte aligned pieces, which is exactly what in-place ``reduce_scatter`` /
  ``all_gather`` (ZeRO-1) need, and every view starts 16-byte aligned for the vectorised kernels;
* bucket size defaults to 512 MiB: with 288 GB of HBM per GPU there is no memory pressure to keep
  buckets small, and on point-to-point xGMI fewer, larger ring collectives amortise per-call latency
  (~16 GB of Llama-3-8B bf16 gradients -> ~32 buckets).

Readiness is counted per parameter *use* (tied embeddings are used twice): when all uses of all
parameters of a bucket have written their gradient, the bucket's ``on_ready`` callback fires.

Forward gates (optimizer overlap): the fused AdamW may run on its own HIP stream, bucket by bucket in the
order the forward pass first touches them, and publish a *gate* per bucket (an event, or the RCCL
all-gather work under ZeRO-1). The kernels' Python wrappers call ``await_param`` on every weight they read,
which makes the compute stream wait for that bucket's gate only -- so the memory-bound optimizer of step k
streams underneath the compute-bound forward GEMMs of step k+1 instead of running alone.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import torch
import torch.nn as nn

ALIGN = 128  # elements (256 bytes of bf16)


def _round_up(n: int, m: int) -> int:
    return (n + m - 1) // m * m


@dataclass
class ParamSpec:
    name: str
    param: nn.Parameter
    weight_decay: bool = True
    uses: int = 1
    init: str = "normal"  # normal | ones | zeros | normal_scaled
    std: float = 0.02
    shard: bool = False  # tensor-parallel shard (parallel.tensor): own buckets, own init stream per TP rank


@dataclass
class Bucket:
    index: int
    start: int
    end: int  # padded end (exclusive)
    names: list = field(default_factory=list)
    expected: int = 0
    pending: int = 0
    decay: bool = True
    shard: bool = False  # holds tensor-parallel shards (replicated parameters never share its bucket)

    @property
    def numel(self) -> int:
        return self.end - self.start

    def piece(self, rank: int, world: int) -> tuple[int, int]:
        n = self.numel // world
        return self.start + rank * n, self.start + (rank + 1) * n


def _resolve(gate) -> None:
    if isinstance(gate, torch.cuda.Event):
        torch.cuda.current_stream().wait_event(gate)
    else:  # torch.distributed work: wait() orders the current stream after the collective
        gate.wait()


class GradHooks:
    """Shared by all parameters of a store; consulted by the backward kernels (see ops.functional._sink)."""

    def __init__(self, store: "FlatParamStore"):
        self.store = store
        self.microbatch = 0
        self.writes: dict[int, int] = {}

    def accumulate_for(self, p) -> bool:
        return self.microbatch > 0 or self.writes.get(id(p), 0) > 0

    @property
    def accumulate(self) -> bool:  # legacy single-use form
        return self.microbatch > 0

    def ready(self, p) -> None:
        k = id(p)
        self.writes[k] = self.writes.get(k, 0) + 1
        self.store._param_written(p)


# ``record_stream`` on the side stream's inputs as well as ``hold_side``'s references (KOP_SIDE_RECORD_STREAM=1, the
# round-2..5 behaviour): redundant -- the reference is dropped only after the side stream has passed the reading
# launch -- and harmful: a block freed with a recorded stream waits for that stream's work queued AT FREE TIME, and the
# lagging side stream always has some, so the compute stream kept allocating fresh segments. GPT-2-small reserved
# 245 GB for 57 GB allocated at micro-batch 32 and ran out of memory (then every step synchronised and freed the
# cache: 4x slower) at micro-batch 64 (profiles/r6_gpt2_side_memory_ab.jsonl)
_RECORD_STREAM = os.environ.get("KOP_SIDE_RECORD_STREAM", "0") == "1"


class FlatParamStore:
    def __init__(self, module: nn.Module, specs: list[ParamSpec], device, dtype=torch.bfloat16, world: int = 1,
                 bucket_bytes: int = 512 * 1024 * 1024, grad_dtype=None):
        self.module = module
        self.world = world
        self.dtype = dtype
        # bf16 by default (half the collective bytes); fp32 keeps micro-batch accumulation and the
        # data-parallel reduction in fp32 (many accumulation steps x large worlds)
        self.grad_dtype = grad_dtype or dtype
        self.device = torch.device(device)
        names = [s.name for s in specs]
        own = dict(module.named_parameters())
        missing = set(own) - set(names)
        if missing:
            raise ValueError(f"parameters not covered by the flat layout: {sorted(missing)}")
        decay = [s for s in specs if s.weight_decay]
        nodecay = [s for s in specs if not s.weight_decay]
        esize = torch.tensor([], dtype=dtype).element_size()
        cap = max(ALIGN, bucket_bytes // esize)
        quantum = ALIGN * max(1, world)
        self.buckets: list[Bucket] = []
        offsets: dict[str, int] = {}
        off = 0

        def close(b: Bucket):
            b.end = _round_up(b.end, quantum)
            self.buckets.append(b)
            return b.end

        for region, is_decay in ((decay, True), (nodecay, False)):
            cur = None
            for s in region:
                n = s.param.numel()
                if cur is not None and ((cur.end - cur.start) + n > cap or cur.shard != s.shard):
                    off = close(cur)
                    cur = None
                if cur is None:
                    cur = Bucket(len(self.buckets), off, off, decay=is_decay, shard=s.shard)
                offsets[s.name] = cur.end
                cur.end = _round_up(cur.end + n, ALIGN)
                cur.names.append(s.name)
                cur.expected += s.uses
            if cur is not None:
                off = close(cur)
        self.numel = off
        self.decay_end = max([b.end for b in self.buckets if b.decay], default=0)
        self.params = torch.zeros(self.numel, dtype=dtype, device=self.device)
        self.grads = torch.zeros(self.numel, dtype=self.grad_dtype, device=self.device)
        self.hooks = GradHooks(self)
        self.specs = {s.name: s for s in specs}
        self.offsets = offsets
        self._bucket_of: dict[int, Bucket] = {}
        self._param_by_name: dict[str, nn.Parameter] = {}
        self.on_ready = None  # callable(Bucket)
        # True while readiness launches gradient collectives this micro-batch (DataParallel sets it); defer() refuses then
        self.collectives_live = lambda: False
        self.gates: dict[int, object] = {}  # bucket index -> torch.cuda.Event | collective work
        self.use_order: list[int] = []  # bucket indices in the order the forward pass first reads them
        self._used: set[int] = set()
        self._side = None  # weight-gradient stream (ops.functional._sink)
        self._held: list = []  # (event, tensors) the side stream still reads (hold_side)
        # side-stream gradient launches deferred past the next micro-batch's forward (ops.functional._sink(defer=True));
        # allowed only while a later micro-batch of the step follows (the trainer sets defer_ok)
        self._deferred: list = []
        self.defer_ok = False
        # side-stream launches issued as one group (``side_submit``): every group costs the compute stream one event
        # record, a marker packet that holds its next kernel back ~12 us on MI355X, and the side stream one wait.
        # KOP_SIDE_BATCH launches per group (1: each launch forks on its own). GPT-2-small, same box: 8 -> +1.6-2.0 %
        # over 1; 12-64 no better (profiles/r6_gpt2_side_batch_bucket_ab.jsonl, r6_gpt2_side_hint_ab.jsonl)
        self.side_batch = max(1, int(os.environ.get("KOP_SIDE_BATCH", "8")))
        self._side_q: list = []
        self._flush_at_end = False  # an end-of-backward flush is queued with the autograd engine
        self.gate_waits: list | None = None  # (event, event) around collective-gate waits (exposed comm timing)
        self.wgrad_stream = False  # issue weight gradients on it (set by the trainer)
        name_to_bucket = {nm: b for b in self.buckets for nm in b.names}
        for s in specs:
            n = s.param.numel()
            o = offsets[s.name]
            view = self.params[o:o + n].view(s.param.shape)
            p = nn.Parameter(view, requires_grad=True)
            p.main_grad = self.grads[o:o + n].view(s.param.shape)
            p._kop_hooks = self.hooks
            p._kop_name = s.name
            self._replace(s.name, p)
            self._bucket_of[id(p)] = name_to_bucket[s.name]
            self._param_by_name[s.name] = p
            # CPU / non-kernel path: autograd accumulates into p.grad -> copy into main_grad
            p.register_post_accumulate_grad_hook(self._fallback_hook)
        self.reset_readiness()

    # -------------------------------------------------------------------------------------------
    def _replace(self, name: str, p: nn.Parameter) -> None:
        mod = self.module
        parts = name.split(".")
        for a in parts[:-1]:
            mod = getattr(mod, a)
        mod._parameters[parts[-1]] = p

    def _fallback_hook(self, p: nn.Parameter) -> None:
        g = p.grad
        if g is None:
            return
        if self.hooks.accumulate_for(p):
            p.main_grad.add_(g.to(p.main_grad.dtype))
        else:
            p.main_grad.copy_(g)
        p.grad = None
        self.hooks.ready(p)

    def param(self, name: str) -> nn.Parameter:
        return self._param_by_name[name]

    def named_params(self):
        return self._param_by_name.items()

    # -------------------------------------------------------------------------------------------
    def init_weights(self, seed: int = 0, shard_rank: int = 0) -> None:
        """Initialise every parameter in place on its device (no host round trip at 8B params). Tensor-parallel
        shards draw from a stream seeded by their TP rank; replicated parameters from one stream every rank
        shares (so they start identical across the TP group)."""
        g = torch.Generator(device=self.device)
        g.manual_seed(seed)
        gs = torch.Generator(device=self.device)
        gs.manual_seed(seed + 7919 * (shard_rank + 1))
        with torch.no_grad():
            for name, p in self._param_by_name.items():
                s = self.specs[name]
                if s.init == "ones":
                    p.fill_(1.0)
                elif s.init == "zeros":
                    p.zero_()
                else:
                    p.normal_(0.0, s.std, generator=gs if s.shard else g)

    def reset_readiness(self) -> None:
        for b in self.buckets:
            b.pending = b.expected
        self.hooks.writes.clear()

    def begin_microbatch(self, index: int) -> None:
        self.flush_side()  # the previous backward's queued launches mark their parameters ready in ITS micro-batch
        self.hooks.microbatch = index
        self.reset_readiness()

    def _param_written(self, p) -> None:
        b = self._bucket_of.get(id(p))
        if b is None:
            return
        b.pending -= 1
        if b.pending == 0 and self.on_ready is not None:
            # (no collective this micro-batch: on_ready does nothing, and the fork would only cost a marker packet)
            if self._side is not None and self.collectives_live():
                # the bucket's gradients come from both streams: its collective is issued from the side stream
                # after that stream has also caught up with everything the compute stream wrote so far
                self._side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(self._side):
                    self.on_ready(b)
            else:
                self.on_ready(b)

    # weight-gradient stream ---------------------------------------------------------------------
    def side_stream(self):
        if self._side is None:
            # KOP_SIDE_PRIORITY: HIP stream priority of the weight-gradient stream (lower value = higher priority;
            # torch.cuda.Stream.priority_range()); 0 = the compute stream's own priority
            prio = int(os.environ.get("KOP_SIDE_PRIORITY", "0"))
            self._side = torch.cuda.Stream(device=self.device, priority=prio)
        return self._side

    def hold_side(self, tensors) -> None:
        """Keep references to tensors the side stream reads until it has passed them (see ops.functional._sink:
        a tensor autograd holds the only reference to may be accumulated into IN PLACE on the compute stream, and
        memory the allocator may not hand out again before the side stream has read it). Entries whose event has
        completed are dropped on the way (host-side query, no synchronisation); ``join_side`` drops the rest once
        the compute stream is ordered after the side stream."""
        ev = torch.cuda.Event()
        ev.record(self._side)
        held = self._held
        while held and held[0][0].query():
            held.pop(0)
        held.append((ev, tuple(tensors)))

    def side_submit(self, launch, inputs, ready=()) -> None:
        """Queue ``launch()`` for the weight-gradient stream; ``inputs`` are the tensors it reads, ``ready`` the
        parameters whose gradients it completes (marked ready once it is issued). Issued in groups of
        ``side_batch``, and by ``flush_side``: every caller flushes before anything that depends on the queued
        launches having been issued (deferred launches, the end of backward, the join)."""
        self._side_q.append((launch, tuple(inputs), tuple(ready)))
        if not self._flush_at_end:
            # whatever the caller: the last group goes out when the backward pass that queued it ends
            try:
                torch.autograd.Variable._execution_engine.queue_callback(self._end_of_backward)
                self._flush_at_end = True
            except RuntimeError:  # not inside a backward pass: the caller flushes
                pass
        if len(self._side_q) >= self.side_batch:
            self.flush_side()

    def _end_of_backward(self) -> None:
        self._flush_at_end = False
        self.flush_side()

    def flush_side(self) -> None:
        """Issue the queued side-stream launches behind one fork from the compute stream: the side stream waits for
        everything queued on the compute stream so far (a superset of what each launch reads), runs them in queue
        order, and keeps their inputs referenced until it has passed them (``hold_side``)."""
        q, self._side_q = self._side_q, []
        if not q:
            return
        side = self.side_stream()
        side.wait_stream(torch.cuda.current_stream())
        # no_grad: a group flushed after backward has returned (the trainer, the next micro-batch) runs outside
        # autograd's own no-grad context, and its GEMMs write into out= buffers from saved tensors that require grad
        with torch.cuda.stream(side), torch.no_grad():
            for launch, _, _ in q:
                launch()
        ins = [t for _, inputs, _ in q for t in inputs]
        if _RECORD_STREAM:
            for t in ins:
                t.record_stream(side)
        self.hold_side(ins)
        for _, _, ready in q:
            for p in ready:
                self.hooks.ready(p)

    def defer(self, launch) -> None:
        """Queue a side-stream gradient launch for ``run_deferred`` (ops.functional._sink(defer=True)).

        ``_sink`` marks the parameter ready BEFORE the deferred launch writes its gradient, which is only sound while
        no bucket collective fires on readiness this micro-batch (data parallelism reduces buckets on the last
        micro-batch only, where the trainer turns ``defer_ok`` off). Enforced here, not assumed."""
        if self.collectives_live():
            raise RuntimeError("weight-gradient launch deferred while bucket collectives are live: a bucket would be "
                               "reduced before its deferred gradient is written (defer_ok must be off on the "
                               "micro-batch whose backward reduces)")
        self.flush_side()  # side-stream launches keep their issue order (tied weights: overwrite before accumulate)
        self._deferred.append(launch)

    def run_deferred(self) -> None:
        """Issue the deferred side-stream gradient launches (the trainer calls this once the next micro-batch's forward
        is queued; ``join_side`` flushes whatever is left)."""
        self.flush_side()
        pending, self._deferred = self._deferred, []
        for launch in pending:
            launch()

    def join_side(self) -> None:
        """The compute stream waits for every weight gradient issued on the side stream (end of backward);
        from here on every compute-stream write is ordered after the side stream's reads."""
        self.run_deferred()
        if self._side is not None:
            torch.cuda.current_stream().wait_stream(self._side)
        self._held.clear()

    # forward gates ------------------------------------------------------------------------------
    def await_param(self, p) -> None:
        """Called before a kernel reads parameter ``p``: wait (on the current stream) for its bucket's gate."""
        b = self._bucket_of.get(id(p))
        if b is None:
            return
        if b.index not in self._used:
            self._used.add(b.index)
            self.use_order.append(b.index)
        g = self.gates.pop(b.index, None)
        if g is not None:
            self._resolve_timed(g)

    def set_gate(self, index: int, gate) -> None:
        self.gates[index] = gate

    def await_all(self) -> None:
        """Resolve every outstanding gate (before checkpointing, evaluation, or the next optimizer step)."""
        for i in list(self.gates):
            self._resolve_timed(self.gates.pop(i))

    def _resolve_timed(self, gate) -> None:
        """Resolve a gate; with ``gate_waits`` set (bench.py), a collective gate (ZeRO-1 all-gather) is bracketed by
        two timing events on the compute stream: their distance is the time the compute stream stalled on it."""
        if self.gate_waits is None or isinstance(gate, torch.cuda.Event):
            _resolve(gate)
            return
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _resolve(gate)
        e1.record()
        self.gate_waits.append((e0, e1))

    # transposed weight copies (data-gradient GEMMs) ----------------------------------------------
    def enable_transposed(self, min_width: int = 2048) -> int:
        """Keep a transposed bf16 copy ``p.wt`` ([in, out]) of every 2-D parameter whose both dims are
        >= ``min_width``, so the backward's dX = dY . W runs in the forward's K-contiguous GEMM layout
        (hipBLASLt: 1.28-1.60 vs 1.09-1.36 PF/s at Llama-3-8B shapes, tools/bench_dgrad_layouts.py). The
        copies share the flat layout of ``params`` (same offsets); they are refreshed per bucket right after
        the bucket's update lands (see ``refresh_transposed``). Returns the number of weights covered."""
        self.params_t = torch.zeros_like(self.params)
        self._t_names: dict[int, list[str]] = {}
        n = 0
        for name, p in self._param_by_name.items():
            if p.dim() == 2 and min(p.shape) >= min_width and p.shape[0] % 8 == 0 and p.shape[1] % 8 == 0:
                o = self.offsets[name]
                p.wt = self.params_t[o:o + p.numel()].view(p.shape[1], p.shape[0])
                self._t_names.setdefault(self._bucket_of[id(p)].index, []).append(name)
                n += 1
        return n

    @property
    def has_transposed(self) -> bool:
        return getattr(self, "params_t", None) is not None

    def refresh_transposed(self, bucket: int | None = None) -> None:
        """Re-derive the transposed copies of one bucket (or all) on the current stream (HIP transpose)."""
        if not self.has_transposed:
            return
        from ..ops.functional import transpose_into

        idx = self._t_names.keys() if bucket is None else [bucket]
        for b in idx:
            for name in self._t_names.get(b, ()):
                p = self._param_by_name[name]
                transpose_into(p.detach(), p.wt)

    # FP8 weight copies (forward / data-gradient GEMMs in E4M3, ops/fp8.py) ---------------------------
    def enable_fp8(self, names) -> int:
        """Keep E4M3 copies of the named 2-D weights -- ``p.w8`` ([out, in]) and, where the transposed bf16
        copy exists, ``p.wt8`` ([in, out]) -- with their dequantization scales, refreshed per bucket after
        every update (``refresh_fp8``). 1 byte per element and orientation (~15 GB at Llama-3-8B)."""
        from ..ops.fp8 import FP8

        self.params_fp8 = torch.empty(self.numel, dtype=FP8, device=self.device)
        self.params_t_fp8 = torch.empty(self.numel, dtype=FP8, device=self.device) if self.has_transposed else None
        self._fp8_names: dict[int, list[str]] = {}
        n = 0
        for name in names:
            p = self._param_by_name[name]
            if p.dim() != 2:
                continue
            o, k = self.offsets[name], p.numel()
            p.w8 = self.params_fp8[o:o + k].view(p.shape)
            p.w8_scale = torch.ones((), dtype=torch.float32, device=self.device)
            if self.params_t_fp8 is not None and getattr(p, "wt", None) is not None:
                p.wt8 = self.params_t_fp8[o:o + k].view(p.shape[1], p.shape[0])
                p.wt8_scale = torch.ones((), dtype=torch.float32, device=self.device)
            self._fp8_names.setdefault(self._bucket_of[id(p)].index, []).append(name)
            n += 1
        return n

    @property
    def has_fp8(self) -> bool:
        return getattr(self, "params_fp8", None) is not None

    def refresh_fp8(self, bucket: int | None = None) -> None:
        """Re-quantize one bucket's (or every) FP8 weight copy from the bf16 values, on the current stream."""
        if not self.has_fp8:
            return
        from ..ops.fp8 import quantize_into

        idx = self._fp8_names.keys() if bucket is None else [bucket]
        for b in idx:
            for name in self._fp8_names.get(b, ()):
                p = self._param_by_name[name]
                quantize_into(p.detach(), p.w8, p.w8_scale)
                if getattr(p, "wt8", None) is not None:
                    quantize_into(p.wt, p.wt8, p.wt8_scale)

    def zero_grads(self) -> None:
        self.grads.zero_()

    def regions(self):
        """[(start, end, decay)] of the two weight-decay regions."""
        out = []
        if self.decay_end > 0:
            out.append((0, self.decay_end, True))
        if self.numel > self.decay_end:
            out.append((self.decay_end, self.numel, False))
        return out

    def memory_bytes(self) -> int:
        return self.params.numel() * self.params.element_size() + self.grads.numel() * self.grads.element_size()
