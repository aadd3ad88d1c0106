"""Fused AdamW over flat (segmented) parameter storage.

The optimizer does not see ``nn.Parameter`` objects: it is handed *segments* -- pairs of equally sized
views into the flat bf16 parameter buffer and the flat bf16 gradient buffer, each with its weight decay --
and keeps fp32 master weights, exp_avg and exp_avg_sq for all segments in three contiguous fp32 buffers.
One ``adamw_`` kernel launch per segment (a handful per step: one per weight-decay region, or one per
ZeRO-1 bucket shard). Gradient clipping is computed on device (sum of squares -> clip coefficient) and fed
to the kernel as a device scalar, so a step never synchronises with the host.

Overlap (``store`` given, GPU): the update runs on the optimizer's own HIP stream, one launch per bucket
in the order the next forward pass reads the buckets (``FlatParamStore.use_order``), and each launch
publishes a gate for its bucket (an event, or what ``on_segment`` returns -- the ZeRO-1 all-gather work).
The forward kernels wait only for the gate of the bucket they read, so the HBM-bound AdamW (~28 B/param)
runs underneath the next step's compute-bound forward instead of in its own serial phase.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import torch

# race-detection hook: GPU clock cycles of ``torch.cuda._sleep`` enqueued on the optimizer stream before every
# bucket's update, so the stream deterministically lags the compute stream; a forward that read a bucket without
# waiting for its gate, or a backward that overwrote gradients AdamW still reads, then changes the result
# (tests/test_stream_lag_gpu.py; ops.functional.SIDE_LAG_CYCLES is the weight-gradient stream's twin)
OPTIM_LAG_CYCLES = int(os.environ.get("KOP_OPTIM_LAG_CYCLES", "0"))


@dataclass
class Segment:
    param: torch.Tensor  # bf16 view (flat)
    grad: torch.Tensor   # bf16 view (flat), same numel
    weight_decay: float
    bucket: int = -1     # flat-store bucket this segment belongs to (for overlap gates)
    norm_weight: float = 1.0  # weight of its sum of squares in the global grad norm (1/tp: TP-replicated)


class FusedAdamW:
    def __init__(self, segments: list[Segment], lr: float = 3e-4, betas=(0.9, 0.95), eps: float = 1e-8,
                 weight_decay: float = 0.1, max_grad_norm: float = 1.0, grad_scale: float = 1.0,
                 norm_allreduce=None, store=None, on_segment=None):
        # a segment's weight_decay of None means "the optimizer's default"
        for sg in segments:
            if sg.weight_decay is None:
                sg.weight_decay = weight_decay
        self.segments = segments
        self.lr = lr
        self.b1, self.b2 = betas
        self.eps = eps
        self.default_wd = weight_decay
        self.max_grad_norm = max_grad_norm
        self.grad_scale = grad_scale
        self.norm_allreduce = norm_allreduce  # callable(tensor) summing a device scalar across shards
        self.step_count = 0
        n = sum(s.param.numel() for s in segments)
        dev = segments[0].param.device if segments else torch.device("cpu")
        self.master = torch.empty(n, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self._views = []
        off = 0
        for s in segments:
            k = s.param.numel()
            self.master[off:off + k].copy_(s.param.reshape(-1).float())
            self._views.append((off, off + k))
            off += k
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self._sumsq_w = torch.zeros(1, dtype=torch.float32, device=dev)  # segments with norm_weight != 1
        self._norm_w = {s.norm_weight for s in segments if s.norm_weight != 1.0}
        if len(self._norm_w) > 1:
            raise ValueError("one replicated-segment norm weight per optimizer")
        self._coef = torch.ones(1, dtype=torch.float32, device=dev)
        self.last_grad_norm = torch.zeros(1, dtype=torch.float32, device=dev)
        self.store = store
        self.on_segment = on_segment  # callable(Segment) -> gate or None, runs on the optimizer stream
        self.overlap = store is not None and dev.type == "cuda" and all(sg.bucket >= 0 for sg in segments)
        self._stream = torch.cuda.Stream(device=dev) if self.overlap else None

    # -------------------------------------------------------------------------------------------
    def state_bytes(self) -> int:
        return self.master.numel() * 4 * 3

    def _native(self) -> bool:
        return self.master.is_cuda

    def clip(self):
        """Compute the global grad norm and the clip coefficient on device (no host sync)."""
        if self.max_grad_norm is None or self.max_grad_norm <= 0:
            self._coef.fill_(1.0)
            return
        self._sumsq.zero_()
        if self._norm_w:
            self._sumsq_w.zero_()
        if self._native():
            from . import load

            lib = load()
            for s in self.segments:
                if s.grad.numel():
                    lib.grad_sumsq_(s.grad.reshape(-1), self._sumsq if s.norm_weight == 1.0 else self._sumsq_w)
        else:
            for s in self.segments:
                acc = self._sumsq if s.norm_weight == 1.0 else self._sumsq_w
                acc += s.grad.float().pow(2).sum()
        if self._norm_w:  # TP-replicated gradients: every TP rank holds a copy, counted once after the sum
            self._sumsq.add_(self._sumsq_w, alpha=next(iter(self._norm_w)))
        if self.grad_scale != 1.0:
            self._sumsq.mul_(self.grad_scale * self.grad_scale)
        if self.norm_allreduce is not None:
            self.norm_allreduce(self._sumsq)
        if self._native():
            from . import load

            load().clip_coef_(self._sumsq, float(self.max_grad_norm), self._coef, self.last_grad_norm)
        else:
            nrm = self._sumsq.sqrt()
            self.last_grad_norm.copy_(nrm)
            self._coef.copy_(torch.clamp(self.max_grad_norm / (nrm + 1e-6), max=1.0))

    def _launch_order(self) -> list[int]:
        pos = {b: i for i, b in enumerate(self.store.use_order)}
        return sorted(range(len(self.segments)), key=lambda k: (pos.get(self.segments[k].bucket, 1 << 30), k))

    def step(self, lr: float | None = None):
        lr = self.lr if lr is None else lr
        self.step_count += 1
        if self.store is not None:
            self.store.await_all()
        self.clip()
        if self._native():
            from . import load

            lib = load()

            def launch(k):
                s, (a, b) = self.segments[k], self._views[k]
                if b > a:
                    lib.adamw_(s.param.reshape(-1), s.grad.reshape(-1), self.master[a:b], self.exp_avg[a:b],
                               self.exp_avg_sq[a:b], lr, self.b1, self.b2, self.eps, s.weight_decay,
                               self.step_count, self.grad_scale, self._coef)

            if not self.overlap:
                for k in range(len(self.segments)):
                    launch(k)
                return
            self._stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self._stream):
                for k in self._launch_order():
                    if OPTIM_LAG_CYCLES > 0:
                        torch.cuda._sleep(OPTIM_LAG_CYCLES)
                    launch(k)
                    b = self.segments[k].bucket
                    gate = self.on_segment(self.segments[k]) if self.on_segment is not None else None
                    if self.store.has_transposed or self.store.has_fp8:
                        # the transposed / FP8 copies follow the bucket's final values (after the ZeRO-1 gather)
                        if gate is not None:
                            gate.wait()  # optimizer stream waits for the collective
                        self.store.refresh_transposed(b)
                        self.store.refresh_fp8(b)
                        gate = None
                    if gate is None:
                        gate = torch.cuda.Event()
                        gate.record(self._stream)
                    self.store.set_gate(b, gate)
        else:
            t = self.step_count
            bc1 = 1 - self.b1 ** t
            bc2 = 1 - self.b2 ** t
            for s, (a, b) in zip(self.segments, self._views):
                g = s.grad.reshape(-1).float() * self.grad_scale * self._coef
                m, v, w = self.exp_avg[a:b], self.exp_avg_sq[a:b], self.master[a:b]
                m.mul_(self.b1).add_(g, alpha=1 - self.b1)
                v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
                w.mul_(1 - lr * s.weight_decay)
                w.sub_(lr * (m / bc1) / (v.sqrt() / math.sqrt(bc2) + self.eps))
                s.param.reshape(-1).copy_(w)

    def sync_master(self) -> None:
        """Re-derive the fp32 master weights from the bf16 parameters (after parameters were loaded)."""
        for s, (a, b) in zip(self.segments, self._views):
            self.master[a:b].copy_(s.param.reshape(-1).float())

    # checkpointing -------------------------------------------------------------------------------
    def state_dict(self):
        if self.store is not None:
            self.store.await_all()
        return {"step": self.step_count, "master": self.master, "exp_avg": self.exp_avg,
                "exp_avg_sq": self.exp_avg_sq, "lr": self.lr}

    def load_state_dict(self, sd):
        if self.store is not None:
            self.store.await_all()
        self.step_count = int(sd["step"])
        self.master.copy_(sd["master"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        for s, (a, b) in zip(self.segments, self._views):
            s.param.reshape(-1).copy_(self.master[a:b])
