"""Trainer of the bundled PyTorch-ROCm chart: model on the flat bucketed store, RCCL data parallelism,
fused AdamW with on-device clipping, warmup + cosine LR, gradient accumulation, checkpoint/resume.

A training step never synchronises with the host: the loss is returned as a device tensor and only read
when logging.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import asdict, dataclass, field

import torch

from ..models import build_model, get_config
from ..ops.optim import FusedAdamW
from ..parallel.ddp import DataParallel
from ..parallel.dist import DistInfo
from ..parallel.flat import FlatParamStore
from ..parallel.tensor import check_llama_tp, make_groups


@dataclass
class TrainConfig:
    model: str = "llama3_8b"
    micro_batch: int = 1
    seq_len: int = 8192
    grad_accum: int = 1
    lr: float = 3e-4
    min_lr: float = 3e-5
    warmup_steps: int = 100
    total_steps: int = 10000
    weight_decay: float = 0.1
    betas: tuple = (0.9, 0.95)
    eps: float = 1e-8
    grad_clip: float = 1.0
    dp_mode: str = "allreduce"  # allreduce | zero1
    bucket_mb: int = 512
    overlap_optimizer: bool = True  # AdamW on its own stream, gated per bucket into the next forward
    transposed_weights: bool = True  # keep W^T copies of wide weights for the dX GEMMs (GPU only)
    cuda_graph: bool = False  # replay each micro-batch's forward + backward as a captured HIP graph (1 GPU)
    grad_dtype: str = "bf16"  # bf16 | fp32: gradient buffer (micro-batch accumulation + DP reduction) precision
    fp8: bool = False  # E4M3 forward + data-gradient GEMMs of the block projections (ops/fp8.py; opt-in)
    recompute: bool = False  # per-block activation recompute (long sequences: only block inputs stay saved)
    # weight-gradient GEMMs on a side stream: auto (narrow models, hidden < 2048) | on | off
    wgrad_stream: str = "auto"
    tp: int = 1  # tensor-parallel degree (Llama; TP groups of consecutive ranks, DP across them: parallel.tensor)
    sp: bool = False  # sequence parallelism on top of TP (norms, residual stream, LM head on 1/tp of the rows)
    seed: int = 1234
    model_overrides: dict = field(default_factory=dict)

    def to_dict(self):
        return asdict(self)


def lr_at(step: int, tc: TrainConfig) -> float:
    if step < tc.warmup_steps:
        return tc.lr * (step + 1) / tc.warmup_steps
    p = min(1.0, (step - tc.warmup_steps) / max(1, tc.total_steps - tc.warmup_steps))
    return tc.min_lr + 0.5 * (tc.lr - tc.min_lr) * (1 + math.cos(math.pi * p))


class Trainer:
    def __init__(self, tc: TrainConfig, info: DistInfo):
        self.tc = tc
        self.info = info
        # data-parallel view of this rank + its tensor-parallel group (the whole job and no TP when tp == 1)
        check_llama_tp(get_config(tc.model, **tc.model_overrides), tc.tp)
        self.dp_info, self.tp = make_groups(info, tc.tp, tc.sp)
        overrides = dict(tc.model_overrides)
        base = get_config(tc.model)
        if tc.seq_len > base.max_seq_len and base.arch == "llama" and "max_seq_len" not in overrides:
            overrides["max_seq_len"] = tc.seq_len  # RoPE: the context length is a limit, not a weight shape
        self.cfg = get_config(tc.model, **overrides)
        if tc.seq_len > self.cfg.max_seq_len:
            raise ValueError(f"seq_len {tc.seq_len} > model max_seq_len {self.cfg.max_seq_len} "
                             "(learned positions cannot be extended)")
        dev = info.device
        t0 = time.time()
        with torch.device("meta"):
            self.model = build_model(self.cfg, self.tp)
        self.model.recompute = bool(tc.recompute)
        if tc.grad_dtype not in ("bf16", "fp32"):
            raise ValueError(f"grad_dtype must be bf16 or fp32, not {tc.grad_dtype!r}")
        # SP reduces replicated buckets over the whole job: their ZeRO-1 pieces split over every rank
        self.store = FlatParamStore(self.model, self.model.param_specs(), dev,
                                    world=info.world if self.tp.seq_parallel else self.dp_info.world,
                                    bucket_bytes=tc.bucket_mb * 1024 * 1024,
                                    grad_dtype=torch.float32 if tc.grad_dtype == "fp32" else torch.bfloat16)
        self.store.init_weights(seed=tc.seed, shard_rank=self.tp.rank)
        self.dp = DataParallel(self.store, self.dp_info, tc.dp_mode, self.tp)
        self.dp.broadcast_params()
        if tc.transposed_weights and dev.type == "cuda":
            self.store.enable_transposed()
            self.store.refresh_transposed()
        if tc.fp8:
            if dev.type != "cuda" or self.cfg.arch != "llama":
                raise ValueError("fp8 GEMMs need a GPU and a Llama model")
            self.store.enable_fp8(self.model.fp8_param_names())
            self.store.refresh_fp8()
        if tc.wgrad_stream not in ("auto", "on", "off"):
            raise ValueError(f"wgrad_stream must be auto, on or off, not {tc.wgrad_stream!r}")
        env = os.environ.get("KOP_WGRAD_STREAM")
        want = (tc.wgrad_stream == "on" or (tc.wgrad_stream == "auto" and self.cfg.hidden < 2048)) \
            if env not in ("0", "1") else env == "1"
        # multi-rank jobs included: the 2-4 rank data- / tensor-parallel rehearsals on one MI355X with the side stream
        # forced to lag match one process to bf16 reduction noise (profiles/r3_wgrad_multirank_rehearsal.jsonl)
        self.store.wgrad_stream = dev.type == "cuda" and not tc.cuda_graph and want
        self.opt = FusedAdamW(self.dp.optimizer_segments(), lr=tc.lr, betas=tc.betas, eps=tc.eps,
                              weight_decay=tc.weight_decay, max_grad_norm=tc.grad_clip,
                              grad_scale=self.dp.grad_scale / tc.grad_accum, norm_allreduce=self.dp.norm_allreduce(),
                              store=self.store if tc.overlap_optimizer else None,
                              on_segment=self.dp.publish_segment)
        self.step = 0
        if tc.cuda_graph and (dev.type != "cuda" or info.world != 1):
            raise ValueError("cuda_graph needs one GPU rank (collectives are not captured)")
        self._graphs: dict = {}
        self._graph_loss: dict = {}
        self._graph_pool = None
        self._static = None
        self.setup_seconds = time.time() - t0

    @property
    def tokens_per_step(self) -> int:
        """Tokens processed per optimizer step by THIS rank (its TP group shares them)."""
        return self.tc.micro_batch * self.tc.seq_len * self.tc.grad_accum

    @property
    def job_tokens_per_step(self) -> int:
        """Tokens per optimizer step of the whole job: one micro-batch stream per data-parallel rank."""
        return self.dp_info.world * self.tokens_per_step

    def train_step(self, batches) -> torch.Tensor:
        """``batches``: iterable of ``grad_accum`` (ids, targets) pairs, each [micro_batch, seq_len]."""
        losses = []
        n = self.tc.grad_accum
        graphed = self.tc.cuda_graph and self.step > 0  # step 0 runs eagerly: lazy library / workspace init
        if graphed:
            # the captured micro-batch reads no forward gate: join the optimizer stream once instead
            self.store.await_all()
        for i, (ids, tgt) in enumerate(batches):
            self.store.begin_microbatch(i)
            self.dp.sync = i == n - 1
            if graphed:
                losses.append(self._replay(min(i, 1), ids, tgt))
                continue
            # a gradient launch deferred by the previous micro-batch's backward (_sink(defer=True)) goes out now,
            # behind this micro-batch's queued forward; none is deferred out of the last micro-batch
            self.store.defer_ok = i < n - 1
            loss = self.model(ids, tgt)
            self.store.run_deferred()
            loss.backward()
            self.store.flush_side()  # the last queued weight-gradient launches of this backward
            losses.append(loss.detach())
        self.store.join_side()
        self.dp.finish_grads()
        self.opt.step(lr_at(self.step, self.tc))
        self.dp.after_step()
        if (self.store.has_transposed or self.store.has_fp8) and not self.opt.overlap:
            self.store.refresh_transposed()
            self.store.refresh_fp8()
        self.step += 1
        loss = torch.stack(losses).mean()
        if self.tp.seq_parallel:  # each TP rank's loss covers its 1/tp of the rows
            import torch.distributed as dist

            dist.all_reduce(loss, group=self.tp.group)
            loss = loss / self.tp.size
        return loss

    # HIP graphs -----------------------------------------------------------------------------------
    def _replay(self, key: int, ids, tgt) -> torch.Tensor:
        """Forward + backward of one micro-batch as a captured HIP graph (``torch.cuda.CUDAGraph`` is a
        hipGraph on ROCm): one launch for the ~40 kernels per layer, so small micro-batches stop being bound
        by host-side launch and autograd overhead. Two graphs: ``key`` 0 overwrites the flat gradient buffer
        (first micro-batch), ``key`` 1 accumulates into it. Inputs are copied into static buffers; the loss
        is the graph's static output. Both graphs share one memory pool (they never run concurrently)."""
        if self._static is None:
            self._static = (torch.empty_like(ids), torch.empty_like(tgt))
        if key not in self._graphs:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self._graph_pool):
                loss = self.model(*self._static)
                loss.backward()
            self._graph_pool = g.pool()
            self._graphs[key] = g
            self._graph_loss[key] = loss.detach()
        self._static[0].copy_(ids)
        self._static[1].copy_(tgt)
        self._graphs[key].replay()
        return self._graph_loss[key].clone()

    def load_full_weights(self, full: dict) -> None:
        """Load unsharded (tp = 1) weights by name: each TP rank keeps its slice (``parallel.tensor``). The
        fp32 masters and the derived weight copies follow. Weight conversion into a TP job, and the TP tests."""
        from ..parallel.tensor import shard_llama_weight

        self.store.await_all()
        with torch.no_grad():
            for name, p in self.store.named_params():
                w = shard_llama_weight(name, full[name], self.cfg, self.tp.size, self.tp.rank)
                p.copy_(w.to(device=p.device, dtype=p.dtype))
        self.opt.sync_master()
        self.store.refresh_transposed()
        self.store.refresh_fp8()

    # checkpoint -----------------------------------------------------------------------------------
    def layout(self) -> dict:
        """Where every parameter and every optimizer-state segment lives in the flat buffers (they depend on
        the world size through bucket padding): what checkpoint resharding maps through."""
        st = self.store
        names = [n for n, _ in st.named_params()]
        base, es = st.params.data_ptr(), st.params.element_size()
        pieces = [((sg.param.data_ptr() - base) // es, (sg.param.data_ptr() - base) // es + (b - a), a)
                  for sg, (a, b) in zip(self.opt.segments, self.opt._views)]
        return {"names": names, "offsets": [st.offsets[n] for n in names],
                "numels": [st.param(n).numel() for n in names], "numel": st.numel, "pieces": pieces}

    def state_dict(self):
        self.store.await_all()
        return {"step": self.step, "train_config": self.tc.to_dict(), "model_config": self.cfg.to_dict(),
                "params": self.store.params, "optimizer": self.opt.state_dict(), "world": self.dp_info.world,
                "rank": self.dp_info.rank, "dp_mode": self.tc.dp_mode, "layout": self.layout(),
                "tp": self.tp.size, "tp_rank": self.tp.rank}

    def load_state_dict(self, sd):
        """Same world size and layout: direct copy. (Other world sizes: ``checkpoint.load`` reshards.)"""
        if sd.get("tp", 1) != self.tp.size or sd.get("tp_rank", 0) != self.tp.rank:
            raise ValueError("checkpoint was written with another tensor-parallel layout")
        if sd["world"] != self.dp_info.world or sd["params"].numel() != self.store.params.numel():
            raise ValueError("checkpoint layout differs from this run's: load it through checkpoint.load")
        self.store.await_all()
        self.store.params.copy_(sd["params"])
        self.opt.load_state_dict(sd["optimizer"])
        self.store.refresh_transposed()
        self.store.refresh_fp8()
        self.step = int(sd["step"])
