"""Checkpoint / resume for the training chart.

Layout: ``<dir>/step_<N>/rank_<R>.pt`` (one file per rank: ZeRO-1 optimizer shards are per rank; DDP
ranks hold identical state but each writes its own file so resume never needs cross-rank traffic) plus
``<dir>/latest`` containing the newest complete step. A step directory becomes "latest" only after every
rank has written (rank 0 writes the marker after a barrier), so a crash mid-save resumes from the
previous complete checkpoint. Files are written to a temp name and renamed (atomic on POSIX).
Loading uses ``torch.load(weights_only=True)``: checkpoints are tensors + plain containers only.

Elastic resume: a job restarted on a different number of GPUs (a node lost GPUs, or more were added) loads
a checkpoint written at another world size. Every file carries its flat layout (parameter offsets, and
where each optimizer-state segment sits); the loader memory-maps the old ranks' files and copies, per
parameter, the intersection of the old pieces with this rank's new segments -- each rank reads only its own
new shard of the fp32 state (12 B/param / world), never the whole 96 GB of an 8B model.

Tensor parallelism: TP rank t of T keeps its own tree ``<dir>/tp<t>_of<T>/`` written by its data-parallel
group (the shards differ per TP rank); resuming needs the same TP degree, the DP size may change (the
reshard above runs inside each TP rank's tree). A resume takes the newest step complete in EVERY tree.
"""
from __future__ import annotations

import bisect
import os

import torch

from ..parallel.dist import DistInfo, barrier


def _tp_view(trainer, directory: str, info: DistInfo):
    """(directory, data-parallel info) of this rank's checkpoint tree."""
    tp = getattr(trainer, "tp", None)
    if tp is None or not tp.enabled:
        return directory, info
    return os.path.join(directory, f"tp{tp.rank}_of{tp.size}"), trainer.dp_info


def save(trainer, directory: str, info: DistInfo) -> str:
    job = info
    directory, info = _tp_view(trainer, directory, info)
    os.makedirs(directory, exist_ok=True)
    step = trainer.step
    d = os.path.join(directory, f"step_{step}")
    os.makedirs(d, exist_ok=True)
    sd = trainer.state_dict()
    sd["rng_cpu"] = torch.get_rng_state()
    path = os.path.join(d, f"rank_{info.rank}.pt")
    tmp = path + ".tmp"
    torch.save(sd, tmp)
    os.replace(tmp, path)
    barrier(info)
    if info.is_main:
        # a step directory may hold files of an earlier, crashed attempt at a larger world size (same step number,
        # another trajectory): drop every rank file past this world before the step becomes "latest"
        for f in os.listdir(d):
            if f.startswith("rank_") and f.endswith(".pt") and int(f[5:-3]) >= info.world:
                os.remove(os.path.join(d, f))
        with open(os.path.join(directory, "latest.tmp"), "w") as f:
            f.write(str(step))
        os.replace(os.path.join(directory, "latest.tmp"), os.path.join(directory, "latest"))
    barrier(job)
    return d


def latest_step(directory: str):
    p = os.path.join(directory, "latest")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return int(f.read().strip())


def _files(d: str, world: int) -> list[str]:
    """The rank files of a step written at ``world`` ranks: exactly rank_0 .. rank_{world-1}."""
    paths = [os.path.join(d, f"rank_{r}.pt") for r in range(world)]
    missing = [p for p in paths if not os.path.exists(p)]
    if missing:
        raise ValueError(f"incomplete checkpoint {d}: missing {[os.path.basename(p) for p in missing]}")
    return paths


def load(trainer, directory: str, info: DistInfo, step: int | None = None) -> int | None:
    job = info
    directory, info = _tp_view(trainer, directory, info)
    if step is None:
        step = latest_step(directory)
        if info is not job:  # TP: the newest step every TP rank's tree completed
            import torch.distributed as dist

            t = torch.tensor([-1 if step is None else step], dtype=torch.int64,
                             device=job.device if job.backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            step = None if int(t) < 0 else int(t)
    if step is None:
        return None
    d = os.path.join(directory, f"step_{step}")
    head = torch.load(os.path.join(d, "rank_0.pt"), map_location="cpu", weights_only=True, mmap=True)
    files = _files(d, int(head["world"]))
    own = os.path.join(d, f"rank_{info.rank}.pt")
    if info.rank >= int(head["world"]):
        own = files[0]  # a rank the writing job did not have: reshards from the others
    if getattr(getattr(trainer, "tp", None), "seq_parallel", False) and head["world"] != info.world:
        raise ValueError("a sequence-parallel checkpoint resumes on the topology that wrote it")
    if "layout" in head:  # identical flat layout (world size AND bucket boundaries): plain copy
        lay = trainer.layout()
        same = (head["world"] == info.world and head["layout"]["offsets"] == lay["offsets"]
                and head["layout"]["names"] == lay["names"]
                and [tuple(p) for p in head["layout"]["pieces"]] == [tuple(p) for p in lay["pieces"]])
        # (pieces differ per rank under ZeRO-1: compare this rank's own file then)
        if same is False and head["world"] == info.world and os.path.exists(own):
            mine = torch.load(own, map_location="cpu", weights_only=True, mmap=True)
            same = (mine["layout"]["offsets"] == lay["offsets"] and mine["layout"]["names"] == lay["names"]
                    and [tuple(p) for p in mine["layout"]["pieces"]] == [tuple(p) for p in lay["pieces"]])
    else:
        same = head["world"] == info.world and head["params"].numel() == trainer.store.params.numel()
    if same:
        sd = torch.load(own, map_location=info.device, weights_only=True)
        trainer.load_state_dict(sd)
    else:
        _reshard(trainer, head, files)
        sd = torch.load(own, map_location="cpu", weights_only=True, mmap=True) if os.path.exists(own) else head
    if "rng_cpu" in sd:
        torch.set_rng_state(sd["rng_cpu"].cpu())
    return step


def _intersect(a0, a1, b0, b1):
    lo, hi = max(a0, b0), min(a1, b1)
    return (lo, hi) if lo < hi else None


@torch.no_grad()
def _reshard(trainer, head: dict, files: list[str]) -> None:
    """Load a checkpoint written at another world size into this rank's layout."""
    if "layout" not in head:
        raise ValueError("checkpoint predates layout metadata: resume with the world size that wrote it")
    st, opt = trainer.store, trainer.opt
    st.await_all()
    old = head["layout"]
    old_at = {n: (o, k) for n, o, k in zip(old["names"], old["offsets"], old["numels"])}
    new = trainer.layout()
    missing = set(new["names"]) - set(old_at)
    if missing:
        raise ValueError(f"checkpoint lacks parameters {sorted(missing)[:5]}")
    # parameters: replicated, taken from the first file
    for name, p in st.named_params():
        o, k = old_at[name]
        p.data.view(-1).copy_(head["params"][o:o + k].to(p.device))
    # optimizer state: old pieces (any rank's file) -> this rank's segments, per parameter
    params = [(st.offsets[n], old_at[n][0], old_at[n][1]) for n in new["names"]]  # (new off, old off, numel)
    for buf in ("master", "exp_avg", "exp_avg_sq"):
        getattr(opt, buf).zero_()
    new_p = sorted(new["pieces"])
    new_starts = [x[0] for x in new_p]
    for f in files:
        sd = head if f == files[0] else torch.load(f, map_location="cpu", weights_only=True, mmap=True)
        if int(sd["world"]) != int(head["world"]) or int(sd["step"]) != int(head["step"]):
            raise ValueError(f"{f} belongs to another save (world {sd['world']}, step {sd['step']}) than rank_0's "
                             f"(world {head['world']}, step {head['step']})")
        osd = sd["optimizer"]
        old_p = sorted(sd["layout"]["pieces"])
        old_starts = [x[0] for x in old_p]
        for (noff, ooff, k) in params:
            # pieces overlapping the parameter in each layout (pieces are disjoint, sorted by start)
            olds = old_p[max(0, bisect.bisect_right(old_starts, ooff) - 1):bisect.bisect_left(old_starts, ooff + k)]
            news = new_p[max(0, bisect.bisect_right(new_starts, noff) - 1):bisect.bisect_left(new_starts, noff + k)]
            for (oa, oe, om) in olds:
                a = _intersect(ooff, ooff + k, oa, oe)  # param indices held by this old piece (old coords)
                if a is None:
                    continue
                for (na, ne, nm) in news:
                    b = _intersect(noff, noff + k, na, ne)  # param indices this new segment needs
                    if b is None:
                        continue
                    c = _intersect(a[0] - ooff, a[1] - ooff, b[0] - noff, b[1] - noff)
                    if c is None:
                        continue
                    src = om + (ooff + c[0] - oa)
                    dst = nm + (noff + c[0] - na)
                    n = c[1] - c[0]
                    for buf in ("master", "exp_avg", "exp_avg_sq"):
                        getattr(opt, buf)[dst:dst + n].copy_(osd[buf][src:src + n])
        if f != files[0]:
            del sd
    opt.step_count = int(head["optimizer"]["step"])
    # bf16 parameters follow the fp32 masters of this rank's segments (identical values: they were rounded
    # from the same masters), and the transposed weight copies follow the parameters
    st.refresh_transposed()
    st.refresh_fp8()
    trainer.step = int(head["step"])
