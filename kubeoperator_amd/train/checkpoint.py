"""Checkpoint / resume for the training chart.

Layout: ``<dir>/step_<N>/rank_<R>.pt`` (one file per rank: ZeRO-1 optimizer shards are per rank; DDP
ranks hold identical state but each writes its own file so resume never needs cross-rank traffic) plus
``<dir>/latest`` containing the newest complete step. A step directory becomes "latest" only after every
rank has written (rank 0 writes the marker after a barrier), so a crash mid-save resumes from the
previous complete checkpoint. Files are written to a temp name and renamed (atomic on POSIX).
Loading uses ``torch.load(weights_only=True)``: checkpoints are tensors + plain containers only.
"""
from __future__ import annotations

import os

import torch

from ..parallel.dist import DistInfo, barrier


def save(trainer, directory: str, info: DistInfo) -> str:
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
        with open(os.path.join(directory, "latest.tmp"), "w") as f:
            f.write(str(step))
        os.replace(os.path.join(directory, "latest.tmp"), os.path.join(directory, "latest"))
    barrier(info)
    return d


def latest_step(directory: str):
    p = os.path.join(directory, "latest")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return int(f.read().strip())


def load(trainer, directory: str, info: DistInfo, step: int | None = None) -> int | None:
    step = latest_step(directory) if step is None else step
    if step is None:
        return None
    path = os.path.join(directory, f"step_{step}", f"rank_{info.rank}.pt")
    sd = torch.load(path, map_location=info.device, weights_only=True)
    trainer.load_state_dict(sd)
    if "rng_cpu" in sd:
        torch.set_rng_state(sd["rng_cpu"].cpu())
    return step
