"""Library-GEMM selection for the training step (the plain projection GEMMs stay on hipBLASLt via
``torch.matmul``/``F.linear``; the fused hot ops are our HIP kernels).

hipBLASLt's default heuristic picks one solution per shape from a generic model; PyTorch's TunableOp can
instead time every candidate solution for the exact shapes of the model once and record the winners. The
winners for the bundled chart's shapes on gfx950 are committed under ``kubeoperator_amd/tuning/`` and loaded
read-only by default (no tuning inside a timed run); ``mode="tune"`` re-tunes new shapes and rewrites the
file (done once per toolchain / model shape on a real MI355X).
"""
from __future__ import annotations

import os

import torch

TUNING_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning")


def results_path(tag: str = "gfx950") -> str:
    return os.path.join(TUNING_DIR, f"tunableop_results_{tag}.csv")


def setup(mode: str = "use", path: str | None = None, rank: int = 0) -> str:
    """``off`` | ``use`` (load committed winners, never tune) | ``tune`` (tune unseen shapes, write back)."""
    if mode == "off" or not torch.cuda.is_available():
        return "off"
    tun = torch.cuda.tunable
    path = path or os.environ.get("KOP_GEMM_RESULTS") or results_path()
    if mode == "use" and not os.path.exists(path):
        return "off (no tuned results)"
    tun.enable(True)
    if mode == "use":
        # winners are only READ here. Some torch versions rewrite TunableOp's output file at process exit:
        # point that file at a per-rank scratch path so the ranks of a multi-GPU job (and back-to-back jobs
        # reading the committed winners) never race on or rewrite the shared results file
        import tempfile

        tun.set_filename(os.path.join(tempfile.gettempdir(), f"kop_tunableop_rank{rank}.csv"),
                         insert_device_ordinal=False)
    else:
        tun.set_filename(path, insert_device_ordinal=False)
    if mode == "tune":
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tun.tuning_enable(True)
        tun.set_max_tuning_duration(int(os.environ.get("KOP_TUNE_MS", "150")))
        tun.set_max_tuning_iterations(int(os.environ.get("KOP_TUNE_ITERS", "40")))
        tun.record_untuned_enable(False)
    else:
        tun.tuning_enable(False)
    if os.path.exists(path):
        tun.read_file(path)
    return f"{mode} ({path})"


def finish(mode: str, rank: int = 0) -> None:
    """Tuned results are written to the results file by TunableOp itself when the process exits."""
    return None
