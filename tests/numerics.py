"""Numerics checks shared by the GPU kernel tests.

A kernel result is compared with an fp32 reference of the same op AND with plain bf16 PyTorch run on the same
inputs, so a tolerance means "no worse than what the framework it replaces would give":

* ``rel_err``: max-abs error / max-abs reference (the whole tensor);
* ``row_errs``: per-row relative error ||x_i - ref_i|| / ||ref_i|| -- small-norm rows (early causal rows, GQA
  tails, rows the softmax nearly zeroes) are judged against their own scale, not the tensor's maximum;
* ``check_against_bf16``: the kernel's error must be <= ``factor`` x plain bf16's error against the same
  reference, on the whole tensor and on the ``frac`` smallest-norm rows (floor: ``floor``, about one bf16
  rounding, for outputs plain bf16 gets exactly right).
"""
from __future__ import annotations

import json
import os

import torch


def rel_err(a, b) -> float:
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def row_errs(a, ref, rows) -> torch.Tensor:
    a, ref = a.float()[rows], ref.float()[rows]
    return (a - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-12)


def smallest_rows(ref, frac=0.01, min_rows=16) -> torch.Tensor:
    n = ref.float().norm(dim=1)
    nz = torch.nonzero(n > 0).flatten()
    k = max(min_rows, int(frac * nz.numel()))
    return nz[torch.argsort(n[nz])[:k]]


def check_against_bf16(name, kernel, ref, plain_bf16, factor=2.0, floor=2.0 ** -9, frac=0.01) -> dict:
    """Assert the kernel is within ``factor`` x plain bf16's error (whole tensor and smallest-norm rows)."""
    k2, ref2, b2 = (t.reshape(t.shape[0], -1) for t in (kernel, ref, plain_bf16))
    ek, eb = rel_err(k2, ref2), rel_err(b2, ref2)
    rows = smallest_rows(ref2, frac)
    rk, rb = row_errs(k2, ref2, rows).max().item(), row_errs(b2, ref2, rows).max().item()
    out = {"name": name, "kernel": ek, "bf16": eb, "rows_kernel": rk, "rows_bf16": rb, "rows": int(rows.numel())}
    ev = os.environ.get("KOP_EVIDENCE_DIR")
    if ev:  # one JSON line per check, tagged with the running test (GPU sessions keep them as evidence)
        os.makedirs(ev, exist_ok=True)
        with open(os.path.join(ev, "numerics_vs_bf16.jsonl"), "a") as f:
            f.write(json.dumps({"test": os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0], **out}) + "\n")
    assert ek <= factor * eb + floor, out
    assert rk <= factor * rb + floor, out
    return out
