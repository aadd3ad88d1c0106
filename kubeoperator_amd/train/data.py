"""Token data sources for the training chart.

* :class:`SyntheticTokens` -- the benchmark source: uniformly random token ids generated ON DEVICE
  (per-rank seed, no host->device copy in the step), targets = ids shifted by one. Matches the shape of
  real pre-training batches; the benchmark reports ``"data": "synthetic"``.
* :class:`TokenFileDataset` -- memory-mapped flat token file (uint16/uint32), random windows per rank,
  loaded by the native prefetcher in ``kubeoperator_amd/native`` when available (pinned host buffers +
  async copy), else by numpy.
"""
from __future__ import annotations

import os

import numpy as np
import torch


class SyntheticTokens:
    def __init__(self, vocab_size: int, micro_batch: int, seq_len: int, device, seed: int = 0, rank: int = 0):
        self.V = vocab_size
        self.B = micro_batch
        self.S = seq_len
        self.device = torch.device(device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed * 1000003 + rank)

    def next(self):
        buf = torch.randint(0, self.V, (self.B, self.S + 1), device=self.device, generator=self.gen)
        return buf[:, :-1].contiguous(), buf[:, 1:].contiguous()

    def batches(self, n: int):
        return [self.next() for _ in range(n)]


_M64 = (1 << 64) - 1


def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def window_starts(seed: int, index: int, batch: int, ntok: int, window: int) -> list[int]:
    """Start offsets of batch ``index`` -- the same function the native prefetcher computes."""
    span = ntok - window + 1
    return [_splitmix64((seed & _M64) ^ _splitmix64((index * 0x100000001B3 + r) & _M64)) % span for r in range(batch)]


class TokenFileDataset:
    """Random ``seq_len + 1`` windows of a flat token file; batch ``i`` of rank ``r`` is a pure function of
    (seed, r, i), so resuming at step ``k`` continues the exact stream (``start_batch = k * grad_accum``)."""

    def __init__(self, path: str, micro_batch: int, seq_len: int, device, dtype=np.uint16, seed: int = 0,
                 rank: int = 0, world: int = 1, start_batch: int = 0, native: bool = True):
        self.path = path
        self.tokens = np.memmap(path, dtype=dtype, mode="r")
        if len(self.tokens) < seq_len + 2:
            raise ValueError(f"{path}: only {len(self.tokens)} tokens, need > {seq_len + 1}")
        self.B, self.S = micro_batch, seq_len
        self.device = torch.device(device)
        self.seed = seed * 1000003 + rank
        self.rank, self.world = rank, world
        self.index = start_batch
        self._native = None
        if native:
            try:
                from ..native import prefetch  # type: ignore

                self._native = prefetch.TokenPrefetcher(path, np.dtype(dtype).itemsize, micro_batch, seq_len + 1,
                                                        self.seed, depth=8, threads=4)
                if start_batch:
                    self._native.skip(start_batch)
            except ImportError:
                self._native = None

    def next(self):
        if self._native is not None:
            arr = self._native.next()
        else:
            starts = window_starts(self.seed, self.index, self.B, len(self.tokens), self.S + 1)
            arr = np.stack([np.asarray(self.tokens[s:s + self.S + 1], dtype=np.int64) for s in starts])
        self.index += 1
        t = torch.from_numpy(arr)
        if self.device.type == "cuda":
            t = t.pin_memory().to(self.device, non_blocking=True)
        return t[:, :-1].contiguous(), t[:, 1:].contiguous()

    def batches(self, n: int):
        return [self.next() for _ in range(n)]


def write_token_file(path: str, tokens, dtype=np.uint16) -> str:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    np.asarray(tokens, dtype=dtype).tofile(path)
    return path
