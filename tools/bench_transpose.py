"""Bandwidth of the HIP bf16 transpose at the shapes of a Llama-3-8B step (weight-gradient operands and
W^T refresh): the 64x128-tile kernel in row-tile order (the 64x64-tile and column-order forms it was measured against
in round 4 are no longer built).

usage: python tools/bench_transpose.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeoperator_amd.ops.functional import transpose_into  # noqa: E402

SHAPES = [(8192, 4096), (8192, 6144), (8192, 14336), (8192, 28672), (4096, 14336), (128256, 4096)]


def main():
    res = {"mode": "rows"}
    for R, C in SHAPES:
        x = torch.randn(R, C, device="cuda").to(torch.bfloat16)
        y = torch.empty(C, R, device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            transpose_into(x, y)
        assert torch.equal(y, x.t())
        n = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            transpose_into(x, y)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / n
        res[f"{R}x{C}"] = {"us": round(us, 1), "TB/s": round(4 * R * C / us / 1e6, 2)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
