"""Isolated timings of the transposed-companion kernels against the plain kernel + a separate transpose, at the
Llama-3-8B shapes (T = 8192 tokens, H = 4096; dQKV 8192 x 6144): effective HBM bandwidth of each.
Prints one JSON line per kernel. Usage: python tools/bench_norm_t.py [--iters 50]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--T", type=int, default=8192)
    ap.add_argument("--H", type=int, default=4096)
    a = ap.parse_args()
    from kubeoperator_amd.ops.functional import _lib
    from kubeoperator_amd.ops.reference import rope_cache

    lib = _lib()
    T, H = a.T, a.H
    g = torch.Generator(device="cuda").manual_seed(0)
    # a 1 GiB buffer swept between iterations would evict the MALL; instead rotate over 6 input sets (> 256 MB)
    sets = [[torch.randn(T, H, device="cuda", generator=g).bfloat16() for _ in range(3)] for _ in range(6)]
    w = torch.ones(H, device="cuda", dtype=torch.bfloat16)
    rstd = torch.ones(T, device="cuda")
    dw = torch.zeros(H, device="cuda", dtype=torch.bfloat16)
    it = [0]

    def nxt():
        it[0] = (it[0] + 1) % len(sets)
        return sets[it[0]]

    def emit(name, us, nbytes):
        print(json.dumps({"kernel": name, "us": round(us, 1), "TB/s": round(nbytes / us / 1e6, 2)}), flush=True)

    mb = T * H * 2
    emit("norm_fwd(res)", timeit(lambda: lib.norm_fwd(*nxt()[:2], w, None, 1e-5, False), a.iters), 4 * mb)
    emit("rms_norm_fwd_t(res)", timeit(lambda: lib.rms_norm_fwd_t(*nxt()[:2], w, 1e-5), a.iters), 5 * mb)
    emit("transpose", timeit(lambda: lib.transpose_(nxt()[0], torch.empty(H, T, device="cuda", dtype=torch.bfloat16)),
                             a.iters), 2 * mb)

    def bwd():
        x, dy, dr = nxt()
        return lib.norm_bwd(dy, x, w, rstd, None, dr, dw, None, False, False)

    def bwd_t():
        x, dy, dr = nxt()
        return lib.rms_norm_bwd_t(dy, x, w, rstd, dr, dw, False)

    emit("norm_bwd(dres)", timeit(bwd, a.iters), 4 * mb)
    emit("rms_norm_bwd_t(dres)", timeit(bwd_t, a.iters), 5 * mb)
    C = 6144
    qkv = [torch.randn(T, C, device="cuda", generator=g).bfloat16() for _ in range(4)]
    cos, sin = rope_cache(2 * T, 128, 500000.0, device="cuda")
    out = torch.empty(C, T, device="cuda", dtype=torch.bfloat16)
    j = [0]

    def q():
        j[0] = (j[0] + 1) % len(qkv)
        return qkv[j[0]]

    emit("rope(inverse)", timeit(lambda: lib.rope_(q(), cos, sin, None, T, 40, 128, True), a.iters), 2 * T * 5120 * 2)
    emit("rope_t(inverse)", timeit(lambda: lib.rope_t_(q(), cos, sin, T, 40, 128, True, out), a.iters),
         (T * C + T * 5120 + T * C) * 2)


if __name__ == "__main__":
    main()
