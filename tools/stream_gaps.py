"""Per-stream gaps of a rocprofv3 kernel trace of bench.py: for each HIP stream, the idle time between one kernel's
end and the next kernel's start on the SAME stream, summed per (previous kernel, next kernel) pair over the last
``--steps`` optimizer steps (step boundaries: the clip-coefficient kernel, as in tools/trace_breakdown.py).

A compute stream that waits on nothing still shows ~1-2 us between dependent kernels; gaps of ~10-15 us that repeat
at the same kernel pairs are the marker packets of event records (``Stream.wait_stream`` / ``Event.record``: the
next kernel is held until the marker retires) -- what the grouped weight-gradient launches
(``FlatParamStore.side_submit``) remove.

usage: python tools/stream_gaps.py gpurun_out/prof/gpt2/gpt2_kernel_trace.csv [--steps 2] [--min-us 5] [--top 20]
"""
from __future__ import annotations

import argparse
import csv
from collections import Counter, defaultdict


def load(path: str):
    with open(path) as f:
        rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", "0"))
                for r in csv.DictReader(f)]
    rows.sort()
    return rows


def stream_gaps(rows, steps: int, min_us: float):
    starts = [s for s, _, n, _ in rows if "clip_coef" in n]
    if len(starts) < steps + 1:
        raise SystemExit(f"only {len(starts)} optimizer steps found")
    t0, t1 = starts[-steps - 1], starts[-1]
    by_stream = defaultdict(list)
    for r in rows:
        if t0 <= r[0] < t1:
            by_stream[r[3]].append(r)
    out = {}
    for st, ks in by_stream.items():
        busy = sum(e - s for s, e, _, _ in ks) / 1e6 / steps
        pairs, cnt, total, hist = defaultdict(float), Counter(), 0.0, Counter()
        for a, b in zip(ks, ks[1:]):
            g = (b[0] - a[1]) / 1e3
            if g < min_us:
                continue
            key = (a[2][:60], b[2][:60])
            pairs[key] += g / steps
            cnt[key] += 1
            total += g / steps
            hist[min(int(g // 5) * 5, 50)] += 1
        out[st] = {"kernels_per_step": len(ks) / steps, "busy_ms": busy, "gap_ms": total / 1e3, "pairs": pairs,
                   "counts": cnt, "hist": hist}
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--min-us", type=float, default=5.0)
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    res = stream_gaps(load(a.trace), a.steps, a.min_us)
    for st, r in sorted(res.items()):
        print(f"stream {st}: {r['kernels_per_step']:.0f} kernels/step, busy {r['busy_ms']:.2f} ms/step, "
              f"gaps >= {a.min_us:g} us between its own kernels {r['gap_ms']:.2f} ms/step")
        hist = ", ".join(f"{k}-{k + 5}us: {v // a.steps}" if k < 50 else f">=50us: {v // a.steps}"
                         for k, v in sorted(r["hist"].items()))
        print(f"  per step by size: {hist}")
        for (pa, pb), us in sorted(r["pairs"].items(), key=lambda x: -x[1])[:a.top]:
            n = r["counts"][(pa, pb)] // a.steps
            print(f"  {us / 1e3:7.3f} ms {n:4d}x  after {pa:60s} before {pb}")


if __name__ == "__main__":
    main()
