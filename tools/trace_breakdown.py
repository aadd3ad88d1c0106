"""Per-step breakdown of a rocprofv3 kernel trace of bench.py: wall time between optimizer steps, GPU-busy
time (union of kernel intervals over all streams), idle gaps, and time per kernel group.

usage: python tools/trace_breakdown.py gpurun_out/prof/l8b/l8b_kernel_trace.csv [--steps 2]

Step boundaries are the gradient-clip coefficient kernel (one per optimizer step, between backward and
AdamW); the last ``--steps`` complete windows are analysed.
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict

GROUPS = [
    ("gemm", re.compile(r"Cijk_|Custom_Cijk")),
    ("attn_fwd", re.compile(r"fa_fwd")),
    ("attn_bwd", re.compile(r"fa_bwd")),
    ("adamw", re.compile(r"adamw")),
    ("fp8_quant", re.compile(r"fp8_(amax|cast)")),
    ("transpose", re.compile(r"transpose_(wide_)?kernel")),
    ("norm", re.compile(r"norm_|col_reduce|rms_(fwd|bwd)_t")),  # incl. the transposed-companion forms
    ("swiglu/gelu", re.compile(r"swiglu|gelu")),  # incl. the fused transposed-output forms
    ("rope", re.compile(r"rope")),
    ("cross_entropy", re.compile(r"\bce_|cross_entropy|xent")),
    ("splitk_reduce", re.compile(r"splitk_reduce")),
    ("grad_norm", re.compile(r"sumsq|grad_norm")),
    ("rccl", re.compile(r"ncclDevKernel|rccl", re.I)),
    ("torch_misc", re.compile(r"at::native|rocclr")),
]


def group_of(name: str) -> str:
    for g, rx in GROUPS:
        if rx.search(name):
            return g
    return "other"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--gap-us", type=float, default=20.0)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", "0")))
    rows.sort()
    starts = [s for s, e, n, _ in rows if "clip_coef" in n]
    if len(starts) < a.steps + 1:
        raise SystemExit(f"only {len(starts)} optimizer steps found")
    t0, t1 = starts[-a.steps - 1], starts[-1]
    win = [(max(s, t0), min(e, t1), n, st) for s, e, n, st in rows if e > t0 and s < t1]
    wall = (t1 - t0) / 1e6
    busy, cur_s, cur_e, gaps = 0.0, None, None, []
    for s, e, n, _ in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += (cur_e - cur_s) / 1e6
                if (s - cur_e) / 1e3 >= a.gap_us:
                    gaps.append(((s - cur_e) / 1e3, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += (cur_e - cur_s) / 1e6
    per = defaultdict(float)
    cnt = defaultdict(int)
    side = defaultdict(float)  # time off the compute stream (optimizer / weight-gradient / RCCL streams)
    by_stream = defaultdict(float)
    for s, e, n, st in win:
        by_stream[st] += e - s
    main_stream = max(by_stream, key=by_stream.get)
    for s, e, n, st in win:
        g = group_of(n)
        per[g] += (e - s) / 1e6
        cnt[g] += 1
        if st != main_stream:
            side[g] += (e - s) / 1e6
    k = a.steps
    print(f"window: {k} optimizer steps, wall {wall / k:.1f} ms/step, GPU busy (union) {busy / k:.1f} ms/step "
          f"({100 * busy / wall:.1f} %), idle {(wall - busy) / k:.1f} ms/step")
    print(f"idle gaps >= {a.gap_us:.0f} us: {len(gaps) / k:.0f}/step, {sum(g for g, _ in gaps) / 1e3 / k:.2f} ms/step")
    for g, n in sorted(gaps, reverse=True)[:8]:
        print(f"  {g:8.1f} us before {n[:90]}")
    print(f"{'group':<14}{'ms/step':>10}{'calls/step':>12}{'off-main':>10}  (kernel time summed over streams; "
          f"off-main: on other streams than the compute stream, overlapped with it)")
    for g, t in sorted(per.items(), key=lambda x: -x[1]):
        print(f"{g:<14}{t / k:>10.2f}{cnt[g] / k:>12.0f}{side[g] / k:>10.2f}")
    print(f"{'sum':<14}{sum(per.values()) / k:>10.2f}")


if __name__ == "__main__":
    main()
