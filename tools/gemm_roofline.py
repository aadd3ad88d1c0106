"""GEMM roofline of the Llama-3-8B training step: every library GEMM of one optimizer step, in-step vs isolated.

For each GEMM signature (aten op, operand shapes + strides, beta) of the bench step this records
* in-step: the GPU time of each call, CUDA events around the dispatch inside a real training step
  (a ``TorchDispatchMode`` sees the aten call with its exact operands; the events measure only that kernel's
  span on its stream), calls per step, TF/s;
* isolated: the same op on fresh random operands of the same shapes / strides, back to back, median of N;
* the ratio in-step / isolated, so a shape that loses time only inside the step stands out;
* GPU power and shader-clock samples (sysfs hwmon ``power1_average`` / ``pp_dpm_sclk`` of this GPU, read-only)
  taken during the in-step window and during the isolated runs.

Usage (GPU): python tools/gemm_roofline.py [--model llama3_8b] [--out gpurun_out/gemm_roofline.jsonl]
Prints one JSON line per signature (largest in-step time first) and a final summary line.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

aten = torch.ops.aten
GEMM_OPS = {aten.mm.default: "mm", aten.mm.out: "mm", aten.addmm.default: "addmm", aten.addmm.out: "addmm",
            aten.addmm_.default: "addmm_", aten.bmm.default: "bmm", aten.bmm.out: "bmm"}
try:
    GEMM_OPS[aten.mm.dtype_out] = "mm_dtype"
    GEMM_OPS[aten.addmm.dtype_out] = "addmm_dtype"
    GEMM_OPS[aten.bmm.dtype] = "bmm_dtype"
except AttributeError:
    pass


def _operands(name, args):
    if name.startswith("addmm"):
        return args[1], args[2], args[0]
    return args[0], args[1], None


def _sig(name, args, kwargs):
    a, b, c = _operands(name, args)
    beta = kwargs.get("beta", 1) if name.startswith("addmm") else 0
    return (name, tuple(a.shape), tuple(a.stride()), tuple(b.shape), tuple(b.stride()),
            None if c is None else (tuple(c.shape), tuple(c.stride())), str(a.dtype), float(beta))


def _flops(sig):
    _, ash, _, bsh, _, _, _, _ = sig
    if len(ash) == 3:
        return 2.0 * ash[0] * ash[1] * ash[2] * bsh[2]
    return 2.0 * ash[0] * ash[1] * bsh[1]


def label(sig, cfg, T):
    """Projection x pass from (M, K, N) (Llama: hidden H, fused qkv width, ffn F, vocab V, T tokens per
    micro-batch). The o projection's forward and data gradient have the same operand shapes and strides
    ([T, H] . [H, H] with a transposed right operand) and are reported together."""
    H, F, V = cfg.hidden, cfg.ffn_hidden, cfg.vocab_size
    Q = (cfg.n_heads + 2 * cfg.n_kv_heads) * cfg.head_dim
    _, ash, _, bsh, _, _, _, _ = sig
    if len(ash) == 3:
        return f"batched {ash[0]}x{ash[1]}x{ash[2]}x{bsh[2]}"
    table = {(T, H, Q): "qkv fwd", (T, H, H): "o fwd+dgrad", (T, H, 2 * F): "gate|up fwd", (T, F, H): "down fwd",
             (T, H, V): "lm_head fwd", (T, Q, H): "qkv dgrad", (T, 2 * F, H): "gate|up dgrad",
             (T, H, F): "down dgrad", (T, V, H): "lm_head dgrad", (Q, T, H): "qkv wgrad", (H, T, H): "o wgrad",
             (2 * F, T, H): "gate|up wgrad", (H, T, F): "down wgrad", (V, T, H): "lm_head wgrad"}
    return table.get((ash[0], ash[1], bsh[1]), f"{ash[0]}x{ash[1]}x{bsh[1]}")


class Recorder(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.calls = []  # (sig, start event, end event)
        self.on = False

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = GEMM_OPS.get(func)
        if not self.on or name is None:
            return func(*args, **kwargs)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = func(*args, **kwargs)
        e.record()
        self.calls.append((_sig(name, args, kwargs), s, e))
        return out


class Sampler:
    """Board power (W) and current shader clock (MHz) of this GPU (train/gpu_telemetry.py), every ``period`` s."""

    def __init__(self, period=0.05):
        from kubeoperator_amd.train.gpu_telemetry import PowerClockSampler

        self._s = PowerClockSampler(torch.cuda.current_device(), period)

    def start(self):
        self._s.start()
        return self

    def stop(self):
        r = self._s.stop() or {}
        return {"power_w": r.get("power_w"), "sclk_mhz": r.get("sclk_mhz")}


def isolated(sig, iters=20):
    name, ash, ast, bsh, bst, c, dt, beta = sig
    dtype = getattr(torch, dt.split(".")[-1])

    def make(shape, stride, dtype=dtype):
        n = 1 + sum((s - 1) * st for s, st in zip(shape, stride))
        return torch.empty(n, dtype=dtype, device="cuda").uniform_(-1, 1).as_strided(shape, stride)

    a, b = make(ash, ast), make(bsh, bst)
    if c is not None:
        cc = make(c[0], c[1], dtype=torch.float32 if "dtype" in name else dtype)
    outs = torch.empty(a.shape[0], b.shape[-1], dtype=dtype, device="cuda") if len(ash) == 2 else None

    def run():
        if name == "addmm_":
            cc.addmm_(a, b)
        elif name == "addmm":
            torch.addmm(cc, a, b, out=cc)
        elif name == "addmm_dtype":
            aten.addmm.dtype_out(cc, a, b, torch.float32, beta=1, alpha=1, out=cc)
        elif name == "mm_dtype":
            aten.mm.dtype_out(a, b, torch.float32, out=torch.empty(a.shape[0], b.shape[1], device="cuda"))
        elif name.startswith("bmm"):
            torch.bmm(a, b, out_dtype=torch.float32) if "dtype" in name else torch.bmm(a, b)
        else:
            torch.mm(a, b, out=outs)

    for _ in range(3):
        run()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        run()
        e.record()
        ts.append((s, e))
    torch.cuda.synchronize()
    ms = sorted(s.elapsed_time(e) for s, e in ts)
    del a, b
    return {"median_ms": ms[len(ms) // 2], "min_ms": ms[0]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3_8b")
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--accum", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--out", default="gpurun_out/gemm_roofline.jsonl")
    args = ap.parse_args()

    from kubeoperator_amd.parallel.dist import init_distributed
    from kubeoperator_amd.train import SyntheticTokens, TrainConfig, Trainer, gemm_tuning

    info = init_distributed("cuda")
    tuning = gemm_tuning.setup("use")
    tc = TrainConfig(model=args.model, micro_batch=1, seq_len=args.seq, grad_accum=args.accum, dp_mode="allreduce",
                     bucket_mb=512, warmup_steps=10, total_steps=1000)
    tr = Trainer(tc, info)
    data = SyntheticTokens(tr.cfg.vocab_size, 1, args.seq, info.device, seed=tc.seed)
    for _ in range(args.warmup):
        tr.train_step(data.batches(args.accum))
    torch.cuda.synchronize()
    rec = Recorder()
    samp = Sampler().start()
    t0 = time.perf_counter()
    with rec:
        rec.on = True
        tr.train_step(data.batches(args.accum))
        rec.on = False
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) * 1e3
    step_power = samp.stop()
    by = {}
    for sig, s, e in rec.calls:
        by.setdefault(sig, []).append(s.elapsed_time(e))
    del tr
    torch.cuda.empty_cache()
    rows = []
    samp = Sampler().start()
    for sig, ts in by.items():
        iso = isolated(sig)
        fl = _flops(sig)
        ins = statistics.median(ts)
        rows.append({"gemm": label(sig, tc_cfg(args.model), args.seq), "op": sig[0], "a": [sig[1], sig[2]],
                     "b": [sig[3], sig[4]], "beta": sig[7], "calls_per_step": len(ts),
                     "in_step_ms_total": round(sum(ts), 3), "in_step_ms_median": round(ins, 4),
                     "in_step_ms_min": round(min(ts), 4), "in_step_tfs": round(fl / ins / 1e9, 1),
                     "isolated_ms_median": round(iso["median_ms"], 4), "isolated_tfs": round(fl / iso["median_ms"] / 1e9, 1),
                     "in_step_over_isolated": round(ins / iso["median_ms"], 3)})
    iso_power = samp.stop()
    rows.sort(key=lambda r: -r["in_step_ms_total"])
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        for r in rows:
            print(json.dumps(r), flush=True)
            f.write(json.dumps(r) + "\n")
        tot = sum(r["in_step_ms_total"] for r in rows)
        fl = sum(_flops(sig) * len(ts) for sig, ts in by.items())
        summ = {"summary": True, "model": args.model, "gemm_selection": tuning, "step_wall_ms": round(step_ms, 1),
                "gemm_ms_per_step": round(tot, 1), "gemm_tfs_in_step": round(fl / tot / 1e9, 1),
                "gemm_calls_per_step": sum(len(ts) for ts in by.values()),
                "power_clock_in_step": step_power, "power_clock_isolated": iso_power}
        print(json.dumps(summ), flush=True)
        f.write(json.dumps(summ) + "\n")


def tc_cfg(model):
    from kubeoperator_amd.models import get_config

    return get_config(model)


if __name__ == "__main__":
    main()
