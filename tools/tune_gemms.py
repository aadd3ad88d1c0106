"""Offline hipBLASLt solution tuning for the training step's GEMM shapes (TunableOp), one shape at a time
with a progress line per shape (a long silent tuning run looks hung to the job runner).

1. one training step with TunableOp recording (not tuning) every GEMM it calls;
2. each recorded GEMM is tuned on its own (max KOP_TUNE_MS ms / KOP_TUNE_ITERS iterations per solution);
3. the winners are written (at exit) to kubeoperator_amd/tuning/tunableop_results_gfx950.csv, which bench.py and the
   trainer load read-only (``--gemm-tuning use``).

Usage (one MI355X): python tools/tune_gemms.py [--model llama3_8b --seq 8192 --mbs 1]
Re-tune under other settings into a separate file (A/B against the committed winners with KOP_GEMM_RESULTS=<out>):
  KOP_TUNE_MS=200 KOP_TUNE_ITERS=100 python tools/tune_gemms.py --fresh --skip 128256 --out gpurun_out/t.csv
(--fresh: re-tune every recorded shape, --skip: keep the committed winner of shapes matching the regex; the output
is the committed file with the re-tuned rows replaced.)
"""
import argparse
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def merge_results(committed_lines, results):
    """The committed TunableOp file with the rows of re-tuned signatures replaced (Validator and untouched rows kept
    in place) and signatures new to it appended. ``results``: tuples (op, params, solution, ms)."""
    new = {(r[0], r[1]): r for r in results}
    rows, seen = [], set()
    for ln in committed_lines:
        f = ln.rstrip("\n").split(",")
        key = (f[0], f[1]) if len(f) >= 4 and not f[0].startswith("Validator") else None
        if key in new:
            r = new[key]
            rows.append(f"{r[0]},{r[1]},{r[2]},{r[3]}\n")
            seen.add(key)
        else:
            rows.append(ln if ln.endswith("\n") else ln + "\n")
    for key, r in new.items():
        if key not in seen:
            rows.append(f"{r[0]},{r[1]},{r[2]},{r[3]}\n")
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3_8b")
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--mbs", type=int, default=1)
    ap.add_argument("--out", default="", help="write the merged winners here instead of the committed file")
    ap.add_argument("--fresh", action="store_true", help="re-tune shapes that already have a committed winner")
    ap.add_argument("--skip", default="", help="regex: recorded GEMMs to leave alone (e.g. the LM head, 128256)")
    a = ap.parse_args()

    import torch
    import torch.cuda.tunable as tun

    from kubeoperator_amd.parallel.dist import init_distributed
    from kubeoperator_amd.train import SyntheticTokens, TrainConfig, Trainer
    from kubeoperator_amd.train.gemm_tuning import results_path

    committed = results_path()
    out = os.path.abspath(a.out) if a.out else committed
    os.makedirs(os.path.dirname(out), exist_ok=True)
    untuned = os.path.join(os.path.dirname(out), "untuned_gemms.csv")
    for p in (untuned,):
        if os.path.exists(p):
            os.remove(p)
    os.environ["PYTORCH_TUNABLEOP_UNTUNED_FILENAME"] = untuned
    tun.enable(True)
    tun.tuning_enable(False)
    tun.record_untuned_enable(True)
    # TunableOp's own exit-time dump goes to a scratch file; the merged winners are written below
    tun.set_filename(out + ".tunableop", insert_device_ordinal=False)
    if os.path.exists(committed) and not a.fresh:
        tun.read_file(committed)  # keep the committed winners: only shapes without one are recorded and tuned

    info = init_distributed("auto")
    tr = Trainer(TrainConfig(model=a.model, micro_batch=a.mbs, seq_len=a.seq, warmup_steps=10, total_steps=100), info)
    data = SyntheticTokens(tr.cfg.vocab_size, a.mbs, a.seq, info.device, seed=1)
    tr.train_step(data.batches(1))
    torch.cuda.synchronize()
    tun.record_untuned_enable(False)
    # the untuned file is flushed when recording stops / at exit; give the writer a moment
    for _ in range(50):
        if os.path.exists(untuned) and os.path.getsize(untuned) > 0:
            break
        time.sleep(0.1)
    cands = [p for p in (untuned, untuned.replace(".csv", "0.csv")) if os.path.exists(p)]
    if not cands:
        print("no untuned GEMM file was written", flush=True)
        return 1
    lines = [ln for ln in open(cands[0]) if ln.startswith(("Gemm", "ScaledGemm"))]
    lines = sorted(set(lines), key=lines.index)
    if a.skip:
        lines = [ln for ln in lines if not re.search(a.skip, ln)]
    print(f"{len(lines)} distinct GEMMs to tune", flush=True)

    tun.tuning_enable(True)
    tun.set_max_tuning_duration(int(os.environ.get("KOP_TUNE_MS", "30")))
    tun.set_max_tuning_iterations(int(os.environ.get("KOP_TUNE_ITERS", "10")))
    dev = torch.cuda.current_device()
    for i, ln in enumerate(lines):
        t0 = time.time()
        tun._process_single_offline_gemm(ln, dev)
        torch.cuda.synchronize()
        print(f"[{i + 1}/{len(lines)}] {time.time() - t0:6.1f}s {ln.strip()[:160]}", flush=True)
    res = tun.get_results()
    rows = merge_results(open(committed).readlines() if os.path.exists(committed) else [], res)
    new = {(r[0], r[1]) for r in res}
    with open(out, "w") as fh:
        fh.writelines(rows)
    print(f"wrote {len(new)} tuned results merged into {out}", flush=True)
    for r in res:
        print("  ", r, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
