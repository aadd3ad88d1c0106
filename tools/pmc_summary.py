"""Aggregate rocprofv3 --pmc counter_collection CSVs per kernel (sum over dispatches), print one row per
kernel with derived ratios. Usage: python tools/pmc_summary.py gpurun_out/pmc/*/*_counter_collection.csv"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0][:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((path, r["Dispatch_Id"]))
for k, c in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    out = {n: v for n, v in c.items()}
    wc = out.get("SQ_WAVE_CYCLES", 0)
    busy = out.get("SQ_BUSY_CYCLES", 0)
    line = [f"{k:60s} disp={len(disp[k])}"]
    if busy:
        line.append(f"mfma_busy/busy={out.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / busy:.3f}")
    if wc:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_MFMA",
                  "SQ_ACTIVE_INST_LDS"):
            if n in out:
                line.append(f"{n[3:]}/wc={out[n] / wc:.3f}")
    for n in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_LDS_BANK_CONFLICT",
              "SQ_WAVES", "GRBM_GUI_ACTIVE"):
        if n in out:
            line.append(f"{n[3:] if n.startswith('SQ_') else n}={out[n]:.3g}")
    print("  ".join(line))
