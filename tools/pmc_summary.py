"""Aggregate rocprofv3 --pmc counter_collection CSVs per kernel and print one row per kernel with NORMALIZED ratios.

Usage: python tools/pmc_summary.py gpurun_out/pmc/*/*_counter_collection.csv

Every counter pass is a separate run, so each counter is averaged over the dispatches of ITS pass (dispatch ids are
per pass) before two counters are combined. Units (MI355X_MICROARCH.md 'rocprofv3 PMC slots', 'Per-instruction cycle
constants', 'DVFS give-back'):

* ``SQ_VALU_MFMA_BUSY_CYCLES`` counts matrix-pipe cycles summed over every SIMD (= 32 x the MFMA count for
  ``v_mfma_f32_32x32x16_bf16``, 16 x for ``16x16x32``);
* ``GRBM_GUI_ACTIVE`` counts GPU-active cycles summed over the 8 XCDs, so the kernel's cycles are GRBM / 8;
* the CSV's Start/End timestamps give each dispatch's wall time (ns).

Derived per dispatch:

* ``mfma_util`` = MFMA busy cycles / (1024 SIMDs x kernel cycles): the fraction of the chip's matrix-pipe cycles
  spent issuing MFMAs, in [0, 1] (1.0 = every SIMD's matrix pipe busy for the whole kernel);
* ``clk_GHz`` = kernel cycles / wall time (the clock the chip held; profiled passes clock 2-5 % lower than unprofiled);
* ``mfma_TFs`` = MFMA FLOPs / wall time, with FLOPs = busy cycles x 1,024 (a dense bf16 MFMA does 1,024 FLOP per SIMD
  cycle: 32,768 per 32-cycle 32x32x16) -- comparable with the 2,500 TF/s dense bf16 peak at 2.4 GHz;
* wave-cycle fractions (``WAIT_ANY/wc`` ...) as before (SQ wave counters count in the same units, ratios are safe);
* ``FETCH_SIZE`` / ``WRITE_SIZE`` (KB per dispatch) as MB and TB/s over the dispatch's wall time, and
  ``l2_hit`` = TCC_HIT / (TCC_HIT + TCC_MISS) when both passes ran.
"""
import collections
import csv
import sys

N_SIMD, N_XCD, FLOP_PER_MFMA_CYCLE = 1024, 8, 1024.0


def main(paths):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))  # kernel -> counter -> sum
    ndisp = collections.defaultdict(lambda: collections.defaultdict(set))  # kernel -> counter -> dispatches
    wall = collections.defaultdict(dict)  # kernel -> (pass, dispatch) -> ns
    for path in paths:
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0][:60]
            c = r["Counter_Name"]
            tot[k][c] += float(r["Counter_Value"])
            ndisp[k][c].add((path, r["Dispatch_Id"]))
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                wall[k][(path, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])

    def per(k, c):  # mean per dispatch of counter c, over its own pass
        n = len(ndisp[k].get(c, ()))
        return tot[k][c] / n if n else None

    for k in sorted(tot, key=lambda x: -(per(x, "SQ_WAVE_CYCLES") or 0)):
        line = [f"{k:60s}"]
        ns = sorted(wall[k].values())
        dur = ns[len(ns) // 2] * 1e-9 if ns else None  # median wall time of a dispatch
        busy, grbm = per(k, "SQ_VALU_MFMA_BUSY_CYCLES"), per(k, "GRBM_GUI_ACTIVE")
        if dur:
            line.append(f"wall_us={dur * 1e6:.1f}")
        if grbm:
            cyc = grbm / N_XCD
            if dur:
                line.append(f"clk_GHz={cyc / dur * 1e-9:.2f}")
            if busy is not None:
                line.append(f"mfma_util={busy / (N_SIMD * cyc):.3f}")
        if busy and dur:
            line.append(f"mfma_TFs={busy * FLOP_PER_MFMA_CYCLE / dur * 1e-12:.0f}")
        wc = tot[k].get("SQ_WAVE_CYCLES", 0)
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_MFMA",
                      "SQ_ACTIVE_INST_LDS"):
                v, w = per(k, n), per(k, "SQ_WAVE_CYCLES")
                if v is not None and w:
                    line.append(f"{n[3:]}/wc={v / w:.3f}")
        # HBM-side traffic (rocprofv3 derived counters, KB per dispatch) and the L2 hit rate
        for n, tag in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
            v = per(k, n)
            if v is not None:
                line.append(f"{tag}_MB={v / 1024:.1f}")
                if dur:
                    line.append(f"{tag}_TBs={v * 1024 / dur * 1e-12:.2f}")
        hit, miss = per(k, "TCC_HIT_sum"), per(k, "TCC_MISS_sum")
        if hit is not None and miss is not None and hit + miss > 0:
            line.append(f"l2_hit={hit / (hit + miss):.3f}")
        for n in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_LDS_BANK_CONFLICT"):
            v = per(k, n)
            if v is not None:
                line.append(f"{n[3:]}/disp={v:.3g}")
        print("  ".join(line))


if __name__ == "__main__":
    main(sys.argv[1:])
