"""Summarise tools/gpu_pmc_step.sh: per (kernel family, grid) of the bench step, the mean of each
counter per dispatch, with derived ratios (MFMA busy share of the chip, VALU / MFMA instructions,
LDS bank-conflict share, bytes per dispatch with the FETCH_SIZE calibration applied).
Usage: python tools/pmc_step_summary.py gpurun_out/pmc_step"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import family  # noqa: E402

N_SIMD = 256 * 4


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return []
    return list(csv.DictReader(open(f[0])))


def key_of(r):
    grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
    wg = r.get("Workgroup_Size") or r.get("Workgroup_Size_X") or "1"
    try:
        blocks = int(grid) // max(1, int(wg))
    except ValueError:
        blocks = grid
    return family(r["Kernel_Name"]), blocks


def calib(d):
    """FETCH_SIZE and WRITE_SIZE per launch of tools/fetch_calib.py vs its exact bytes."""
    out = {}
    for m in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = [r for r in load(os.path.join(d, f"calib_{m}")) if "bn_apply" in r["Kernel_Name"]]
        txt = open(os.path.join(d, f"calib_{m}.txt")).read() if os.path.exists(
            os.path.join(d, f"calib_{m}.txt")) else ""
        mm = re.search(r"read (\d+) .* write (\d+)", txt)
        if rows and mm:
            meas = sum(float(r["Counter_Value"]) for r in rows) / len(rows) * 1024.0
            exact = float(mm.group(1) if m == "FETCH_SIZE" else mm.group(2))
            out[m] = exact / meas
    return out


def main():
    d = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(float))
    n = defaultdict(lambda: defaultdict(int))
    dur = defaultdict(list)
    for g in sorted(glob.glob(os.path.join(d, "g*"))):
        if not os.path.isdir(g):
            continue
        for r in load(g):
            k = key_of(r)
            c = r["Counter_Name"]
            acc[k][c] += float(r["Counter_Value"])
            n[k][c] += 1
            if c in ("SQ_WAVES", "FETCH_SIZE") and r.get("End_Timestamp"):
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    cf = calib(d)
    fr, wr = cf.get("FETCH_SIZE", 1.0), cf.get("WRITE_SIZE", 1.0)
    print("# Step PMC per kernel (bench.py bf16 bs400, counters per dispatch, dispatches serialised)\n")
    print(f"FETCH_SIZE calibration (exact / counted bytes, bn_apply_u on 642 MB tensors): {fr:.3f}; "
          f"WRITE_SIZE: {wr:.3f}. Bytes below are calibrated.\n")
    print("| kernel | blocks | launches | us | MFMA busy % | VALU/MFMA | LDS/MFMA | LDS conflict % "
          "| wait % | read MB | write MB | GB/s |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    rows = []
    for k, a in acc.items():
        def m(c):
            return a[c] / n[k][c] if n[k][c] else float("nan")
        us = sum(dur[k]) / len(dur[k]) if dur[k] else float("nan")
        launches = max(n[k].values()) if n[k] else 0
        gui = m("GRBM_GUI_ACTIVE") / 8.0
        busy = 100.0 * m("SQ_VALU_MFMA_BUSY_CYCLES") / (gui * N_SIMD) if gui else float("nan")
        mf = m("SQ_INSTS_MFMA")
        rd = m("FETCH_SIZE") * 1024.0 * fr / 1e6
        wt = m("WRITE_SIZE") * 1024.0 * wr / 1e6
        gbs = (rd + wt) / us * 1e3 if us == us and us > 0 else float("nan")
        rows.append((us * launches if us == us else 0, k, launches, us, busy,
                     m("SQ_INSTS_VALU") / mf if mf else float("nan"),
                     m("SQ_INSTS_LDS") / mf if mf else float("nan"),
                     100.0 * m("SQ_LDS_BANK_CONFLICT") / m("SQ_LDS_IDX_ACTIVE") if m("SQ_LDS_IDX_ACTIVE") else float("nan"),
                     100.0 * m("SQ_WAIT_ANY") / m("SQ_WAVE_CYCLES") if m("SQ_WAVE_CYCLES") else float("nan"),
                     rd, wt, gbs))
    for r in sorted(rows, key=lambda r: -r[0])[:60]:
        _, (fam, blocks), launches, us, busy, vm, lm, lc, wa, rd, wt, gbs = r
        print(f"| {fam} | {blocks} | {launches} | {us:.1f} | {busy:.1f} | {vm:.2f} | {lm:.2f} | {lc:.1f} "
              f"| {wa:.0f} | {rd:.0f} | {wt:.0f} | {gbs:.0f} |")


if __name__ == "__main__":
    main()
