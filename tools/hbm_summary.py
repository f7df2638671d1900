"""HBM bytes per step by kernel family from tools/gpu_hbm.sh (rocprofv3 FETCH_SIZE / WRITE_SIZE,
KiB per dispatch), against the kernel time of the same dispatches.
Usage: python tools/hbm_summary.py <hbm_dir> <steps_in_trace>"""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import family  # noqa: E402


def load(d, metric):
    f = glob.glob(os.path.join(d, metric, "**", "*counter_collection.csv"), recursive=True)[0]
    out = defaultdict(float)
    t = defaultdict(float)
    for r in csv.DictReader(open(f)):
        fam = family(r["Kernel_Name"])
        out[fam] += float(r["Counter_Value"]) * 1024.0   # KiB -> bytes
        if "End_Timestamp" in r:
            t[fam] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return out, t


def main():
    d, steps = sys.argv[1], int(sys.argv[2])
    rd, _ = load(d, "FETCH_SIZE")
    wr, _ = load(d, "WRITE_SIZE")
    fams = sorted(set(rd) | set(wr), key=lambda k: -(rd.get(k, 0) + wr.get(k, 0)))
    tot_r = sum(rd.values()) / steps
    tot_w = sum(wr.values()) / steps
    print("# HBM traffic per step (rocprofv3 FETCH_SIZE + WRITE_SIZE)\n")
    print(f"total: read {tot_r / 1e9:.2f} GB + write {tot_w / 1e9:.2f} GB = "
          f"{(tot_r + tot_w) / 1e9:.2f} GB per step\n")
    print("| kernel family | read GB/step | write GB/step |")
    print("|---|---|---|")
    for k in fams[:30]:
        print(f"| {k} | {rd.get(k, 0) / steps / 1e9:.3f} | {wr.get(k, 0) / steps / 1e9:.3f} |")


if __name__ == "__main__":
    main()
