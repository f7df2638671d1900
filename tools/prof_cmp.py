"""Per-launch comparison of rocprofv3 kernel traces (one training step each).
Usage: python tools/prof_cmp.py DIR_A DIR_B   (dirs holding run_kernel_trace.csv)
Steps are delimited by the synthetic-data kernel; the last complete step of each trace is used.
Kernels are matched by family and occurrence order within the step."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def fam(n):
    m = re.search(r"conv_gemm_kernel<(\d)", n)
    if m:
        return {"0": "conv_fwd", "1": "conv_dgrad", "2": "conv_wgrad"}[m.group(1)]
    n = re.sub(r"^void ", "", n).replace("(anonymous namespace)::", "")
    return re.sub(r"[<(].*", "", n)[:40]


def last_step(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "synth_s2d" in r["Kernel_Name"]]
    a, b = starts[-2], starts[-1]
    step = rows[a:b]
    out = defaultdict(list)
    for r in step:
        out[fam(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    t0, t1 = int(step[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    return out, (t1 - t0) / 1e3


def main():
    A, ta = last_step(sys.argv[1])
    B, tb = last_step(sys.argv[2])
    print(f"step span: A {ta:.0f} us  B {tb:.0f} us")
    print(f"{'family':40s} {'nA':>4s} {'nB':>4s} {'sumA':>9s} {'sumB':>9s} {'delta':>8s}")
    for k in sorted(set(A) | set(B), key=lambda k: -(sum(B.get(k, [])) + sum(A.get(k, [])))):
        sa, sb = sum(A.get(k, [])), sum(B.get(k, []))
        print(f"{k:40s} {len(A.get(k, [])):4d} {len(B.get(k, [])):4d} {sa:9.0f} {sb:9.0f} {sb - sa:8.0f}")
    for k in ("conv_fwd", "conv_dgrad", "conv_wgrad"):
        a, b = A.get(k, []), B.get(k, [])
        if len(a) == len(b):
            print(k, "per launch (A -> B, us):")
            print("  " + "  ".join(f"{x:.0f}->{y:.0f}" for x, y in zip(a, b)))


if __name__ == "__main__":
    main()
