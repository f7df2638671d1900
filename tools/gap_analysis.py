"""Idle gaps between consecutive kernels of a single-stream rocprofv3 kernel trace: how much
device time per step is lost between launches (dependent small kernels, tails/ramps), and after
which kernel families the largest gaps occur.
Usage: python tools/gap_analysis.py <prof_dir> <steps_to_analyse>"""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import family  # noqa: E402


def main():
    d = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
           family(r.get("Kernel_Name") or r.get("KernelName") or "")) for r in rows]
    # the last `steps` steps: split at the synthetic-data kernel that starts every step
    starts = [i for i, k in enumerate(ks) if k[2].startswith("synth_labels")]
    if len(starts) > steps:
        ks = ks[starts[-steps - 1]:starts[-1]] if len(starts) > steps else ks
    gaps = defaultdict(float)
    busy = sum(e - s for s, e, _ in ks)
    tot_gap = 0.0
    for (s0, e0, f0), (s1, e1, f1) in zip(ks, ks[1:]):
        g = s1 - e0
        if g > 0:
            gaps[f0 + " -> " + f1] += g
            tot_gap += g
    span = ks[-1][1] - ks[0][0]
    print(f"per step: span {span / 1e6 / steps:.3f} ms, kernel time {busy / 1e6 / steps:.3f} ms, "
          f"gaps {tot_gap / 1e6 / steps:.3f} ms over {len(ks) / steps:.0f} launches")
    for k, v in sorted(gaps.items(), key=lambda kv: -kv[1])[:15]:
        print(f"  {v / 1e3 / steps:8.1f} us/step  {k}")


if __name__ == "__main__":
    main()
