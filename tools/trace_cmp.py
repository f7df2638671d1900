"""Per (kernel family, grid) time of two rocprofv3 kernel traces of the bench step, side by side.
Usage: python tools/trace_cmp.py <prof_dir_A> <prof_dir_B> [top]
Rows: us/step (whole trace window of full steps, see prof_summary.py), launches/step, and B - A."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import family  # noqa: E402


def load(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows)
              if re.match(r"(void )?(\(anonymous namespace\)::)?synth(_s2d)?_kernel", r["Kernel_Name"])]
    steps = 1
    if len(starts) >= 2:
        rows, steps = rows[starts[0]:starts[-1]], len(starts) - 1
    t = defaultdict(float)
    n = defaultdict(int)
    for r in rows:
        k = (family(r["Kernel_Name"]), int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])),
             int(r["Grid_Size_Y"]), r["Stream_Id"])
        t[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        n[k] += 1
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3 / steps
    return {k: (v / steps, n[k] / steps) for k, v in t.items()}, span


def main():
    a, sa = load(sys.argv[1])
    b, sb = load(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 60
    keys = sorted(set(a) | set(b), key=lambda k: -max(a.get(k, (0, 0))[0], b.get(k, (0, 0))[0]))
    print(f"span/step: A {sa:.0f} us, B {sb:.0f} us, B - A {sb - sa:+.0f} us\n")
    print("| kernel | blocks | y | stream | A us/step | A n | B us/step | B n | B - A |")
    print("|---|---|---|---|---|---|---|---|---|")
    for k in keys[:top]:
        ta, na = a.get(k, (0.0, 0))
        tb, nb = b.get(k, (0.0, 0))
        print(f"| {k[0]} | {k[1]} | {k[2]} | {k[3]} | {ta:.1f} | {na:.1f} | {tb:.1f} | {nb:.1f} | {tb - ta:+.1f} |")
    ta = sum(v[0] for v in a.values())
    tb = sum(v[0] for v in b.values())
    print(f"\nkernel-time sum/step: A {ta:.0f} us, B {tb:.0f} us, B - A {tb - ta:+.0f} us")


if __name__ == "__main__":
    main()
