"""The main stream's kernel sequence of one profiled step (rocprofv3 kernel trace): every launch in
order with its duration, the gap before it and its grid, plus the forward / backward split (the
forward ends at the first cross-entropy launch). Usage: python tools/step_sequence.py <prof_dir>"""
import csv
import glob
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import family  # noqa: E402


def main():
    f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if re.search(r"synth(_s2d)?_kernel", r["Kernel_Name"])]
    rows = rows[starts[-2]:starts[-1]]
    main_id = rows[0]["Stream_Id"]
    m = [r for r in rows if r["Stream_Id"] == main_id]
    t0 = int(m[0]["Start_Timestamp"])
    prev_end = t0
    phase = "fwd"
    tot = {"fwd": [0.0, 0.0, 0], "bwd": [0.0, 0.0, 0]}
    for r in m:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = family(r["Kernel_Name"])
        if phase == "fwd" and "xent" in name:
            phase = "bwd"
        gap = (s - prev_end) / 1e3
        dur = (e - s) / 1e3
        tot[phase][0] += dur
        tot[phase][1] += max(gap, 0.0)
        tot[phase][2] += 1
        g = f"{int(r['Grid_Size_X']) // max(int(r['Workgroup_Size_X']), 1)}x{r['Grid_Size_Y']}"
        print(f"{phase} {(s - t0) / 1e3:9.1f} {dur:8.1f} gap {gap:6.1f}  {name:34s} {g}")
        prev_end = e
    for k, (d, gp, n) in tot.items():
        print(f"# {k}: {n} launches, kernel {d / 1e3:.2f} ms + gaps {gp / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
