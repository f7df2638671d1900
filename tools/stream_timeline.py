"""Per-stream busy time and the critical path of the native step from a rocprofv3 kernel trace:
for each HIP stream, the union of its kernel intervals per step; plus the time during which ONLY
the main stream is busy (the side stream idle) -- the part a faster side stream cannot hide.
Usage: python tools/stream_timeline.py <prof_dir>"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    if not iv:
        return 0, []
    out, (cs, ce) = [], iv[0]
    for s, e in iv[1:]:
        if s > ce:
            out.append((cs, ce))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    out.append((cs, ce))
    return sum(e - s for s, e in out), out


def main():
    f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if re.search(r"synth(_s2d)?_kernel", r["Kernel_Name"])]
    rows = rows[starts[0]:starts[-1]]
    steps = len(starts) - 1
    by = defaultdict(list)
    for r in rows:
        by[r["Stream_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    main_id = max(by, key=lambda k: len(by[k]))
    tot, allu = union([iv for v in by.values() for iv in v])
    span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
    print(f"{steps} steps, span {span / 1e6 / steps:.2f} ms/step, any-stream busy {tot / 1e6 / steps:.2f} ms/step")
    unions = {}
    for k, v in sorted(by.items()):
        b, u = union(v)
        unions[k] = u
        print(f"stream {k}{' (main)' if k == main_id else ''}: {len(v) / steps:.0f} kernels/step, "
              f"busy {b / 1e6 / steps:.2f} ms/step")
    # main-only time: main busy minus overlap with any other stream
    others = union([iv for k, v in by.items() if k != main_id for iv in v])[1]
    ov = 0
    j = 0
    for s, e in unions[main_id]:
        while j < len(others) and others[j][1] <= s:
            j += 1
        k = j
        while k < len(others) and others[k][0] < e:
            ov += max(0, min(e, others[k][1]) - max(s, others[k][0]))
            k += 1
    mb = sum(e - s for s, e in unions[main_id])
    print(f"main stream alone {(mb - ov) / 1e6 / steps:.2f} ms/step, main with others "
          f"{ov / 1e6 / steps:.2f} ms/step, others alone {(tot - mb) / 1e6 / steps:.2f} ms/step")


if __name__ == "__main__":
    main()
