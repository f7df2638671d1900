"""Main-stream launches, busy time, gaps and per-family time of the last full step in a rocprofv3
kernel trace. Usage: python tools/main_stream_summary.py <prof_dir>"""
import sys, os, re
sys.path.insert(0, "tools")
import csv, glob
from collections import defaultdict
from prof_summary import family
d = sys.argv[1]
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if re.match(r"(void )?(\(anonymous namespace\)::)?synth(_s2d)?_kernel", r["Kernel_Name"])]
rows, steps = rows[starts[-2]:starts[-1]], 1
m = [r for r in rows if r["Stream_Id"] == rows[0]["Stream_Id"]]
s = [r for r in rows if r["Stream_Id"] != rows[0]["Stream_Id"]]
t0 = int(rows[0]["Start_Timestamp"]); t1 = int(rows[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in m)
print("span", (t1-t0)/1e3, "main launches", len(m), "main busy", busy/1e3, "gaps", (t1-t0-busy)/1e3, "side launches", len(s))
fam = defaultdict(lambda: [0.0, 0])
for r in m:
    k = family(r["Kernel_Name"]).split()[0]
    fam[k][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))/1e3; fam[k][1] += 1
for k, v in sorted(fam.items(), key=lambda x: -x[1][0]):
    print(f"  {k:32s} {v[0]:8.1f} us  n={v[1]}")
# gaps distribution
g = []
for a, b in zip(m, m[1:]):
    g.append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"]))/1e3)
import statistics
print("gap median", statistics.median(g), "sum", sum(x for x in g if x>0), "n>5us", sum(1 for x in g if x>5))
# forward/backward split: find first xent kernel
print("--- bn_stats by grid")
bs = defaultdict(lambda: [0.0, 0])
prev = None
for i, r in enumerate(m):
    if "bn_stats" in r["Kernel_Name"]:
        k = (int(r["Grid_Size_X"])//256, int(r["Grid_Size_Y"]), family(m[i-1]["Kernel_Name"]))
        bs[k][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))/1e3; bs[k][1] += 1
for k, v in sorted(bs.items(), key=lambda x: -x[1][0]):
    print(f"  {str(k):60s} {v[0]:8.1f} us  n={v[1]} avg {v[0]/v[1]:.1f}")
