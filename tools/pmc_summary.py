"""Summarise rocprofv3 --pmc CSVs of tools/gpu_pmc.sh: mean counter values per conv case
(kernels whose name matches the regex PMC_KERNEL, default conv_gemm)."""
import collections
import csv
import glob
import os
import re
import sys


def main():
    root = sys.argv[1]
    cases = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(root, "*_g*", "p_counter_collection.csv")):
        case = os.path.basename(os.path.dirname(f)).rsplit("_g", 1)[0]
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if re.search(os.environ.get("PMC_KERNEL", "conv_gemm"), r["Kernel_Name"]):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            cases[case][k] = sum(v) / len(v)
    for case, d in sorted(cases.items()):
        print(case)
        for k, v in sorted(d.items()):
            print(f"  {k:24s} {v:14.4g}")
        w = d.get("SQ_WAVE_CYCLES")
        if w:
            print(f"  wait_any/wave_cycles   {d.get('SQ_WAIT_ANY', 0) / w:.2f}   "
                  f"wait_inst/wave_cycles {d.get('SQ_WAIT_INST_ANY', 0) / w:.2f}   "
                  f"active/wave_cycles {d.get('SQ_ACTIVE_INST_ANY', 0) / w:.2f}")


if __name__ == "__main__":
    main()
