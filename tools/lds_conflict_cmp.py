"""LDS bank-conflict share (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE) per (kernel family, grid) of
two step PMC runs side by side -- e.g. the full tools/gpu_pmc_step.sh group 2 of the in-tree
library against tools/gpu_lds_variant.sh's run of a variant.
Usage: python tools/lds_conflict_cmp.py gpurun_out/pmc_step/g2 gpurun_out/ldsv/g2 [min_blocks]"""
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_step_summary import key_of, load  # noqa: E402


def shares(d):
    acc = defaultdict(lambda: defaultdict(float))
    for r in load(d):
        acc[key_of(r)][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for k, c in acc.items():
        act = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
        if act > 0:
            out[k] = (100.0 * c.get("SQ_LDS_BANK_CONFLICT", 0.0) / act, c.get("SQ_INSTS_LDS", 0.0))
    return out


def main():
    a, b = shares(sys.argv[1]), shares(sys.argv[2])
    mb = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    print("| kernel | blocks | conflict % A | conflict % B | LDS instrs B / A |")
    print("|---|---|---|---|---|")
    for k in sorted(set(a) & set(b), key=lambda k: -a[k][0]):
        if isinstance(k[1], int) and k[1] < mb:
            continue
        ra = a[k][1] or 1.0
        print(f"| {k[0]} | {k[1]} | {a[k][0]:.1f} | {b[k][0]:.1f} | {b[k][1] / ra:.2f} |")


if __name__ == "__main__":
    main()
