"""Static instruction mix of the conv kernels (device asm from ``hipcc -S --cuda-device-only``).

Usage: python tools/asm_stats.py conv.s [name-substring ...]
Prints per kernel: VALU / MFMA / LDS / VMEM / SALU counts, plus the split before the first and
after the last MFMA (prologue+loop vs epilogue), and the kernel's VGPR / spill metadata.
"""
import re
import sys
from collections import Counter


def classify(op: str) -> str:
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path = sys.argv[1]
    subs = sys.argv[2:]
    lines = open(path).read().splitlines()
    starts = [(i, l.split(":")[0]) for i, l in enumerate(lines)
              if re.match(r"^_Z\S*conv_gemm_kernel\S*:", l)]
    for k, (i0, name) in enumerate(starts):
        if subs and not any(s in name for s in subs):
            continue
        i1 = starts[k + 1][0] if k + 1 < len(starts) else len(lines)
        body = []
        meta = {}
        for l in lines[i0:i1]:
            t = l.strip()
            m = re.match(r";\s*(NumVgprs|NumAgprs|ScratchSize|Occupancy|TotalNumVgprs):\s*(\d+)", t)
            if m:
                meta[m.group(1)] = int(m.group(2))
            if not t or t.startswith((";", ".", "_")) or t.endswith(":"):
                continue
            body.append(t.split()[0])
        cls = [classify(o) for o in body]
        mf = [j for j, c in enumerate(cls) if c == "mfma"]
        pre = Counter(cls[:mf[0]]) if mf else Counter()
        post = Counter(cls[mf[-1] + 1:]) if mf else Counter()
        tot = Counter(cls)
        tag = re.search(r"kernelILi(\d)ELi(\d)ELi(\d+)ELi(\d+)ELi(\d)E", name)
        print(f"PASS{tag.group(1)} DT{tag.group(2)} {tag.group(3)}x{tag.group(4)} ST{tag.group(5)}  "
              f"{dict(meta)}")
        for lab, c in (("total", tot), ("pre-mfma", pre), ("post-mfma", post)):
            print(f"   {lab:10s} " + " ".join(f"{x}={c.get(x, 0)}" for x in
                                             ("valu", "mfma", "lds", "vmem", "salu")))


if __name__ == "__main__":
    main()
