"""Inter-kernel gaps on one stream by kernel kind, for rocprofv3 --kernel-trace: n back-to-back
launches each of (1) a streaming BatchNorm apply, (2) a 1x1 conv forward (ConvParams by value,
~0.9 KB of kernel arguments), (3) a 1x1 conv data gradient (the same struct read in place from the
kernarg segment), (4) conv forward -> BN statistics pairs, as in the forward. The trace gives each
kernel's start / end; tools/gap_bench.py --summary <trace dir> prints the median gap before each kind.
Usage: rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python tools/gap_bench.py [n]
       python tools/gap_bench.py --summary DIR"""
import csv
import glob
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def summary(d):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from prof_summary import family
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    gaps = {}
    for a, b in zip(rows, rows[1:]):
        if a["Stream_Id"] != b["Stream_Id"]:
            continue
        ka, kb = family(a["Kernel_Name"]), family(b["Kernel_Name"])
        g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
        gaps.setdefault((ka, kb), []).append(g)
    for (ka, kb), v in sorted(gaps.items(), key=lambda x: -len(x[1])):
        if len(v) >= 10:
            print(f"{ka[:28]:28s} -> {kb[:28]:28s} n={len(v):4d} median gap {statistics.median(v):6.2f} us"
                  f"  mean {statistics.mean(v):6.2f}")


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
        return
    import torch
    from pytorch_distributed_amd.ops import ext
    from pytorch_distributed_amd.ops import native_ops as K
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    ext.load(required=True)
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    B, H, Cin, Cout = 100, 28, 256, 256
    g = K.ConvGeom(B, H, H, Cin, Cout, 1, 1, 1, 0)
    x = torch.randn(B, H, H, Cin, device=dev).to(dt)
    w = (torch.randn(Cout, Cin, device=dev) * 0.05).to(dt)
    y = torch.empty(B, H, H, Cout, device=dev, dtype=dt)
    dx = torch.empty_like(x)
    sc = torch.rand(Cin, device=dev) + 0.5
    sh = torch.randn(Cin, device=dev) * 0.1
    a = torch.empty_like(x)
    ws = K.Workspace(dev)
    M = B * H * H
    st = [torch.empty(Cout, device=dev) for _ in range(4)]
    bn = K.BnStats(ws, torch.ones(Cout, device=dev), torch.zeros(Cout, device=dev), 1e-5, 0.1,
                   st[0], st[1], st[2], st[3], update_running=False)
    stats = torch.empty(math.ceil(M / 64) * 3 * Cout, device=dev)
    for _ in range(2):
        for _ in range(n):
            K.bn_apply(x, sc, sh, a, relu=True)
        for _ in range(n):
            K.conv_fwd(x, w, g, y, stats=stats, tile=(-128, 128))
        for _ in range(n):
            K.conv_dgrad(y, w.view(Cout, 1, 1, Cin), g, dx, tile=(-128, 128))
        for _ in range(n):
            K.conv_fwd(x, w, g, y, bn=bn, tile=(-128, 128))
        torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
