"""Stem weight gradient (WGRAD_BNA: dY = k1*dz + k2*y + k3 formed while staging; M = 64, N = 256,
K = B*112*112) at several split-K block targets, incl. the slab reduce; median of 5 interleaved
rounds x 3 reps (us), and the result checked against the default target.
Usage (GPU box): python tools/stem_wgrad_sweep.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_amd.ops import ext  # noqa: E402
from pytorch_distributed_amd.ops import native_ops as K  # noqa: E402


def main():
    ext.load(required=True)
    B = 400
    dev = torch.device("cuda", 0)
    g = K.stem_s2d_geom(B, 224)
    x = (torch.randn(B, 112, 112, 16, device=dev) * 0.5).to(torch.bfloat16)
    dz = (torch.randn(B, g.Ho, g.Wo, 64, device=dev) * 0.01).to(torch.bfloat16)
    y = torch.randn(B, g.Ho, g.Wo, 64, device=dev).to(torch.bfloat16)
    k = torch.randn(3 * 64, device=dev) * 0.1
    ws = K.Workspace(dev)
    out = torch.empty(64 * 256, device=dev)
    # (round 6 also timed a double-buffered 64x256 build: 440-446 us at 512-1536 blocks vs
    # 395-397 us single-stage -- not built; profiles/ab_r6.md section 14)
    # (("tap", n): the tap-reuse stem kernel with n blocks, csrc/wgrad_tap.hip)
    targets = [((-64, 256), 1024), ((-64, 128), 1536), ((-64, 256), 512), ((-64, 256), 768),
               ((64, 128), 1024)]
    if K.stem_wgrad_tap_ok(g, torch.bfloat16, force=True):
        targets += [("tap", 256), ("tap", 384), ("tap", 512), ("tap", 768), ("tap", 1024)]

    def run(tb):
        if tb[0] == "tap":
            K.conv_wgrad_stem_tap(dz, y, k, x, g, out, ws, blocks=tb[1])
        else:
            K.conv_wgrad(dz, x, g, out, ws, bna=(y, k), tile=tb[0], target_blocks=tb[1])
    res = {}
    for tb in targets:
        run(tb)
        torch.cuda.synchronize()
        res[tb] = out.clone()
    ref = res[targets[0]]
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {tb: [] for tb in targets}
    for _ in range(5):
        for tb in targets:
            st.record()
            for _ in range(3):
                run(tb)
            en.record()
            en.synchronize()
            times[tb].append(st.elapsed_time(en) / 3 * 1e3)
    for tb in targets:
        plan = "-" if tb[0] == "tap" else K.wgrad_plan(g, B, tile=tb[0], target_blocks=tb[1])
        err = ((res[tb] - ref).norm() / ref.norm()).item()
        print(f"tile {str(tb[0]):>10} target {tb[1]:5d} plan {plan}: {statistics.median(times[tb]):8.1f} us  "
              f"rel diff vs the first: {err:.2e}")


if __name__ == "__main__":
    main()
