"""Analytic byte ledger of the native ResNet-50 bf16 training step (bs 400, 224 px), default plan.

Walks the schedule of models/native.py (forward: stem + pool, FWD_TAIL folds of layers 1-2, the
BN+ReLU operand prologues by PDA_FUSE_PROLOGUE "1x1:56", bn_apply where a 3x3 HALO consumer needs a
materialised input, shortcut convs and the forward-time Gram of the folded tails on the second
stream; backward: the fused dgrad epilogues, bn_bwd_finish apply passes, the DGRAD_BNF / WGRAD_BNA
tail folds of layers 1-3, weight gradients and their split-K slabs, the stem's fused backward) and
lists, per kernel launch, the activation / gradient bytes it reads and writes (weights, BN
coefficients and statistics partials are counted only where they are MB-scale: the f32 split-K
slabs). Every tensor access is charged once per kernel (an L2/MALL-served re-read inside a kernel
is not HBM traffic); cross-kernel re-reads are charged every time (the 256 MiB Infinity Cache may
serve some of them -- the measured FETCH_SIZE is the arbiter, profiles/pmc_*_step.md).

Then, per tensor: who writes it, who reads it, total bytes moved, against the minimum the
schedule's data flow needs (one write + one read per consumer pass that cannot be fused).

Usage: python tools/byte_ledger.py [--md]"""
from __future__ import annotations

import sys
from collections import defaultdict

B = 400
ES = 2          # bf16
MB = 1e6

# (stage, blocks, mid channels, out channels, input size, stride of the first block)
STAGES = [(1, 3, 64, 256, 56, 1), (2, 4, 128, 512, 56, 2), (3, 6, 256, 1024, 28, 2),
          (4, 3, 512, 2048, 14, 2)]


def T(h, c, es=ES):
    return B * h * h * c * es / MB


class Ledger:
    def __init__(self):
        self.launches = []      # (phase, stream, kernel, {tensor: bytes} reads, writes)
        self.tensors = {}

    def t(self, name, h, c, es=ES):
        self.tensors[name] = T(h, c, es)
        return name

    def wg(self, phase, kernel, reads, slab_mb):
        """A split-K weight gradient (side stream): its f32 slab written, then read by the reduce."""
        self.k(phase, "side", kernel, reads, (), extra_w=slab_mb)
        self.k(phase, "side", kernel.split(" ")[0] + " wgrad_reduce", (), (), extra_r=slab_mb)

    def k(self, phase, stream, kernel, reads=(), writes=(), extra_r=0.0, extra_w=0.0):
        r = {n: self.tensors[n] for n in reads}
        w = {n: self.tensors[n] for n in writes}
        if extra_r:
            r["(slab/partials)"] = extra_r
        if extra_w:
            w["(slab/partials)"] = extra_w
        self.launches.append((phase, stream, kernel, r, w))


def wslab(cin, cout, taps, h, splits_target=1024):
    """f32 split-K slab bytes of a weight gradient (written once, read once by the reduce)."""
    M, N = cout, cin * taps
    tiles = max(1, (M // 128) * max(1, N // 128))
    rows = B * h * h
    splits = max(1, min(-(-splits_target // tiles), -(-rows // 256)))
    return splits * M * N * 4 / MB


def build():
    L = Ledger()
    # ------------------------------------------------------------------ forward
    L.t("x0", 112, 16)                 # s2d input [B,112,112,16]
    L.t("y0", 112, 64)
    L.t("p", 56, 64)
    L.t("arg", 56, 64, 1)
    L.k("fwd", "main", "synth_s2d", (), ("x0",))
    L.k("fwd", "main", "stem_fwd", ("x0",), ("y0",))
    L.k("fwd", "main", "stem_pool", ("y0",), ("p", "arg"))
    h_in, hname = 56, "p"
    cin = 64
    prev = None     # the previous block's tail: (y3, res name, mode, out name, hout, cout)
    blocks = []
    for (si, nb, mid, out, hin, st) in STAGES:
        for bi in range(nb):
            name = f"l{si}.{bi}"
            stride = st if bi == 0 else 1
            hi = h_in
            ho = hi // stride
            ds = bi == 0
            L.t(f"{name}.y1", hi, mid)
            L.t(f"{name}.y2", ho, mid)
            L.t(f"{name}.y3", ho, out)
            # conv1: FWD_TAIL fold of the previous tail when this conv1 has <= 128 channels
            fuse_tail = prev is not None and mid <= 128
            if prev is not None:
                py3, pres, pmask, pout = prev
                if fuse_tail:
                    r = [py3, pres]
                    w = [pout] + ([pmask] if pmask else [])
                    L.k("fwd", "main", f"{name}.conv1 FWD_TAIL", r, w + [f"{name}.y1"])
                else:
                    w = [pout] + ([pmask] if pmask else [])
                    L.k("fwd", "main", f"{prev[0][:-3]}.tail bn_apply", [py3, pres], w)
                    L.k("fwd", "main", f"{name}.conv1", [pout], [f"{name}.y1"])
            else:
                L.k("fwd", "main", f"{name}.conv1", [hname], [f"{name}.y1"])
            xin = hname if prev is None else prev[3]
            if ds:
                L.t(f"{name}.yd", ho, out)
                L.k("fwd", "side", f"{name}.ds conv", [xin], [f"{name}.yd"])
            # bn1: fused into conv2 only for H >= 56 (3x3 consumer), else a1 materialised
            if hi >= 56:
                L.k("fwd", "main", f"{name}.conv2 (pro)", [f"{name}.y1"], [f"{name}.y2"])
                a1 = None
            else:
                L.t(f"{name}.a1", hi, mid)
                L.k("fwd", "main", f"{name}.bn1 apply", [f"{name}.y1"], [f"{name}.a1"])
                L.k("fwd", "main", f"{name}.conv2 HALO" if stride == 1 else f"{name}.conv2",
                    [f"{name}.a1"], [f"{name}.y2"])
                a1 = f"{name}.a1"
            L.k("fwd", "main", f"{name}.conv3 (pro)", [f"{name}.y2"], [f"{name}.y3"])
            if si <= 3:   # forward-time Gram of the folded tail (second stream)
                L.k("fwd", "side", f"{name}.gram", [f"{name}.y2"], [])
            res = f"{name}.yd" if ds else xin
            L.t(f"{name}.out", ho, out)
            mask = None
            if not ds:
                L.t(f"{name}.mask", ho, out // 16)
                mask = f"{name}.mask"
            blocks.append(dict(name=name, si=si, hi=hi, ho=ho, mid=mid, out=out, cin=cin, ds=ds,
                               xin=xin, a1=a1, res=res, mask=mask, stride=stride))
            prev = (f"{name}.y3", res, mask, f"{name}.out")
            h_in, cin = ho, out
    # last tail: pooled
    L.k("fwd", "main", "l4.2.tail_pool", [prev[0], prev[1]], [])
    # ------------------------------------------------------------------ backward
    nbk = len(blocks)
    # last block: standalone tail reduce from the pooled gradient: writes dz
    b = blocks[-1]
    L.t(f"{b['name']}.dz", b["ho"], b["out"])
    L.k("bwd", "main", f"{b['name']}.tail bn_bwd_reduce", [f"{b['name']}.y3", b["res"]],
        [f"{b['name']}.dz"])
    for i in range(nbk - 1, -1, -1):
        b = blocks[i]
        n = b["name"]
        hi, ho, mid, out, si = b["hi"], b["ho"], b["mid"], b["out"], b["si"]
        fold = si <= 3
        dz = f"{n}.dz"
        if b["ds"]:
            L.t(f"{n}.dyd", ho, out)
            L.t(f"{n}.scg", hi, b["cin"])
            if fold:
                L.k("bwd", "main", f"{n}.tail finish + apply(ds)", [dz, f"{n}.yd"], [f"{n}.dyd"])
            else:
                L.t(f"{n}.dy3", ho, out)
                L.k("bwd", "main", f"{n}.tail finish + apply2", [dz, f"{n}.y3", f"{n}.yd"],
                    [f"{n}.dy3", f"{n}.dyd"])
            L.k("bwd", "side", f"{n}.ds dgrad", [f"{n}.dyd"], [f"{n}.scg"])
            L.wg("bwd", f"{n}.ds wgrad", [f"{n}.dyd", b["xin"]], wslab(b["cin"], out, 1, ho))
        elif not fold:
            L.t(f"{n}.dy3", ho, out)
            L.k("bwd", "main", f"{n}.tail finish + apply", [dz, f"{n}.y3"], [f"{n}.dy3"])
        # conv3 (1x1): dgrad -> dz2 (epilogue: relu mask of bn2(y2), partials), wgrad
        L.t(f"{n}.dz2", ho, mid)
        L.t(f"{n}.dy2", ho, mid)
        if fold:
            L.k("bwd", "main", f"{n}.conv3 DGRAD_BNF", [dz, f"{n}.y2"], [f"{n}.dz2"])
            L.wg("bwd", f"{n}.conv3 wgrad (dz^T a2)", [dz, f"{n}.y2"], wslab(mid, out, 1, ho))
        else:
            L.k("bwd", "main", f"{n}.conv3 dgrad", [f"{n}.dy3", f"{n}.y2"], [f"{n}.dz2"])
            L.wg("bwd", f"{n}.conv3 wgrad", [f"{n}.dy3", f"{n}.y2"], wslab(mid, out, 1, ho))
        L.k("bwd", "main", f"{n}.bn2 finish + apply", [f"{n}.dz2", f"{n}.y2"], [f"{n}.dy2"])
        # conv2 (3x3): dgrad -> dz1 (epilogue on y1), wgrad (tap-reuse at 56/28, else generic)
        L.t(f"{n}.dz1", hi, mid)
        L.t(f"{n}.dy1", hi, mid)
        L.k("bwd", "main", f"{n}.conv2 dgrad", [f"{n}.dy2", f"{n}.y1"], [f"{n}.dz1"])
        a1 = b["a1"] or f"{n}.y1"
        L.wg("bwd", f"{n}.conv2 wgrad", [f"{n}.dy2", a1], wslab(mid, mid, 9, ho))
        L.k("bwd", "main", f"{n}.bn1 finish + apply", [f"{n}.dz1", f"{n}.y1"], [f"{n}.dy1"])
        # conv1 (1x1): wgrad; dgrad whose epilogue forms the PREVIOUS tail's dz (+ shortcut grad)
        L.wg("bwd", f"{n}.conv1 wgrad", [f"{n}.dy1", b["xin"]], wslab(b["cin"], mid, 1, hi))
        sc = f"{n}.scg" if b["ds"] else dz
        if i > 0:
            pb = blocks[i - 1]
            pn = pb["name"]
            L.t(f"{pn}.dz", pb["ho"], pb["out"])
            r = [f"{n}.dy1", f"{pn}.y3", sc]
            r += [pb["mask"]] if pb["mask"] else [pb["res"]]
            if pb["ds"]:
                r.append(f"{pn}.yd")
            L.k("bwd", "main", f"{n}.conv1 dgrad (epi: {pn} tail)", r, [f"{pn}.dz"])
        else:
            L.t("dp", 56, 64)
            L.k("bwd", "main", f"{n}.conv1 dgrad", [f"{n}.dy1"], ["dp"])
            stem_sc = sc
    # stem: fused maxpool gather + relu mask + partials (writes dz0), finish (k only), wgrad BNA
    L.t("dz0", 112, 64)
    L.k("bwd", "main", "stem_bwd_reduce", ["dp", stem_sc, "arg", "y0"], ["dz0"])
    L.k("bwd", "main", "stem wgrad BNA", ["dz0", "y0", "x0"], [], extra_w=wslab(16, 64, 16, 112))
    L.k("bwd", "main", "stem wgrad_reduce", (), (), extra_r=wslab(16, 64, 16, 112))
    return L


def report(L: Ledger, md: bool):
    tot = defaultdict(float)
    by_tensor = defaultdict(lambda: {"w": [], "r": []})
    lines = []
    for phase, st, kern, r, w in L.launches:
        rb, wb = sum(r.values()), sum(w.values())
        tot[(phase, st, "r")] += rb
        tot[(phase, st, "w")] += wb
        lines.append((phase, st, kern, rb, wb))
        for n, v in r.items():
            by_tensor[n]["r"].append(kern)
        for n, v in w.items():
            by_tensor[n]["w"].append(kern)
    gr = sum(v for (p, s, k), v in tot.items() if k == "r")
    gw = sum(v for (p, s, k), v in tot.items() if k == "w")
    out = []
    out.append("# Analytic byte ledger of the native ResNet-50 bf16 step (bs 400, 224 px)\n")
    out.append("Generated by `tools/byte_ledger.py` from the default schedule of `models/native.py`. "
               "Activation / gradient bytes per kernel launch (MB = 1e6 B); every tensor charged once "
               "per kernel that touches it; f32 split-K slabs as '(slab/partials)' (written by the "
               "weight gradient, read by its reduce; slab sizes estimated from the split targets).\n")
    out.append("| phase | stream | read GB | write GB |\n|---|---|---|---|")
    for ph in ("fwd", "bwd"):
        for s in ("main", "side"):
            out.append(f"| {ph} | {s} | {tot[(ph, s, 'r')] / 1e3:.2f} | {tot[(ph, s, 'w')] / 1e3:.2f} |")
    out.append(f"| **total** | | **{gr / 1e3:.2f}** | **{gw / 1e3:.2f}** |")
    out.append(f"\nTotal analytic traffic: **{(gr + gw) / 1e3:.1f} GB/step** "
               f"(the calibrated PMC counts every L2 miss, incl. gather re-reads and the "
               f"Infinity-Cache-served ones).\n")
    out.append("## Per launch\n\n| phase | stream | kernel | read MB | write MB |\n|---|---|---|---|---|")
    for phase, st, kern, rb, wb in lines:
        out.append(f"| {phase} | {st} | {kern} | {rb:.0f} | {wb:.0f} |")
    out.append("\n## Per tensor (largest first)\n\n| tensor | MB | writers | readers | moved MB | "
               "minimum MB |\n|---|---|---|---|---|---|")
    rows = []
    for n, d in by_tensor.items():
        if n == "(slab/partials)":
            continue
        size = L.tensors[n]
        moved = size * (len(d["w"]) + len(d["r"]))
        # minimum: one write (unless an input) and one read per consumer kernel that cannot be fused
        # with another consumer of the same tensor in this schedule: what the schedule moves,
        # less the apply-pass write + re-read where a consumer could form the value itself
        rows.append((moved, n, size, d))
    rows.sort(reverse=True)
    for moved, n, size, d in rows:
        out.append(f"| {n} | {size:.0f} | {len(d['w'])} | {len(d['r'])}: "
                   f"{', '.join(k.split(' ', 1)[0] if False else k for k in d['r'])} | {moved:.0f} | |")
    print("\n".join(out))


if __name__ == "__main__":
    report(build(), "--md" in sys.argv)
