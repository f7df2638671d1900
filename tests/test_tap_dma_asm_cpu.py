"""Pins the pipelining of the tap-reuse weight gradients (csrc/wgrad_tap.hip).

Their operands stream into LDS by LDS-DMA several steps ahead, retired by counted
``s_waitcnt vmcnt(N)``. Issued through the ``buffer_load ... lds`` builtin, hipcc tracked each DMA
as a pending LDS store and put an ``s_waitcnt vmcnt(0)`` before the first transposed read of every
step -- draining the whole pipeline each step (in-step 442 -> 366 us once removed,
profiles/ab_r6.md section 15). The kernels now issue the DMA from asm (common.h ``dma16_asm``).
This test reads the gfx950 device assembly: no main loop of a tap kernel (the loop holding its
MFMAs) contains a full ``vmcnt(0)`` drain."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "pytorch_distributed_amd", "csrc")
HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")


@pytest.fixture(scope="module")
def tap_asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("asm") / "wgrad_tap.s"
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                        "-S", "-I", CSRC, os.path.join(CSRC, "wgrad_tap.hip"), "-o", str(out)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return out.read_text().splitlines()


def _functions(lines, pattern):
    out, cur = {}, None
    for l in lines:
        m = re.match(r"^(_Z\S*" + pattern + r"\S*):", l)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur is not None:
            if l.startswith(".Lfunc_end"):
                cur = None
                continue
            out[cur].append(l)
    return out


def _mfma_loops(body):
    """[(header line, body lines)] of every loop (header label .. last branch back to it) that
    holds MFMAs."""
    loops = []
    for i, l in enumerate(body):
        if "Loop Header" not in l:
            continue
        lab = l.split(":")[0].strip()
        back = [k for k, t in enumerate(body) if "branch" in t and t.strip().endswith(lab)]
        if not back:
            continue
        seg = body[min([i] + back):max([i] + back) + 1]   # (a rotated loop branches back from above)
        if sum("v_mfma" in t for t in seg) >= 16:
            loops.append((l.strip(), seg))
    return loops


def test_tap_main_loops_do_not_drain_the_dma_pipeline(tap_asm):
    funcs = _functions(tap_asm, "wgrad(_stem)?_tap_kernel")
    assert len(funcs) >= 6, list(funcs)   # <bf16 / f16> x <plain / BN prologue>, stem x 2
    for sym, body in funcs.items():
        assert any("offen lds" in t for t in body), (sym, "no LDS-DMA")
        loops = _mfma_loops(body)
        assert loops, (sym, "no MFMA loop found")
        for hdr, seg in loops:
            drains = [t.strip() for t in seg if re.search(r"s_waitcnt\s+vmcnt\(0\)", t)]
            assert not drains, (sym, hdr, drains)
