"""Pins the instruction lowering the ``bn_stats_kernel`` hand-off relies on (csrc/bn.hip:221-246).

The blocks of a statistics group publish their slab with relaxed agent-scope stores (``st_wt``),
drain them (``s_waitcnt vmcnt(0)``), then bump a relaxed agent-scope counter; the last arriver runs
an agent-scope acquire fence and reads the slabs with plain loads. Under the HIP/LLVM memory model
alone that is not a release/acquire pair: it is correct on gfx950 because a relaxed agent-scope
store lowers to a write-through ``sc1`` store (it reaches the coherent level before vmcnt drops)
and the acquire fence lowers to ``buffer_inv sc1`` (the reader's stale L2/L1 lines are dropped).
A compiler that lowered either differently would silently corrupt BatchNorm statistics, and the
numerics tests could miss it, so this test reads the gfx950 device assembly: every
instantiation's slab stores carry ``sc1``, a ``vmcnt(0)`` drain sits between them and the counter
atomic, and a ``buffer_inv sc1`` sits between the atomic and the first load after it."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "pytorch_distributed_amd", "csrc")
HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")


@pytest.fixture(scope="module")
def bn_asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("asm") / "bn.s"
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                        "-S", "-I", CSRC, os.path.join(CSRC, "bn.hip"), "-o", str(out)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return out.read_text().splitlines()


def _bodies(lines, name):
    """{symbol: [instruction lines]} of every instantiation of kernel ``name``."""
    out, cur = {}, None
    for l in lines:
        m = re.match(r"^(_Z\S*" + name + r"\S*):", l)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur is not None:
            if l.startswith(".Lfunc_end") or l.strip().startswith(".size"):
                cur = None
                continue
            t = l.strip()
            if t and not t.startswith((";", ".")):
                out[cur].append(t)
    return out


def test_bn_stats_handoff_lowering(bn_asm):
    bodies = _bodies(bn_asm, "bn_stats_kernel")
    assert len(bodies) >= 3, list(bodies)
    for sym, ins in bodies.items():
        atom = [i for i, t in enumerate(ins) if t.startswith("global_atomic_add")]
        assert len(atom) == 1, (sym, "one arrival atomic", atom)
        a = atom[0]
        slab_stores = [i for i, t in enumerate(ins[:a]) if t.startswith("global_store_dwordx2")]
        assert slab_stores, (sym, "slab stores before the arrival")
        for i in slab_stores:
            assert re.search(r"\bsc1\b", ins[i]), (sym, "slab store not write-through", ins[i])
        last = slab_stores[-1]
        assert any(t.startswith("s_waitcnt") and "vmcnt(0)" in t for t in ins[last:a]), \
            (sym, "no vmcnt(0) drain between the slab stores and the arrival")
        after = ins[a + 1:]
        inv = next((i for i, t in enumerate(after) if t.startswith("buffer_inv") and "sc1" in t), None)
        assert inv is not None, (sym, "no buffer_inv sc1 after the arrival")
        first_load = next((i for i, t in enumerate(after) if t.startswith("global_load")), None)
        assert first_load is None or inv < first_load, \
            (sym, "a slab load precedes the acquire invalidate")
