"""The analytic byte ledger (tools/byte_ledger.py, profiles/ledger_r6.md): internally consistent and
within the calibrated hardware-counter total of the same step (profiles/pmc_r6_step.md: 106.0 GB)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import byte_ledger as bl  # noqa: E402


def test_ledger_totals_and_tensor_accounting():
    L = bl.build()
    reads = sum(sum(r.values()) for _, _, _, r, _ in L.launches)
    writes = sum(sum(w.values()) for _, _, _, _, w in L.launches)
    total_gb = (reads + writes) / 1e3
    # the analytic count charges each tensor once per kernel: at or below the measured traffic
    # (which also holds re-reads that miss L2 inside a kernel), and not far below it
    assert 90.0 < total_gb < 106.0, total_gb
    # every tensor a launch touches was declared, with its size
    for _, _, kern, r, w in L.launches:
        for name, mb in list(r.items()) + list(w.items()):
            if name.startswith("("):
                assert mb > 0, kern
                continue
            assert name in L.tensors and abs(L.tensors[name] - mb) < 1e-9, (kern, name)
    # activations with a consumer are written before they are read (forward order of the walk);
    # the inputs the step starts from (the batch, the labels' consumers) are exempt
    written = set()
    for _, _, kern, r, w in L.launches:
        for name in r:
            if not name.startswith("(") and name not in written:
                assert name in ("x", "x0", "ids") or name not in {n for *_, ww in L.launches for n in ww}, \
                    (kern, name)
        written.update(w)


def test_ledger_layer1_tensors_have_the_batch_400_sizes():
    L = bl.build()
    # a 256-channel 56x56 bf16 activation at batch 400: 400 * 56 * 56 * 256 * 2 B
    assert abs(bl.T(56, 256) - 642.2528) < 1e-3
    assert any(abs(mb - bl.T(56, 256)) < 1e-6 for mb in L.tensors.values())
