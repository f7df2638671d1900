"""PARITY.md must not rot: every test module / test function and every source file it cites exists."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parity_map_references_exist():
    text = open(os.path.join(ROOT, "PARITY.md")).read()
    missing = []
    for path, fn in re.findall(r"`(tests/[\w/]+\.py)(?:::(\w+)\*?)?`", text):
        full = os.path.join(ROOT, path)
        if not os.path.exists(full):
            missing.append(path)
        elif fn and f"def {fn}" not in open(full).read() and not fn.endswith("_"):
            # `test_bn_*`-style prefixes are written with a trailing '_' before the '*'
            missing.append(f"{path}::{fn}")
    for path in re.findall(r"`(pda/[\w/]+\.(?:py|hip|cpp))", text):
        if not os.path.exists(os.path.join(ROOT, path.replace("pda/", "pytorch_distributed_amd/"))):
            missing.append(path)
    for path in re.findall(r"`((?:tools|profiles)/[\w.]+)`", text):
        if not os.path.exists(os.path.join(ROOT, path)):
            missing.append(path)
    assert not missing, missing


def test_every_runtime_knob_is_documented():
    """Every PDA_* environment variable the package or bench.py reads has a README row."""
    readme = open(os.path.join(ROOT, "README.md")).read()
    table = readme.split("## Runtime knobs", 1)[1].split("\n## ", 1)[0]
    knobs = set()
    files = [os.path.join(ROOT, "bench.py")]
    for d, _, names in os.walk(os.path.join(ROOT, "pytorch_distributed_amd")):
        files += [os.path.join(d, n) for n in names if n.endswith(".py")]
    for f in files:
        knobs |= set(re.findall(r"environ(?:\.get\(|\[)\"(PDA_[A-Z0-9_]+)\"", open(f).read()))
    assert len(knobs) > 15
    assert not sorted(k for k in knobs if f"`{k}`" not in table)
