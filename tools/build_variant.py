"""Build an A/B variant of the kernel library from a git revision of one or more sources.

    python tools/build_variant.py NAME REF|DIR [file ...]   (files default to csrc/conv_gemm.hip)

Writes pytorch_distributed_amd/_lib/ab/libpda_kernels_NAME.so: the listed sources are taken
from git REF, the rest from the working tree. Select it at run time with
PDA_KERNEL_LIB=ab/libpda_kernels_NAME.so, so that two variants can be timed back to back on
ONE device in one call (cdna_hip_programming.md §5.4 rule 24)."""
import os
import subprocess
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from pytorch_distributed_amd import _build  # noqa: E402


def main():
    name, ref = sys.argv[1], sys.argv[2]
    files = sys.argv[3:] or ["conv_gemm.hip"]
    out = _build.OUT / "ab"
    out.mkdir(parents=True, exist_ok=True)
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        objs = []
        for src in _build.KERNEL_SRCS:
            if src in files:
                if os.path.isdir(ref):   # a directory holding the variant sources
                    text = (Path(ref) / src).read_text()
                else:
                    text = subprocess.run(["git", "show", f"{ref}:pytorch_distributed_amd/csrc/{src}"],
                                          capture_output=True, text=True, check=True).stdout
                s = td / src
                s.write_text(text)
            else:
                s = _build.CSRC / src
            o = td / (src + ".o")
            _build._compile(s, o, [], verbose=False)
            objs.append(o)
        lib = out / f"libpda_kernels_{name}.so"
        _build._link(objs, lib, [], verbose=False)
    print(lib)


if __name__ == "__main__":
    main()
