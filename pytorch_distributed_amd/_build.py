"""In-tree build of the native libraries for gfx950 (no JIT cache, no torch headers).

* ``libpda_kernels.so`` -- every HIP kernel (``csrc/*.hip``), C ABI launchers.
* ``libpda_comm.so``    -- the C++ RCCL communicator and gradient-bucket reducer
  (``csrc/comm/*.cpp``), links ``librccl``.

Both are loaded with ``ctypes`` by :mod:`pytorch_distributed_amd.ops.ext` /
:mod:`pytorch_distributed_amd.parallel.rccl`, so they travel with the repo
snapshot to the GPU box and show up as in-tree ``.so`` files in the process.
Incremental: an object is rebuilt only when its source or a header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
OUT = PKG / "_lib"
BUILD = PKG / "_lib" / "obj"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("PDA_ARCH", "gfx950")

KERNEL_SRCS = ["conv_gemm.hip", "bn.hip", "misc.hip", "stem.hip", "wgrad_tap.hip"]
COMM_SRCS = ["comm/rccl_comm.cpp", "comm/reducer.cpp"]
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result"]


def _newer(src: Path, obj: Path, deps) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return src.stat().st_mtime > t or any(d.stat().st_mtime > t for d in deps)


# per-source flags: the conv kernels keep their operand-prologue math in scalar f32 FMAs, which
# beside MFMAs issue far cheaper than the v_pk_fma_f32 the SLP vectorizer would form
FILE_FLAGS = {"conv_gemm.hip": ["-fno-slp-vectorize"]}


def _compile(src: Path, obj: Path, extra, verbose: bool) -> None:
    cmd = [HIPCC, *CFLAGS, *FILE_FLAGS.get(src.name, []), *extra, "-I", str(CSRC), "-c", str(src),
           "-o", str(obj)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")


def _link(objs, out: Path, libs, verbose: bool) -> None:
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(out), *libs]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {out}\n{r.stdout}\n{r.stderr}")


def _build_lib(name: str, srcs, libs, verbose: bool, jobs: int, extra=()) -> Path:
    OUT.mkdir(parents=True, exist_ok=True)
    BUILD.mkdir(parents=True, exist_ok=True)
    headers = list(CSRC.glob("*.h")) + list(CSRC.glob("comm/*.h"))
    todo = []
    objs = []
    for s in srcs:
        src = CSRC / s
        obj = BUILD / (s.replace("/", "_") + ".o")
        objs.append(obj)
        if _newer(src, obj, headers):
            todo.append((src, obj))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(lambda so: _compile(so[0], so[1], list(extra), verbose), todo))
    out = OUT / name
    if todo or not out.exists() or any(o.stat().st_mtime > out.stat().st_mtime for o in objs):
        _link(objs, out, libs, verbose)
    return out


def build_kernels(verbose: bool = False, jobs: int = 4) -> Path:
    return _build_lib("libpda_kernels.so", KERNEL_SRCS, [], verbose, jobs)


def build_comm(verbose: bool = False, jobs: int = 2) -> Path:
    return _build_lib("libpda_comm.so", COMM_SRCS, [f"-L{ROCM}/lib", "-lrccl", f"-Wl,-rpath,{ROCM}/lib"],
                      verbose, jobs, extra=[f"-I{ROCM}/include"])


def build_all(verbose: bool = False) -> None:
    jobs = min(4, os.cpu_count() or 1)
    build_kernels(verbose, jobs)
    if (CSRC / COMM_SRCS[0]).exists():
        build_comm(verbose)


if __name__ == "__main__":
    build_all(verbose="-v" in sys.argv)
