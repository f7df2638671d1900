"""Host-side sanitizer runs of the native communicator + gradient-bucket reducer (SURVEY §5.2 race
detection, §5.3 failure detection), on the CPU.

``csrc/comm/rccl_comm.cpp`` and ``csrc/comm/reducer.cpp`` -- the exact sources of
``libpda_comm.so`` -- are compiled with g++ against a host stub of the HIP/RCCL calls they use
(``csrc/comm/hoststub/``), whose collectives run across threads, and driven by
``hoststub/harness.cpp`` with world sizes 2-8 (8 = the driver's one-node scaling run and
resnet_dp.py's node): bucket sequencing under rank-specific readiness
patterns, reset, the communicator closed before its reducer, a dead peer with the watchdog
aborting while another thread is blocked inside a bucket all-reduce, bad arguments, and the
in-process DataParallel group. Run twice: AddressSanitizer + UBSan (+ LeakSanitizer), and
ThreadSanitizer."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMM = os.path.join(ROOT, "pytorch_distributed_amd", "csrc", "comm")
SRCS = ["rccl_comm.cpp", "reducer.cpp", "hoststub/stub_runtime.cpp", "hoststub/harness.cpp"]

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


def _build_and_run(tmp_path, name, flags, env):
    exe = str(tmp_path / name)
    cmd = ["g++", "-std=c++17", "-g", "-O1", "-fno-omit-frame-pointer", *flags,
           "-I", os.path.join(COMM, "hoststub"), "-I", COMM,
           *[os.path.join(COMM, s) for s in SRCS], "-o", exe, "-lpthread"]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if b.returncode != 0 and "sanitizer" in (b.stderr or "").lower() and "cannot find" in b.stderr:
        pytest.skip(f"sanitizer runtime unavailable: {b.stderr[-300:]}")
    assert b.returncode == 0, b.stderr[-3000:]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=180,
                       env={**os.environ, **env})
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "ALL PASS" in r.stdout
    for s in ("multi_rank_average world 4", "multi_rank_average world 8",
              "destroy_comm_before_reducer", "abort_while_enqueuing", "bad_arguments", "collectives",
              "dp_group 4 devices", "dp_group 8 devices"):
        assert f"PASS {s}" in r.stdout
    assert "ERROR: AddressSanitizer" not in out and "WARNING: ThreadSanitizer" not in out
    return out


def test_comm_reducer_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, "h_asan", ["-fsanitize=address,undefined",
                                        "-fno-sanitize-recover=undefined"],
                   {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
                    "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})


def test_comm_reducer_tsan(tmp_path):
    _build_and_run(tmp_path, "h_tsan", ["-fsanitize=thread"],
                   {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"})
