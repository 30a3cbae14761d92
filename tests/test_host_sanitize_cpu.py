"""CPU sanitizer build of the C ABI's host logic (the "CPU sanitizer build" of the aux list).

Every dl4ss_amd/csrc/*.hip is compiled host-only (--cuda-host-only: no device code) with
AddressSanitizer + UBSan, linked with tests/sanitize/host_abi_check.cpp and run with
halt_on_error: the recurrence planner over a grid of (cell, B, H, precision, budget) with its
invariants, the GEMM workspace queries, and the argument validation of the compute entry points
(which must fail before any device call).  Builds into a temporary directory, never the tree."""
import os
import shutil
import subprocess
import tempfile
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dl4ss_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
       "-Xarch_host", "-fno-sanitize-recover=undefined"]
# host-only objects in relocatable-device-code form: the link's (empty) device link then supplies the
# fat binary every translation unit's registration references
FLAGS = ["-O1", "-g", "-fPIC", "-std=c++17", "--offload-arch=gfx950", "--cuda-host-only", "-fgpu-rdc",
         "-Wno-unused-result", "-Wno-undefined-internal", "-I", CSRC, *SAN]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_host_abi_under_asan_ubsan():
    with tempfile.TemporaryDirectory() as td:
        srcs = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))

        def comp(f):
            o = os.path.join(td, f[:-4] + ".o")
            r = subprocess.run([HIPCC, *FLAGS, "-c", os.path.join(CSRC, f), "-o", o], capture_output=True, text=True)
            assert r.returncode == 0, (f, r.stderr[-2000:])
            return o

        with ThreadPoolExecutor(4) as ex:
            objs = list(ex.map(comp, srcs))
        drv = os.path.join(ROOT, "tests", "sanitize", "host_abi_check.cpp")
        dro = os.path.join(td, "host_abi_check.o")
        exe = os.path.join(td, "host_abi_check")
        # the driver is plain C++ (the header is C): compiled apart, then one hipcc link of objects only
        r = subprocess.run([CLANG, "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-c", drv, "-o", dro],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-2000:]
        r = subprocess.run([HIPCC, "-fgpu-rdc", "--offload-arch=gfx950", *SAN, dro, *objs, "-o", exe],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-2000:]
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0",
                   UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", HIP_VISIBLE_DEVICES="")
        r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
        assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
        assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
