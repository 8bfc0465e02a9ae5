"""`make -C optimobo_amd/csrc asan` (CPU, no GPU): the host side of the C-ABI under AddressSanitizer + UBSan.

* ``build/asan/omb_host_fuzz``: every entry point's argument checks, the expected-decomposition parameter block and
  the Sobol' state packing (optimobo_amd/csrc/omb_host.cpp, the code the library runs before it touches the device)
  driven with hostile arguments and exactly-sized arrays, return codes against the header's contract
  (tests/asan/omb_host_fuzz.cpp).  It found two signed overflows in round 5's checks (``4 * C`` in the HV-PoI
  cell check, ``k * M`` in the scalarisation check, for C or M near INT_MAX); both now form the product in 64 bits.
* ``build/asan/liboptimobo_hip.so``: the library with omb_api.hip's host code and omb_host.cpp instrumented,
  loaded by tests/test_lib_cpu.py in a child process under LD_PRELOAD of clang's ASan runtime.
"""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "optimobo_amd", "csrc")
CLANGXX = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.fixture(scope="module")
def asan_build():
    if not os.path.exists(CLANGXX) or shutil.which("make") is None:
        pytest.skip("needs ROCm's clang++ and make (the build container)")
    if not os.path.exists(os.path.join(REPO, "optimobo_amd", "liboptimobo_hip.so")):
        pytest.skip("the library is not built (make -C optimobo_amd/csrc)")
    r = subprocess.run(["make", "-C", CSRC, "-j4", "asan"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rt = subprocess.run([CLANGXX, "-print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True, text=True)
    return rt.stdout.strip()


def test_host_checks_fuzz_under_asan_ubsan(asan_build):
    r = subprocess.run([os.path.join(CSRC, "build", "asan", "omb_host_fuzz")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert " 0 mismatches" in r.stdout and "runtime error" not in r.stderr


def test_asan_library_is_instrumented(asan_build):
    lib = os.path.join(CSRC, "build", "asan", "liboptimobo_hip.so")
    out = subprocess.run(["nm", "-D", "--undefined-only", lib], capture_output=True, text=True).stdout
    assert "__asan_report_load8" in out and "__ubsan_handle" in out


def test_lib_cpu_under_asan(asan_build):
    """tests/test_lib_cpu.py (symbols, ABI version, no-GPU refusal) against the sanitized build, plus null-context
    and hostile-argument calls of the k-generic EHVI entry points, in a child process with the ASan runtime first."""
    lib = os.path.join(CSRC, "build", "asan", "liboptimobo_hip.so")
    env = dict(os.environ, LD_PRELOAD=asan_build, OMB_LIB_PATH=lib,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "-x",
                        os.path.join(REPO, "tests", "test_lib_cpu.py")], capture_output=True, text=True, env=env,
                       cwd=REPO, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    snippet = (
        "import ctypes, numpy as np\n"
        "from optimobo_amd import _lib\n"
        f"assert _lib.LIB_PATH == {lib!r}\n"
        "L = _lib.load()\n"
        "c = np.zeros((4, 9))\n"
        "r = _lib.darr(np.ones(9))\n"
        "assert L.omb_plan_ehvi_mc(None, 9, _lib.host_ptr(c), 4, r, 0.0) == _lib.OMB_EINVAL\n"
        "assert L.omb_ehvi_mc(None, 4, None, None, 0, -1, None, 2**31 - 1, r, 0.0, None, None) == _lib.OMB_EINVAL\n"
        "assert L.omb_last_error(None) == b'null context'\n"
        "print('ok')\n")
    r = subprocess.run([sys.executable, "-c", snippet], capture_output=True, text=True, env=env, cwd=REPO, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr[-3000:]
