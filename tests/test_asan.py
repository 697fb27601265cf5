"""SURVEY §5 "Race detection / sanitizers": the CPU side under AddressSanitizer.

  * the oracle (oracle/lsr_oracle.c) built with -fsanitize=address,undefined,
    driven by its own CPU test suite (tests/test_oracle.py) in a subprocess with
    gcc's libasan preloaded;
  * the C-ABI driver's host code (csrc/lsr_api.hip compiled with
    -Xarch_host -fsanitize=address, GPU code untouched) driven by
    tools/asan_host_check.py through every validation path, the stage-name
    parser and the profiling tables, with clang's ASan runtime preloaded.
GPU-side ASan is not available on the pool; these run here, without a GPU."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(preload, **kw):
    e = dict(os.environ)
    e.update(LD_PRELOAD=preload, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
             UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", **kw)
    return e


def test_oracle_under_asan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    libubsan = subprocess.run(["gcc", "-print-file-name=libubsan.so"], capture_output=True, text=True).stdout.strip()
    so = os.path.join(ROOT, "oracle", "_build", "liblsr_oracle_asan.so")
    p = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu",
                        os.path.join(ROOT, "tests", "test_oracle.py")],
                       env=_env(f"{libasan}:{libubsan}", LSO_ORACLE_LIB=so), capture_output=True, text=True,
                       timeout=900, cwd=ROOT)
    tail = (p.stdout + p.stderr)[-3000:]
    assert p.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in tail and "runtime error" not in tail
    assert " passed" in p.stdout


def test_host_driver_under_asan():
    rt = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    if not rt:
        pytest.skip("clang ASan runtime not found")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "langsplatv2_amd", "csrc"), "asan"], check=True)
    so = os.path.join(ROOT, "langsplatv2_amd", "_build", "asan", "liblsr.so")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "asan_host_check.py")],
                       env=_env(rt[-1], LSR_LIB=so), capture_output=True, text=True, timeout=300, cwd=ROOT)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-3000:]
    assert "AddressSanitizer" not in out and p.stdout.startswith("ok ")
