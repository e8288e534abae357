"""ASan + UBSan over the CPU-side code (after the reference's
configure --toolchain=*-asan/-usan): `make -C oracle sanitize` builds the
oracle, csrc/synth.c and the 2-pass host arithmetic with both sanitizers,
and tests/sanitize_run.py drives them in a child Python with the ASan
runtime preloaded.  Any sanitizer report fails the test."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "oracle", "_asan")
CLANG = "/opt/rocm/llvm/bin/clang"


@pytest.mark.skipif(not os.path.exists(CLANG), reason="ROCm clang (sanitizer runtime) not present")
def test_cpu_code_under_asan_and_ubsan():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"])
    rt = subprocess.check_output([CLANG, "-print-file-name=libclang_rt.asan-x86_64.so"], text=True).strip()
    env = dict(os.environ,
               LD_PRELOAD=rt,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               FFV1_ORACLE_LIB=os.path.join(ASAN, "libffv1_oracle.so"),
               FFV1HIP_SYNTH_LIB=os.path.join(ASAN, "libffv1synth.so"),
               FFV1HIP_TWOPASS_LIB=os.path.join(ASAN, "libffv1twopass.so"))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "sanitize_run.py")], env=env,
                       capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in out, out[-4000:]
    assert "runtime error:" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert "sanitize run done" in r.stdout
