"""Host-side AddressSanitizer run of the C ABI ("-fsanitize=address host build of
the C ABI").  Builds libvitmi with ASan on the host code only (`make asan`: -Xarch_host
-fsanitize=address; GPU ASan is not available on this pool) and runs tests/asan/abi_driver.c
against it: every host-only path (argument validation, workspace queries, conv geometry,
resize tables, comm entry points without a communicator, the work table).  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "transformer-stm_amd")
CLANG = "/opt/rocm/lib/llvm/bin/clang"


@pytest.mark.timeout(600)
def test_abi_host_paths_under_asan(tmp_path):
    if not (shutil.which("make") and os.path.exists(CLANG)):
        pytest.skip("needs make and the ROCm clang")
    subprocess.run(["make", "-C", PKG, "asan", "-j8"], check=True, capture_output=True, timeout=540)
    exe = str(tmp_path / "abi_driver")
    libdir = os.path.join(PKG, "build-asan")
    subprocess.run([CLANG, "-g", "-fsanitize=address", "-fno-omit-frame-pointer",
                    os.path.join(ROOT, "tests", "asan", "abi_driver.c"), "-o", exe, "-L" + libdir, "-lvitmi_asan",
                    "-Wl,-rpath," + libdir, "-Wl,-rpath,/opt/rocm/lib"], check=True, timeout=120)
    # leak checking off: the HIP runtime keeps process-lifetime allocations
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0")
    r = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "AddressSanitizer" not in r.stderr, r.stderr
    assert "all checks passed" in r.stdout
