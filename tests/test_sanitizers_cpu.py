"""Host-code sanitizers: build libomeio + a self-test driver with
-fsanitize=address,undefined and run it (no GPU involved)."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.timeout(300)
def test_omeio_asan_ubsan(tmp_path):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None or not Path("/opt/rocm/include/hip/hip_runtime_api.h").exists():
        pytest.skip("no host compiler / HIP headers")
    exe = tmp_path / "omeio_selftest"
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", str(ROOT / "csrc/omeio/omeio.cpp"),
           str(ROOT / "csrc/omeio/xet.cpp"),
           str(ROOT / "csrc/tests/omeio_selftest.cpp"), "-o", str(exe), "-L/opt/rocm/lib", "-lamdhip64",
           "-lcrypto", "-pthread", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, timeout=120,
                       env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1", "UBSAN_OPTIONS": "halt_on_error=1"})
    assert r.returncode == 0 and "selftest OK" in r.stdout, r.stdout + r.stderr[-3000:]
