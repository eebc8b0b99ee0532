"""Native host runtime under AddressSanitizer+UBSan and ThreadSanitizer (CPU only).

GPU sanitizers are not available on the MI355X pool, so the host C++ runtime
(threaded pread/pwrite engine, safetensors index, block gather) is built as a
standalone test executable with ``-fsanitize`` and run here.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _build_and_run(tmp_path, san):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path / f"test_runtime_{san}")
    cmd = [cxx, "-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer", "-D__HIP_PLATFORM_AMD__",
           f"-fsanitize={san}", "-I", os.path.join(ROOT, "csrc", "include"), "-I", os.path.join(ROCM, "include"),
           os.path.join(ROOT, "csrc", "tests", "test_runtime.cpp"), os.path.join(ROOT, "csrc", "runtime", "runtime.cpp"),
           "-L", os.path.join(ROCM, "lib"), f"-Wl,-rpath,{ROCM}/lib", "-lamdhip64", "-lpthread", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        pytest.skip(f"sanitizer build unavailable: {r.stderr[-500:]}")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "runtime host test ok" in r.stdout


def test_runtime_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, "address,undefined")


def test_runtime_tsan(tmp_path):
    _build_and_run(tmp_path, "thread")
