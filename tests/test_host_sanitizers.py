"""Host-only library code under AddressSanitizer + UndefinedBehaviorSanitizer
("Race detection / sanitizers": host tests; GPU sanitizers are not
available on the pool).  tests/cpp/host_sanitize.cc drives the mesh
generator (host/mesh.cc) and brick discovery (csrc/brick_discovery.cc),
compiled here by the ROCm clang for the host only; any report fails."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.mark.skipif(not os.path.exists(CLANG), reason="ROCm clang++ not installed")
def test_host_code_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_sanitize")
    cmd = [CLANG, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-D__HIP_PLATFORM_AMD__",
           "-I/opt/rocm/include", "-I" + os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cpp", "host_sanitize.cc"),
           os.path.join(ROOT, "dealii-ns-gls_amd", "host", "mesh.cc"),
           os.path.join(ROOT, "dealii-ns-gls_amd", "csrc", "brick_discovery.cc"), "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-3000:]
    assert "0 failures" in out
