"""ASan + UBSan run of the host-side C++: the CPU oracle, the FreeGraph builder
of the C-ABI and the shared sampler header, built into one instrumented executable
(tests/sanitize_main.cpp) with g++ and run on the CPU. No GPU code is instrumented (GPU
sanitizers are not available on this pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_code_under_address_and_undefined_behaviour_sanitizers(tmp_path):
    exe = tmp_path / "sanitize_main"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-ffp-contract=off", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           os.path.join(ROOT, "tests", "sanitize_main.cpp"), "-o", str(exe), "-lpthread"]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "sanitize ok" in r.stdout
    assert "runtime error" not in r.stderr
