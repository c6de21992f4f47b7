"""AddressSanitizer + UndefinedBehaviorSanitizer run of the library's host code.

tests/native/build_sanitized.sh compiles every libwam_hip.so source host-only with the sanitizers
on the host side, links tests/native/plan_fuzz.cpp against them, and the binary probes host-only
plans (wam_plan_create_host) over odd, tiny, huge and invalid shapes, every level count, filter
length, mode and plan flag, plus the c1-c5 geometries: band layout, reconstruction shapes,
workspace sizes, the fused kernels' support predicates and the refusal of host plans by the
compute entry points. Any sanitizer report aborts the binary (-fno-sanitize-recover). No GPU.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("gcc") is None,
                    reason="needs hipcc and gcc")
def test_host_code_under_asan_ubsan():
    b = subprocess.run(["bash", os.path.join(ROOT, "tests", "native", "build_sanitized.sh")], capture_output=True,
                       text=True, timeout=600)
    assert b.returncode == 0, b.stdout[-2000:] + b.stderr[-4000:]
    exe = b.stdout.strip().splitlines()[-1]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "runtime error" not in out and "ERROR: AddressSanitizer" not in out, out[-4000:]
    assert "0 failed checks" in out
