"""Exact probe arithmetic of the kernels (sketch_common.h), checked on the
host: fastmod vs %, incremental probe stepping vs (a + i*b) mod 2^64 mod bits
including 64-bit wraparound, and hllPatLen."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_arith(tmp_path):
    src = os.path.join(ROOT, "tests", "native", "host_arith.cpp")
    exe = str(tmp_path / "host_arith")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-o", exe, src], check=True)
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad=0" in out.stdout
