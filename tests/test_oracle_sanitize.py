"""The oracle under AddressSanitizer + UndefinedBehaviorSanitizer (host code)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_asan_ubsan():
    odir = os.path.join(ROOT, "oracle")
    subprocess.run(["make", "-s", "-C", odir, "oracle_asan"], check=True)
    env = dict(os.environ, UBSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1")
    out = subprocess.run([os.path.join(odir, "oracle_asan")], capture_output=True, text=True, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad=0" in out.stdout
