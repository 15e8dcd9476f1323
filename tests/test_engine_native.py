"""Host-only unit tests of the native harness (tests/native/engine_test.cc):
schedulers against a mock engine with the reference's cases
(band/test/scheduler_test.cc), model-analyzer partitioning, JSON."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_native_engine_unit_tests():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "band_amd", "csrc"), "engine_test"], check=True,
                   timeout=600)
    r = subprocess.run([os.path.join(ROOT, "tests", "native", "engine_test")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
