"""Host-code sanitizers (ASan+UBSan, TSan) over csrc/cpu.cpp (tests/native/host_driver.cpp) and
csrc/host_prep.cpp's worker pool + conversions (tests/native/host_prep_driver.cpp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_host_sanitizers(tmp_path):
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize_host.sh"), str(tmp_path)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("host driver: OK") == 2
    assert r.stdout.count("host prep driver: OK") == 3
