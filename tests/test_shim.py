"""include/OsqpEigen/OsqpEigen.h -- the OsqpEigen-compatible C++ front end -- driven with the
mpcPlanner::solveTraj call sequence (reference mpcPlanner.cpp:436-527) by tests/native/shim_test.cpp
(compiled against a test-only Eigen stand-in, since Eigen is not in this image)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "build", "shim_test")


def run(mode):
    p = subprocess.run([EXE, mode], capture_output=True, text=True, timeout=120)
    return p.returncode, p.stdout + p.stderr


def test_shim_conversion_and_no_device_behaviour():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible: the no-device path is not reachable")
    rc, out = run("cpu")
    assert rc == 0, out
    assert "no HIP device" in out  # fails loudly: no CPU fallback


@pytest.mark.gpu
def test_shim_solves_on_gpu():
    rc, out = run("gpu")
    assert rc == 0, out
