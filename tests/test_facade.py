"""The reference's BundleAdjuster tests (src/optim/bundle_adjustment_test.cc)
rerun in C++ through the colmap_amd facade (include/colmap_amd/) on
libmi_ba.so: structural counts on the host, full Solve on the MI355X."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")


def build():
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    return os.path.join(CPP, "bundle_adjustment_test")


def run(mode):
    exe = build()
    out = subprocess.run([exe, mode], capture_output=True, text=True, timeout=600)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 failure(s)" in out.stdout
    return out.stdout


def test_facade_counts_cpu():
    out = run("counts")
    assert out.count("PASS") == 15


@pytest.mark.gpu
def test_facade_solve_gpu(gpu):
    out = run("solve")
    assert out.count("PASS") == 15
