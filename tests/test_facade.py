"""The reference's BundleAdjuster tests (src/optim/bundle_adjustment_test.cc)
rerun in C++ through the colmap_amd facade (include/colmap_amd/) on
libmi_ba.so: structural counts on the host, full Solve on the MI355X.  Also
the controllers / iteration callbacks / Reconstruction filters
(tests/cpp/controllers_test.cc: reconstruction_test.cc:415-434,510-531 known
answers, controllers/bundle_adjustment.cc:43-103 callback semantics)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")


def build(name="bundle_adjustment_test"):
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    return os.path.join(CPP, name)


def run(mode, name="bundle_adjustment_test"):
    exe = build(name)
    out = subprocess.run([exe, mode], capture_output=True, text=True, timeout=600)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 failure(s)" in out.stdout
    return out.stdout


def test_facade_counts_cpu():
    out = run("counts")
    assert out.count("PASS") == 16


@pytest.mark.gpu
def test_facade_solve_gpu(gpu):
    out = run("solve")
    assert out.count("PASS") == 16


def test_controllers_host():
    out = run("host", "controllers_test")
    assert out.count("PASS") == 3


@pytest.mark.gpu
def test_controllers_gpu(gpu):
    out = run("gpu", "controllers_test")
    assert out.count("PASS") == 11


def test_sba_reference_signature_host():
    """SemanticBundleAdjuster(options, config) with options.data_path
    (semantic_bundle_adjustment.h:219-225): the TIFF maps read back bitwise,
    a missing map file raised as ReadDepthAndSemanticMaps does."""
    out = run("host", "sba_reference_test")
    assert out.count("PASS") == 2


@pytest.mark.gpu
def test_sba_reference_signature_gpu(gpu):
    """The reference controller's construction + Solve
    (controllers/semantic_bundle_adjustment.cc:100-119) from TIFF files equals
    the in-memory-maps solve bitwise."""
    out = run("gpu", "sba_reference_test")
    assert out.count("PASS") == 3
