"""CPU tests of the C-ABI boundary: the product library builds for gfx950,
loads, exports every symbol include/*.h declares, keeps the reference's
option defaults and error conventions — with no compute calls (no GPU here).
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import mi_ba

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mi_ba_[a-z0-9_]+)\s*\(", text)))


def exported(lib_path):
    out = subprocess.run(["nm", "-D", "--defined-only", lib_path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_product_exports_every_declared_symbol():
    syms = declared_symbols("mi_ba.h")
    assert len(syms) >= 20
    have = exported(mi_ba.LIB_PATH)
    missing = [s for s in syms if s not in have]
    assert not missing, missing
    lib = mi_ba.load()
    for s in syms:
        getattr(lib, s)


def test_synthetic_exports_every_declared_symbol():
    syms = declared_symbols("mi_ba_synthetic.h")
    have = exported(mi_ba.SYNTH_PATH)
    assert all(s in have for s in syms), syms


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", mi_ba.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert ".hip_fatbin" in out
    data = open(mi_ba.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_product_library_ships_no_ab_variants():
    """The measured-slower A/B kernel variants are compiled into the
    tools-only build (make ab -> libmi_ba_ab.so) and not into the product
    library: its code object holds none of their kernels."""
    prod = os.path.join(os.path.dirname(mi_ba.__file__), "libmi_ba.so")
    data = open(prod, "rb").read()
    for name in (b"schur_pairs_pipelined_kernel", b"semantic_linearize_kernel", b"panel_factor_kernelILi1E",
                 b"13fblock_kernelI"):
        assert name not in data, name
    assert b"semantic_flat_kernel" in data and b"schur_pairs_kernel" in data


def test_default_options_match_reference():
    # BundleAdjustmentOptions() (bundle_adjustment.h:49-92) + Ceres 2.1 defaults
    o = mi_ba.default_options()
    assert o.loss_function_type == mi_ba.LOSS_TRIVIAL and o.loss_function_scale == 1.0
    assert (o.refine_focal_length, o.refine_principal_point, o.refine_extra_params, o.refine_extrinsics) == (1, 0, 1, 1)
    assert o.max_num_iterations == 100 and o.max_linear_solver_iterations == 200
    assert o.function_tolerance == 0.0 and o.gradient_tolerance == 0.0 and o.parameter_tolerance == 0.0
    assert o.max_num_consecutive_invalid_steps == 10
    assert o.eta == 0.1 and o.initial_trust_region_radius == 1e4 and o.min_relative_decrease == 1e-3


def test_abi_version_and_params():
    lib = mi_ba.load()
    assert lib.mi_ba_abi_version() == 4
    for m, n in mi_ba.NUM_PARAMS.items():
        assert lib.mi_ba_num_params(m) == n
    assert lib.mi_ba_num_params(99) == -1
    assert lib.mi_ba_status_string(mi_ba.ERR_NO_DEVICE).decode().startswith("no HIP device")


def test_product_refuses_without_device_or_fails_loudly():
    """No CPU fallback: without an MI355X every compute entry returns NO_DEVICE."""
    if mi_ba.device_count() > 0:
        pytest.skip("a device is visible")
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 2, 20)).gauge()
    with pytest.raises(mi_ba.MiBaError) as e:
        mi_ba.solve(mi_ba.default_options(), sc)
    assert e.value.status == mi_ba.ERR_NO_DEVICE
    with pytest.raises(mi_ba.MiBaError) as e:
        mi_ba.Context(mi_ba.default_options(), sc)
    assert e.value.status == mi_ba.ERR_NO_DEVICE


def test_setup_error_conventions():
    """glog CHECK / std::domain_error of the reference become status codes."""
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 2, 20))
    bad = sc.copy()
    bad.camera_model = 42
    with pytest.raises(mi_ba.MiBaError) as e:
        mi_ba.setup_stats(mi_ba.default_options(), bad)
    assert e.value.status == mi_ba.ERR_UNSUPPORTED
    bad = sc.copy()
    bad.image_constant_pose = np.array([1, 0], np.uint8)
    bad.image_constant_tvec = np.array([1, 0], np.uint8)  # SetConstantTvec on a constant-pose image
    with pytest.raises(mi_ba.MiBaError) as e:
        mi_ba.setup_stats(mi_ba.default_options(), bad)
    assert e.value.status == mi_ba.ERR_INVALID_ARGUMENT
    bad = sc.copy()
    bad.obs_point = bad.obs_point.copy()
    bad.obs_point[0] = 10_000
    with pytest.raises(mi_ba.MiBaError) as e:
        mi_ba.setup_stats(mi_ba.default_options(), bad)
    assert e.value.status == mi_ba.ERR_INVALID_ARGUMENT
    with pytest.raises(mi_ba.MiBaError) as e:
        mi_ba.setup_stats(mi_ba.default_options(loss_function_scale=-1.0), sc)
    assert e.value.status == mi_ba.ERR_INVALID_ARGUMENT


def test_synthetic_reference_generator_shape():
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 3, 100))
    assert sc.num_obs == 300
    assert np.all(sc.tvec[:, 2] == 10) and np.all(np.abs(sc.tvec[:, :2]) <= 1)
    assert np.all(np.abs(sc.xyz) <= 1)
    assert np.all(sc.camera_params == [1200, 500, 500, 0])
    assert np.all(sc.qvec == [1, 0, 0, 0])
    sc2 = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.OPENCV, 20, 1000, track_length=10, rotation_range=0.05))
    assert sc2.num_obs == 10_000
    counts = np.bincount(sc2.obs_point)
    assert np.all(counts == 10)
    for p in range(0, 1000, 97):
        imgs = sc2.obs_image[sc2.obs_point == p]
        assert len(set(imgs.tolist())) == 10
