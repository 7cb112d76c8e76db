"""COLMAP model files and float32 TIFF rasters (include/colmap_amd/
model_io.h, tiff.h) on the host, against fixtures written by the reference's
own model writer (tests/golden/make_model_fixture.py runs the reference's
scripts/python/read_write_model.py) and by Pillow/libtiff
(tests/golden/make_tiff_fixtures.py).

  * Reconstruction::ReadBinary / ReadText (reconstruction.cc:1525-1880):
    every camera / image / point / track value equal to the writer's (text:
    the writer's repr round-trips exactly through std::stod)
  * WriteBinary / WriteText (reconstruction.cc:1882-2100) then read back:
    identical model; binary files byte-identical to the reference writer's
    for the same content (cameras, images in id order; qvecs are unit)
  * matrixFromTiff (matrix_vis.h:130-176): raster bitwise equal to the
    encoded float32 array, row 0 = first file row, for uncompressed / LZW /
    PackBits / Deflate strips, big-endian strips, floating-point-predictor
    tiles; an 8-bit file is rejected like the reference (bpp != 32)
  * ReadDepthAndSemanticMaps (semantic_bundle_adjustment.cc:1021-1068):
    <data>/depth_tiff/<stem>_depth.tiff, semantic_tiff/<stem>_semantic.tiff
"""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
CPP = os.path.join(HERE, "cpp")


@pytest.fixture(scope="module")
def exe():
    subprocess.run(["make", "-s", "-C", CPP, "model_io_test"], check=True)
    return os.path.join(CPP, "model_io_test")


def dump(exe, d):
    out = subprocess.run([exe, "dump", d], capture_output=True, text=True, check=True).stdout
    return json.loads(out)


def expected():
    with open(os.path.join(GOLD, "model_small", "expected.json")) as f:
        e = json.load(f)
    return e


def canonical_expected():
    e = expected()
    # the facade reports point3D_id -1 for "no point"; the writer's ids as ints
    return e


@pytest.mark.parametrize("fmt", ["bin", "txt"])
def test_read_reference_written_model(exe, fmt):
    got = dump(exe, os.path.join(GOLD, "model_small", fmt))
    exp = canonical_expected()
    assert got == exp


def test_write_read_roundtrip(exe, tmp_path):
    b, t = tmp_path / "b", tmp_path / "t"
    b.mkdir()
    t.mkdir()
    src = os.path.join(GOLD, "model_small", "bin")
    subprocess.run([exe, "write", src, str(b), str(t)], check=True)
    ref = dump(exe, src)
    for got in (dump(exe, str(b)), dump(exe, str(t))):
        # WriteImages* write NormalizeQuaternion(qvec) (reconstruction.cc:1927-1930,
        # 2024-2027): the qvecs move by rounding only, everything else is equal
        for k, im in ref["images"].items():
            assert np.abs(np.array(got["images"][k][0]) - np.array(im[0])).max() <= 4e-16
            got["images"][k][0] = im[0]
        assert got == ref
    # same bytes as the reference writer where no normalisation applies
    for name in ("cameras.bin", "points3D.bin"):
        with open(os.path.join(src, name), "rb") as f1, open(b / name, "rb") as f2:
            assert f1.read() == f2.read(), name


def test_read_prefers_binary_and_fails_on_missing(exe, tmp_path):
    both = tmp_path / "both"
    shutil.copytree(os.path.join(GOLD, "model_small", "bin"), both)
    for name in os.listdir(os.path.join(GOLD, "model_small", "txt")):
        with open(both / name, "w") as f:
            f.write("# corrupt text files must not be read when .bin exist\n1 NOT_A_MODEL 1 1\n")
    assert dump(exe, str(both)) == canonical_expected()
    r = subprocess.run([exe, "dump", str(tmp_path)], capture_output=True, text=True)
    assert r.returncode == 3 and "do not exist" in r.stdout


def read_tiff(exe, path, tmp_path):
    out = tmp_path / "r.f32"
    r = subprocess.run([exe, "tiff", path, str(out)], capture_output=True, text=True)
    if r.returncode != 0:
        return None, r.stdout
    h, w = map(int, r.stdout.split())
    return np.fromfile(out, np.float32).reshape(h, w), r.stdout


@pytest.mark.parametrize("name", ["depth_none", "depth_lzw", "depth_lzw_strips", "depth_packbits", "depth_deflate",
                                  "depth_be_strips", "depth_tiles_fp", "label_none", "label_lzw", "label_packbits",
                                  "label_deflate"])
def test_tiff_rasters_bitwise(exe, tmp_path, name):
    kind = name.split("_")[0]
    exp = np.load(os.path.join(GOLD, "tiff", "expected_%s.npy" % kind))
    got, msg = read_tiff(exe, os.path.join(GOLD, "tiff", name + ".tiff"), tmp_path)
    assert got is not None, msg
    assert got.shape == exp.shape and np.array_equal(got.view(np.uint32), exp.view(np.uint32))


def test_tiff_rejects_non_float32(exe, tmp_path):
    got, msg = read_tiff(exe, os.path.join(GOLD, "tiff", "label_u8.tiff"), tmp_path)
    assert got is None and "Error loading depth map" in msg


def patch_ifd(src, dst, tag, count=None, value=None):
    """Copy a little-endian classic TIFF, overwriting one IFD entry's count
    and / or value field (malformed-input fixtures made from valid ones)."""
    import struct
    d = bytearray(open(src, "rb").read())
    assert d[:2] == b"II"
    ifd = struct.unpack_from("<I", d, 4)[0]
    n = struct.unpack_from("<H", d, ifd)[0]
    for k in range(n):
        e = ifd + 2 + 12 * k
        if struct.unpack_from("<H", d, e)[0] == tag:
            if count is not None:
                struct.pack_into("<I", d, e + 4, count)
            if value is not None:
                typ = struct.unpack_from("<H", d, e + 2)[0]
                struct.pack_into("<H" if typ == 3 else "<I", d, e + 8, value)
            open(dst, "wb").write(bytes(d))
            return
    raise AssertionError("tag %d not found" % tag)


@pytest.mark.parametrize("case", ["rows_per_strip_0", "huge_entry_count", "huge_size", "lzw_short_expect"])
def test_tiff_malformed_inputs_fail_cleanly(exe, tmp_path, case):
    """Hostile headers end in the loader's error, never a crash or an
    unbounded allocation: RowsPerStrip = 0 (was an integer divide by zero),
    an entry count of 2^30 pointing past the file (was allocated before any
    bounds check), a 2^20 x 2^20 image; and an LZW strip decoded against a
    smaller expected size stops at that size (no unbounded output)."""
    src = os.path.join(GOLD, "tiff", "depth_none.tiff")
    bad = str(tmp_path / "bad.tiff")
    if case == "rows_per_strip_0":
        patch_ifd(src, bad, 278, value=0)
    elif case == "huge_entry_count":
        patch_ifd(src, bad, 273, count=1 << 30)
    elif case == "huge_size":
        patch_ifd(src, bad, 256, value=1 << 20)
        patch_ifd(bad, bad, 257, value=1 << 20)
    else:
        # one LZW strip holding the whole image, the height cut to one row:
        # the strip decodes to more bytes than one row needs
        src = os.path.join(GOLD, "tiff", "depth_lzw.tiff")
        patch_ifd(src, bad, 257, value=1)
        patch_ifd(bad, bad, 278, value=1)
    r = subprocess.run([exe, "tiff", bad, str(tmp_path / "r.f32")], capture_output=True, text=True, timeout=60)
    assert r.returncode >= 0, "crashed with signal %d" % -r.returncode
    if case == "lzw_short_expect":
        exp = np.load(os.path.join(GOLD, "tiff", "expected_depth.npy"))
        got, msg = read_tiff(exe, bad, tmp_path)
        assert got is not None, msg
        assert got.shape == (1, exp.shape[1]) and np.array_equal(got[0].view(np.uint32), exp[0].view(np.uint32))
    else:
        assert r.returncode != 0 and "Error loading depth map" in r.stdout, r.stdout


def test_semantic_maps_layout(exe, tmp_path):
    data = tmp_path / "data"
    (data / "depth_tiff").mkdir(parents=True)
    (data / "semantic_tiff").mkdir()
    model = os.path.join(GOLD, "model_small", "bin")
    names = [v[3] for v in canonical_expected()["images"].values()]
    for n in names:
        stem = n[:n.rfind(".")]
        shutil.copy(os.path.join(GOLD, "tiff", "depth_lzw.tiff"), data / "depth_tiff" / (stem + "_depth.tiff"))
        shutil.copy(os.path.join(GOLD, "tiff", "label_deflate.tiff"),
                    data / "semantic_tiff" / (stem + "_semantic.tiff"))
    r = subprocess.run([exe, "maps", str(data), model], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert r.stdout.split() == ["37", "53", str(len(names)), str(len(names))]
    os.remove(data / "semantic_tiff" / (names[0][:names[0].rfind(".")] + "_semantic.tiff"))
    r = subprocess.run([exe, "maps", str(data), model], capture_output=True, text=True)
    assert r.returncode == 3 and "semantic file" in r.stdout and "does not exist" in r.stdout


def write_text_model(sc, d):
    """A flattened single-model scene as a COLMAP text model (ids = index + 1)."""
    import mi_ba
    os.makedirs(d, exist_ok=True)
    name = {v: k for k, v in {"SIMPLE_PINHOLE": mi_ba.SIMPLE_PINHOLE, "PINHOLE": mi_ba.PINHOLE,
                              "SIMPLE_RADIAL": mi_ba.SIMPLE_RADIAL, "RADIAL": mi_ba.RADIAL,
                              "OPENCV": mi_ba.OPENCV}.items()}[sc.camera_model]
    with open(os.path.join(d, "cameras.txt"), "w") as f:
        for c, prm in enumerate(sc.camera_params):
            f.write("%d %s 1000 1000 %s\n" % (c + 1, name, " ".join(repr(float(v)) for v in prm)))
    pts2d = [[] for _ in range(sc.num_images)]
    tracks = [[] for _ in range(sc.num_points)]
    for k in range(sc.num_obs):
        i, p = int(sc.obs_image[k]), int(sc.obs_point[k])
        tracks[p].append((i + 1, len(pts2d[i])))
        pts2d[i].append((float(sc.obs_xy[k, 0]), float(sc.obs_xy[k, 1]), p + 1))
    with open(os.path.join(d, "images.txt"), "w") as f:
        for i in range(sc.num_images):
            f.write("%d %s %s %d img%d.png\n" % (i + 1, " ".join(repr(float(v)) for v in sc.qvec[i]),
                                                 " ".join(repr(float(v)) for v in sc.tvec[i]),
                                                 int(sc.image_camera[i]) + 1, i))
            f.write(" ".join("%r %r %d" % e for e in pts2d[i]) + "\n")
    with open(os.path.join(d, "points3D.txt"), "w") as f:
        for p in range(sc.num_points):
            if not tracks[p]:
                continue
            f.write("%d %s 0 0 0 0 %s\n" % (p + 1, " ".join(repr(float(v)) for v in sc.xyz[p]),
                                            " ".join("%d %d" % t for t in tracks[p])))


@pytest.mark.gpu
def test_bundle_adjuster_workflow_on_model_files(gpu, exe, tmp_path):
    """read model -> BundleAdjustmentController config -> Solve -> write, and
    the same solve through mi_ba.solve on the flattened arrays."""
    import mi_ba
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 12, 1500, track_length=5, rotation_range=0.05,
                                                 extra=(0.05, 0, 0, 0), seed=11))
    write_text_model(sc, str(tmp_path / "in"))
    (tmp_path / "out").mkdir()
    r = subprocess.run([exe, "ba", str(tmp_path / "in"), str(tmp_path / "out"), "10"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    c0, c1, ns, nu = r.stdout.split()
    ref = sc.copy().gauge()
    s = mi_ba.solve(mi_ba.default_options(max_num_iterations=10), ref)
    assert abs(float(c0) - s.initial_cost) <= 1e-12 * s.initial_cost
    assert abs(float(c1) - s.final_cost) <= 1e-6 * s.final_cost
    out = dump(exe, str(tmp_path / "out"))
    xyz = np.array([out["points3D"][str(p + 1)][0] for p in range(sc.num_points)])
    assert np.abs(xyz - ref.xyz).max() <= 1e-5
    cams = np.array([out["cameras"][str(c + 1)][3] for c in range(sc.num_cameras)])
    assert np.abs(cams - ref.camera_params).max() <= 1e-6 * np.abs(ref.camera_params).max()
