"""float32 TIFF fixtures for include/colmap_amd/tiff.h (MatrixFromTiff,
restating matrixFromTiff, src/util/matrix_vis.h:130-176).  Writers: Pillow
(libtiff) for the common encodings, plus hand-built files for big-endian,
tiled and floating-point-predictor layouts.  expected.npy holds the raster
every file encodes (row 0 = the first row in the file), as float32.
Re-run: python3 tests/golden/make_tiff_fixtures.py
"""
import os
import struct

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "tiff")
os.makedirs(OUT, exist_ok=True)

H, W = 37, 53  # ragged against strips and tiles
rng = np.random.default_rng(3)
depth = (rng.uniform(0.5, 30.0, (H, W))).astype(np.float32)
depth[5, :] = 0.0          # a row without depth (skipped by the sampler)
depth[:, 7] = np.float32(1e-5)
labels = rng.integers(0, 20, (H, W)).astype(np.float32)
np.save(os.path.join(OUT, "expected_depth.npy"), depth)
np.save(os.path.join(OUT, "expected_label.npy"), labels)

for name, comp in (("none", None), ("lzw", "tiff_lzw"), ("packbits", "packbits"), ("deflate", "tiff_adobe_deflate")):
    kw = {} if comp is None else {"compression": comp}
    Image.fromarray(depth, mode="F").save(os.path.join(OUT, "depth_%s.tiff" % name), **kw)
    Image.fromarray(labels, mode="F").save(os.path.join(OUT, "label_%s.tiff" % name), **kw)
# a multi-strip LZW file
Image.fromarray(depth, mode="F").save(os.path.join(OUT, "depth_lzw_strips.tiff"), compression="tiff_lzw",
                                      tiffinfo={278: 4})


def classic_tiff(path, be, entries, blocks):
    """entries: list of (tag, type, values); blocks: list of byte strings
    (StripOffsets/TileOffsets patched to point at them)."""
    e = ">" if be else "<"
    n = len(entries)
    ifd_off = 8
    data_off = ifd_off + 2 + 12 * n + 4
    extra = b""
    offs = []
    pos = data_off
    for b in blocks:
        offs.append(pos)
        extra += b
        pos += len(b)
    out_entries = []
    tail = b""
    for tag, typ, vals in entries:
        if tag in (273, 324):
            vals = offs
        size = 2 if typ == 3 else 4
        fmt = "H" if typ == 3 else "I"
        raw = b"".join(struct.pack(e + fmt, v) for v in vals)
        if len(raw) <= 4:
            out_entries.append(struct.pack(e + "HHI", tag, typ, len(vals)) + raw.ljust(4, b"\0"))
        else:
            out_entries.append(struct.pack(e + "HHII", tag, typ, len(vals), pos + len(tail)))
            tail += raw
    head = (b"MM" if be else b"II") + struct.pack(e + "HI", 42, ifd_off)
    ifd = struct.pack(e + "H", n) + b"".join(out_entries) + struct.pack(e + "I", 0)
    with open(path, "wb") as f:
        f.write(head + ifd + extra + tail)


def fp_predict(rows, be_unused=None):
    """TIFF floating-point predictor (3): per row, MSB byte plane first, bytes differenced."""
    out = []
    for r in rows:
        b = r.astype(">f4").tobytes()
        n = len(r)
        planes = bytes(b[4 * c + k] for k in range(4) for c in range(n))
        arr = np.frombuffer(planes, np.uint8).astype(np.int32)
        d = np.concatenate([[arr[0]], np.diff(arr)]) % 256
        out.append(d.astype(np.uint8).tobytes())
    return b"".join(out)


base = [(256, 4, [W]), (257, 4, [H]), (258, 3, [32]), (259, 3, [1]), (262, 3, [1]), (277, 3, [1]),
        (339, 3, [3])]
# big-endian, uncompressed, 3 strips of 16 rows
strips = [depth[s:s + 16] for s in range(0, H, 16)]
classic_tiff(os.path.join(OUT, "depth_be_strips.tiff"), True,
             base + [(273, 4, [0] * len(strips)), (278, 4, [16]),
                     (279, 4, [s.size * 4 for s in strips])],
             [s.astype(">f4").tobytes() for s in strips])
# little-endian, 16 x 16 tiles (edge tiles padded), floating-point predictor
TW = TH = 16
tiles = []
for ty in range(0, H, TH):
    for tx in range(0, W, TW):
        t = np.zeros((TH, TW), np.float32)
        blk = depth[ty:ty + TH, tx:tx + TW]
        t[:blk.shape[0], :blk.shape[1]] = blk
        tiles.append(fp_predict(list(t)))
classic_tiff(os.path.join(OUT, "depth_tiles_fp.tiff"), False,
             base + [(317, 3, [3]), (322, 4, [TW]), (323, 4, [TH]), (324, 4, [0] * len(tiles)),
                     (325, 4, [len(t) for t in tiles])], tiles)
# 8-bit image: rejected like the reference (bpp != 32)
Image.fromarray((labels * 10).astype(np.uint8), mode="L").save(os.path.join(OUT, "label_u8.tiff"))
print("wrote", OUT)
