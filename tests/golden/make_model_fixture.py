"""Writes tests/golden/model_small/{bin,txt}/ with the reference's own model
writer (scripts/python/read_write_model.py of the reference checkout, run
here in the build container only) and expected.json with the model's
contents; tests/test_model_io.py reads both formats with
include/colmap_amd/model_io.h and compares.  Re-run:
    python3 tests/golden/make_model_fixture.py /root/reference
"""
import json
import os
import sys

import numpy as np

ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
sys.path.insert(0, os.path.join(ref, "scripts", "python"))
import read_write_model as rwm  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "model_small")
rng = np.random.default_rng(7)

cameras = {
    1: rwm.Camera(id=1, model="SIMPLE_RADIAL", width=640, height=480, params=np.array([500.5, 320.0, 240.0, 0.0125])),
    2: rwm.Camera(id=2, model="PINHOLE", width=800, height=600, params=np.array([610.0, 612.5, 400.0, 300.0])),
    5: rwm.Camera(id=5, model="OPENCV", width=1024, height=768,
                  params=np.array([700.0, 701.0, 512.0, 384.0, -0.1, 0.01, 1e-4, -2e-4])),
}
P = 12
xyz = rng.normal(0, 1, (P, 3))
images, tracks = {}, {p: [] for p in range(1, P + 1)}
for k, (iid, cid) in enumerate([(1, 1), (2, 2), (4, 5), (7, 1)]):
    q = rng.normal(0, 1, 4)
    q /= np.linalg.norm(q)
    n2d = 9
    xys = rng.uniform(0, 500, (n2d, 2))
    ids = np.full(n2d, -1, np.int64)
    for j in range(n2d):
        if (j + k) % 3 != 0:
            pid = 1 + (j + 2 * k) % P
            ids[j] = pid
            tracks[pid].append((iid, j))
    images[iid] = rwm.Image(id=iid, qvec=q, tvec=rng.normal(0, 2, 3), camera_id=cid, name="img_%02d.png" % iid,
                            xys=xys, point3D_ids=ids)
images[4] = images[4]._replace(xys=np.zeros((0, 2)), point3D_ids=np.zeros(0, np.int64))  # an image without points
for t in tracks.values():
    t[:] = [e for e in t if e[0] != 4]
points = {}
for p in range(1, P + 1):
    if not tracks[p]:
        continue
    points[p] = rwm.Point3D(id=p, xyz=xyz[p - 1], rgb=rng.integers(0, 256, 3).astype(np.uint8),
                            error=float(rng.uniform(0, 2)), image_ids=np.array([e[0] for e in tracks[p]]),
                            point2D_idxs=np.array([e[1] for e in tracks[p]]))

for ext, sub in ((".bin", "bin"), (".txt", "txt")):
    d = os.path.join(OUT, sub)
    os.makedirs(d, exist_ok=True)
    rwm.write_model(cameras, images, points, d, ext=ext)

names = {m.model_name: m.model_id for m in rwm.CAMERA_MODELS}
expected = {
    "cameras": {str(c.id): [names[c.model], c.width, c.height, [float(v) for v in c.params]] for c in cameras.values()},
    "images": {str(i.id): [[float(v) for v in i.qvec], [float(v) for v in i.tvec], i.camera_id, i.name,
                           [[float(x), float(y), int(pid)] for (x, y), pid in zip(i.xys, i.point3D_ids)]]
               for i in images.values()},
    "points3D": {str(p.id): [[float(v) for v in p.xyz], [int(v) for v in p.rgb], float(p.error),
                             [[int(a), int(b)] for a, b in zip(p.image_ids, p.point2D_idxs)]] for p in points.values()},
}
with open(os.path.join(OUT, "expected.json"), "w") as f:
    json.dump(expected, f, indent=1, sort_keys=True)
print("wrote", OUT)
