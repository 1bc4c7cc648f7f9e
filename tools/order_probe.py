"""Experiment: does dequeuing expensive pixels first remove the small-launch
tail?  Classifies C3 pixels by the first object their centre ray meets
(numpy, approximate CSG: spheres only) and renders the frame at SPP in natural
order and in class order (mirror, glass, diffuse, sky).  usage: order_probe.py SPP"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "path-trace_amd"))
import pathtrace as pt  # noqa: E402
from pathtrace import scenes  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 16
W, H = 1920, 1080
S = np.array([[-1, 0, -4, .6, 2], [-.5, 0, -4, .6, 2], [-.7, .3, -3.6, .4, 2], [1, 0, -4, .6, 1],
              [1.4, .2, -4.2, .5, 0], [1, 0, -3.4, .3, 1]])  # class: 0 mirror, 1 glass, 2 diffuse
ys, xs = np.mgrid[0:H, 0:W]
d = np.stack([(2 * (xs + .5) / W - 1) * W, (1 - 2 * (ys + .5) / H) * H, -np.full(xs.shape, 2.0 * H)], -1)
d = d / np.linalg.norm(d, axis=-1, keepdims=True)
best = np.full(xs.shape, np.inf)
cls = np.full(xs.shape, 3)
for cx, cy, cz, r, c in S:
    b = d @ np.array([-cx, -cy, -cz])
    disc = b * b - (cx * cx + cy * cy + cz * cz - r * r)
    t = -b - np.sqrt(np.maximum(disc, 0))
    hit = (disc > 0) & (t > 0) & (t < best)
    best = np.where(hit, t, best)
    cls = np.where(hit, c, cls)
pix = np.arange(W * H, dtype=np.int32)
order = pix[np.argsort(cls.reshape(-1), kind="stable")]
ds = pt.DeviceScene(scenes.scene_p1())
res = {}
for name, p in [("natural", None), ("class", order)]:
    for rep in range(2):
        _, st = pt.render(ds, W, H, spp, 8, pixels=p, stats=True)
        res["%s_%d" % (name, rep)] = {"kernel_ms": round(st["kernel_ms"], 1),
                                      "Msamples_per_s": round(W * H * spp / st["kernel_ms"] / 1e3, 2),
                                      "waves_only": round(W * H * spp / st["wave_ms"] / 1e3, 2)}
print(json.dumps({"spp": spp, "class_counts": np.bincount(cls.reshape(-1).astype(np.int64)).tolist(), **res}))
