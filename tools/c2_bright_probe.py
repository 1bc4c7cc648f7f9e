"""Queries per sample of C2 with and without the demo's matBrightDiffuseWhite
(reference src/test.cpp:115, reflectance 8), measured with the CPU oracle on a
small hashed pixel set: the reason C2 leaves that material out."""
import math
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "path-trace_amd"), os.path.join(ROOT, "oracle")]
import oracle_py as O  # noqa: E402
from pathtrace import scenes  # noqa: E402
from pathtrace.scene import Sphere, union_array, to_text  # noqa: E402


def c2(bright: bool):
    base = scenes.scene_c2(procedural=True)
    if not bright:
        return base
    m = scenes.materials()
    objs = []

    def walk(o):
        if hasattr(o, "a"):
            walk(o.a)
            walk(o.b)
        else:
            objs.append(o)
    walk(base)
    # the demo's mix puts matBrightDiffuseWhite on one sphere: swap it onto the 4th
    k = [i for i, o in enumerate(objs) if isinstance(o, Sphere)][3]
    o = objs[k]
    objs[k] = Sphere(o.center, o.r, m["brightDiffuse"])
    return union_array(objs)


W, H, spp, depth = 1280, 720, 2, 16
rng = np.random.default_rng(5)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
if len(sys.argv) > 2 and sys.argv[2] == "disk":
    # pixels inside the 4th sphere's image (centre ~(430, 397), radius ~80 px)
    ang = rng.uniform(0, 2 * math.pi, n)
    rad = 70 * np.sqrt(rng.uniform(0, 1, n))
    pix = np.unique((397 + rad * np.sin(ang)).astype(np.int32) * W + (430 + rad * np.cos(ang)).astype(np.int32))
else:
    pix = np.sort(rng.choice(W * H, n, replace=False)).astype(np.int32)
cfg = scenes.CONFIGS["C2"]
for bright in (False, True):
    txt = to_text(c2(bright), tempfile.mkdtemp())
    t = time.time()
    img, st = O.render(txt, W, H, spp, depth, screen=cfg.screen, pixels=pix, threads=8, stats=True)
    q = st["queries"] / (len(pix) * spp)
    print("mean radiance", float(img.mean()))
    print({"bright": bright, "pixels": len(pix), "spp": spp, "queries_per_sample": round(q, 1),
           "max_queries_in_a_pixel": None, "seconds": round(time.time() - t, 1)}, flush=True)
