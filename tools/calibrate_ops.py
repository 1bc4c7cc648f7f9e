"""Calibrate the algorithmic work model of SURVEY.md s8(d) for a config:
FP32 op weights per event (sphere miss 23, sphere hit 68, plane 18, CSG merge
step 4, hit shading 60, refraction child 45, scatter child incl. rejection 155)
times the event counts the CPU oracle measures on a hashed pixel sample.
Since round 6 the texture maps' work is in the model too:
one weight per texture evaluation by class, counted from the restated code the
kernel runs (compares and arithmetic, integer or float; selects and bit casts
not counted) -- TransformedTexture 18 (m_apply: 9 mul + 9 add), Multiply 3,
Image 15 (planar texel: two double floor/sub pairs, 1 - y, two scales, two
floors, two conversions, four bounds compares), SphericalCoordinates 93 (zero
test 3, normalize 10, atan2f 50, the theta range 2, asinf 22, the double
scaling 6), MirrorBall 26, Skybox 28 (face selection 12, texel 16), Log 60
(three channels of logf and its scaling).  Prints ops per root query;
bench.py multiplies it by the GPU's exact query count.
usage: calibrate_ops.py [C3] [npix] [spp]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "path-trace_amd"), os.path.join(ROOT, "oracle")]
import oracle_py as O  # noqa: E402
from pathtrace import scenes  # noqa: E402
from pathtrace.scene import to_text  # noqa: E402

W = {"sphere_miss": 23, "sphere_hit": 68, "plane": 18, "merge": 4, "shaded": 60, "refract": 45, "scatter": 155}
TEX_W = {"tex_xform": 18, "tex_multiply": 3, "tex_image": 15, "tex_spherical": 93, "tex_mirrorball": 26,
         "tex_skybox": 28, "tex_log": 60}


def texture_ops(st):
    return sum(w * st.get(k, 0) for k, w in TEX_W.items())


def model_ops(st):
    return (W["sphere_miss"] * (st["sphere_tests"] - st["sphere_hits"]) + W["sphere_hit"] * st["sphere_hits"] +
            W["plane"] * st["plane_tests"] + W["merge"] * st["merge_steps"] + W["shaded"] * st["shaded"] +
            W["refract"] * st["refract_children"] + W["scatter"] * st["scatter_children"] + texture_ops(st))


if __name__ == "__main__":
    name = sys.argv[1] if len(sys.argv) > 1 else "C3"
    npix = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    spp = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    cfg = scenes.CONFIGS[name]
    rng = np.random.default_rng(1)
    pix = np.sort(rng.choice(cfg.width * cfg.height, npix, replace=False)).astype(np.int32)
    txt = to_text(cfg.scene(), "/tmp/pt_calib_img")
    _, st = O.render(txt, cfg.width, cfg.height, spp, cfg.depth, screen=cfg.screen, pixels=pix, stats=True,
                     order=O.ORDER_FAST)
    ops = model_ops(st)
    print(json.dumps({"config": name, "pixels": npix, "spp": spp, "queries_per_sample": st["queries"] / (npix * spp),
                      "ops_per_query": ops / st["queries"], "ops_per_sample": ops / (npix * spp),
                      "texture_ops_per_query": texture_ops(st) / st["queries"], **st}))
