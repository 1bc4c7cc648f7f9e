"""Calibrate the algorithmic work model of SURVEY.md s8(d) for a config:
FP32 op weights per event (sphere miss 23, sphere hit 68, plane 18, CSG merge
step 4, hit shading 60, refraction child 45, scatter child incl. rejection 155)
times the event counts the CPU oracle measures on a hashed pixel sample.
Prints ops per root query; bench.py multiplies it by the GPU's exact query
count.  usage: calibrate_ops.py [C3] [npix] [spp]"""
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


def model_ops(st):
    return (W["sphere_miss"] * (st["sphere_tests"] - st["sphere_hits"]) + W["sphere_hit"] * st["sphere_hits"] +
            W["plane"] * st["plane_tests"] + W["merge"] * st["merge_steps"] + W["shaded"] * st["shaded"] +
            W["refract"] * st["refract_children"] + W["scatter"] * st["scatter_children"])


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
                      "ops_per_query": ops / st["queries"], "ops_per_sample": ops / (npix * spp), **st}))
