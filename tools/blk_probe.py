"""Probe of block-staged launches (one partial per 32-sample block) against
passes of 64 per-sample values, then the config-scale C3 fixture's renders
one at a time, printing before and after each launch."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "path-trace_amd"))
import pathtrace as pt  # noqa: E402
from pathtrace import scenes  # noqa: E402

ds = pt.DeviceScene(scenes.scene_p1())
for (W, H, spp, mb) in [(256, 160, 128, 256 * 160 * 12 * 64), (256, 160, 128, 0)]:
    print("start", W, H, spp, mb, flush=True)
    t = time.time()
    img, st = pt.render(ds, W, H, spp, 8, stats=True, max_buffer_bytes=mb)
    print(json.dumps({"W": W, "spp": spp, "mb": mb, "s": time.time() - t, "launches": st["launches"],
                      "kernel_ms": st["kernel_ms"], "mean": float(img.mean())}), flush=True)
z = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                         "config_C3.npz"))
W, H, spp, depth, seed = [int(v) for v in z["meta"][:5]]
cfg = scenes.CONFIGS["C3"]
ds = cfg.device_scene()
for order in ["reference", "fast"]:
    print("start C3", order, flush=True)
    t = time.time()
    g, st = pt.render(ds, W, H, spp, depth, screen=cfg.screen, seed=seed, pixels=z["pixels"], order=order,
                      stats=True)
    print(json.dumps({"order": order, "s": time.time() - t, "launches": st["launches"], "kernel_ms": st["kernel_ms"],
                      "max_err": float(np.abs(g - z["means"]).max())}), flush=True)
