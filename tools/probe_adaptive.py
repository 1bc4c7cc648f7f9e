"""Adaptive caller (pt_render_adaptive) on a full benchmark frame vs the plain
full-frame render at the same spp.  usage: probe_adaptive.py CONFIG SPP"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "path-trace_amd"))
import numpy as np  # noqa: E402
import pathtrace as pt  # noqa: E402
from pathtrace import scenes  # noqa: E402

name, spp = sys.argv[1], int(sys.argv[2])
cfg = scenes.CONFIGS[name]
ds = cfg.device_scene()
t = time.time()
img_x, info_x = pt.render_adaptive(ds, cfg.width, cfg.height, spp, cfg.depth, screen=cfg.screen, exact_batches=True)
tx = time.time() - t
t = time.time()
img, info = pt.render_adaptive(ds, cfg.width, cfg.height, spp, cfg.depth, screen=cfg.screen)
ta = time.time() - t
assert (img.view(np.uint32) == img_x.view(np.uint32)).all()
t = time.time()
full, st = pt.render(ds, cfg.width, cfg.height, spp, cfg.depth, screen=cfg.screen, stats=True)
tf = time.time() - t
rmse = np.sqrt(np.mean((img.astype(np.float64) - full) ** 2, axis=(0, 1))).tolist()
print(json.dumps({"config": name, "spp": spp, "adaptive_wall_s": ta, "adaptive_kernel_ms": info["kernel_ms"],
                  "traced_pixels": info["traced_pixels"], "traced_frac": info["traced_pixels"] / (cfg.width * cfg.height),
                  "levels": info["levels"], "lookahead_pixels": info["lookahead_pixels"],
                  "exact_batches": {"wall_s": tx, "kernel_ms": info_x["kernel_ms"], "levels": info_x["levels"]},
                  "full_wall_s": tf, "full_kernel_ms": st["kernel_ms"],
                  # the work the adaptive batches did (traced + lookahead points) against the frame's:
                  # time at the frame's rate for that work = full_kernel_ms * query_frac
                  "adaptive_samples": info["samples"], "adaptive_queries": info["queries"],
                  "full_samples": st["samples"], "full_queries": st["queries"],
                  "sample_frac": info["samples"] / st["samples"], "query_frac": info["queries"] / st["queries"],
                  "ms_at_frame_rate": st["kernel_ms"] * info["queries"] / st["queries"],
                  "rmse_adaptive_vs_full": rmse}), flush=True)
