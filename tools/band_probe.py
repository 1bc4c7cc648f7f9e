"""Per-band kernel times of a benchmark config: the frame rendered as row
bands (one pixel-list launch each), one JSON line per band as it finishes, so
a slow region of the frame shows before any time limit.
usage: band_probe.py CONFIG SPP ROWS_PER_BAND [first_row last_row [first_col last_col]]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "path-trace_amd"))
import pathtrace as pt  # noqa: E402
from pathtrace import scenes  # noqa: E402

name, spp, rows = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
cfg = scenes.CONFIGS[name]
y0 = int(sys.argv[4]) if len(sys.argv) > 4 else 0
y1 = int(sys.argv[5]) if len(sys.argv) > 5 else cfg.height
ds = cfg.device_scene()
W = cfg.width
x0 = int(sys.argv[6]) if len(sys.argv) > 6 else 0
x1 = int(sys.argv[7]) if len(sys.argv) > 7 else W
for y in range(y0, y1, rows):
    pix = (np.arange(y, min(y + rows, y1))[:, None] * W + np.arange(x0, x1)[None, :]).astype(np.int32).ravel()
    t = time.time()
    img, st = pt.render(ds, W, cfg.height, spp, cfg.depth, screen=cfg.screen, pixels=pix, stats=True)
    print(json.dumps({"y": y, "rows": rows, "x": [x0, x1], "wall_s": round(time.time() - t, 3), "kernel_ms": round(st["kernel_ms"], 1),
                      "wave_ms": round(st["wave_ms"], 2), "q_per_sample": round(st["queries"] / st["samples"], 1),
                      "leaf_queries": st["leaf_queries"]}), flush=True)
