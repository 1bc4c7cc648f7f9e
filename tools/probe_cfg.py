"""Render one benchmark config at a given size on the GPU and print timing and
counters.  usage: probe_cfg.py CONFIG W H SPP [order]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "path-trace_amd"))
import pathtrace as pt  # noqa: E402
from pathtrace import scenes  # noqa: E402

name, W, H, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
order = sys.argv[5] if len(sys.argv) > 5 else "fast"
cfg = scenes.CONFIGS[name]
ds = cfg.device_scene()
screen = (float(W), float(H), float(2 * min(W, H)))
t = time.time()
img, st = pt.render(ds, W, H, spp, cfg.depth, screen=screen, stats=True, order=order)
dt = time.time() - t
print(json.dumps({"config": name, "W": W, "H": H, "spp": spp, "wall_s": dt, "kernel_ms": st["kernel_ms"],
                  "Msamples_per_s": W * H * spp / st["kernel_ms"] / 1e3,
                  "queries_per_sample": st["queries"] / st["samples"],
                  "slow_frac": st["slow_queries"] / max(1, st["leaf_queries"]), **st}), flush=True)
