"""Per-config GPU probe: render a hashed pixel subset of a benchmark config at
a given spp and print throughput with the kernel's counters.
usage: cfg_probe.py CONFIG NPIX SPP [procedural | disk:CX:CY:R]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "path-trace_amd"))
import pathtrace as pt  # noqa: E402
from pathtrace import scenes  # noqa: E402

name, npix, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
proc = len(sys.argv) > 4 and sys.argv[4] == "procedural"
disk = [float(v) for v in sys.argv[4].split(":")[1:]] if len(sys.argv) > 4 and sys.argv[4].startswith("disk") else None
cfg = scenes.CONFIGS[name]
import dataclasses  # noqa: E402
if os.environ.get("PROBE_LANE_WALK"):  # A/B of pt_scene_set_lane_walk
    cfg = dataclasses.replace(cfg, lane_walk=int(os.environ["PROBE_LANE_WALK"]))
if os.environ.get("PROBE_WG"):  # A/B of pt_scene_set_occupancy
    cfg = dataclasses.replace(cfg, wg_per_cu=int(os.environ["PROBE_WG"]))
if os.environ.get("PROBE_C2_PLAIN"):  # C2 without matBrightDiffuseWhite (round 2's C2)
    from pathtrace.scenes import scene_c2
    cfg = dataclasses.replace(cfg, scene=lambda procedural=False: scene_c2(procedural, full_mix=False))
if os.environ.get("PROBE_FAST_SPINE"):
    cfg = dataclasses.replace(cfg, fast_spine=bool(int(os.environ["PROBE_FAST_SPINE"])))
ds = cfg.device_scene(procedural=proc)
W, H = cfg.width, cfg.height
rng = np.random.default_rng(1)
pix = None if npix <= 0 else np.sort(rng.choice(W * H, npix, replace=False)).astype(np.int32)
if disk:  # disk:cx:cy:r -- npix pixels inside that disk of the frame
    cx, cy, r = disk
    a = rng.uniform(0, 2 * np.pi, npix)
    rr = r * np.sqrt(rng.uniform(0, 1, npix))
    pix = np.unique((cy + rr * np.sin(a)).astype(np.int32) * W + (cx + rr * np.cos(a)).astype(np.int32))
t = time.time()
depth = int(os.environ.get("PROBE_DEPTH", cfg.depth))
order = os.environ.get("PROBE_ORDER", "fast")
img, st = pt.render(ds, W, H, spp, depth, screen=cfg.screen, pixels=pix, stats=True, order=order)
n = (W * H if pix is None else len(pix)) * spp
print(json.dumps({"config": name, "procedural": proc, "depth": depth, "order": order, "pixels": W * H if pix is None else len(pix), "spp": spp,
                  "wall_s": time.time() - t, "Msamples_per_s": n / st["kernel_ms"] / 1e3,
                  "queries_per_sample": st["queries"] / st["samples"], **st}))
