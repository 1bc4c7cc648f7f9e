"""Per-rank kernel time of a sharded config on ONE GPU: renders
each rank's hashed 16x16 tile set (pathtrace.dist.rank_pixels) at the config's
full spp, one after the other, and reports each shard's kernel time.  The
slowest shard bounds a real N-GPU run (every rank renders its shard, then one
reduce), so max/mean is the load-imbalance factor and N * mean / max the
scaling ceiling the partition leaves.  With split "samples" each rank renders
every pixel for its share of the samples (sample_begin, sum_only), as
bench.py's default N > 1 partition.
Tiles are dealt by pathtrace.dist.rank_pixels (deal "lattice" 4x4 by default,
"hashed" 16x16 the round-2..5 partition).
usage: shard_times.py [C4] [world] [spp] [tiles|samples] [tile] [lattice|hashed]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "path-trace_amd"))
import pathtrace as pt  # noqa: E402
from pathtrace import dist as ptdist  # noqa: E402
from pathtrace import scenes  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C4"
cfg = scenes.CONFIGS[name]
world = int(sys.argv[2]) if len(sys.argv) > 2 else cfg.gpus
spp = int(sys.argv[3]) if len(sys.argv) > 3 and int(sys.argv[3]) > 0 else cfg.spp
split = sys.argv[4] if len(sys.argv) > 4 else "tiles"
tile = int(sys.argv[5]) if len(sys.argv) > 5 else 0
deal = sys.argv[6] if len(sys.argv) > 6 else "lattice"
ds = cfg.device_scene()
rows = []
for r in range(world):
    t = time.time()
    if split == "samples":
        s0, s1 = r * spp // world, (r + 1) * spp // world
        pix = np.arange(cfg.width * cfg.height)
        _, st = pt.render(ds, cfg.width, cfg.height, s1 - s0, cfg.depth, screen=cfg.screen, stats=True,
                          max_buffer_bytes=40 << 30, sample_begin=s0, sum_only=True)
    else:
        pix = ptdist.rank_pixels(cfg.width, cfg.height, r, world, tile=tile, deal=deal)
        _, st = pt.render(ds, cfg.width, cfg.height, spp, cfg.depth, screen=cfg.screen, pixels=pix, stats=True,
                          max_buffer_bytes=40 << 30)  # one pass per shard, as bench.py
    rows.append({"rank": r, "split": split, "tile": tile, "deal": deal, "pixels": int(len(pix)), "samples": int(st["samples"]), "kernel_ms": st["kernel_ms"], "reduce_ms": st["reduce_ms"],
                 "launches": st["launches"], "queries_per_sample": st["queries"] / st["samples"],
                 "wall_s": time.time() - t})
    print(json.dumps(rows[-1]), flush=True)
k = np.array([x["kernel_ms"] for x in rows])
samples = cfg.width * cfg.height * spp
print(json.dumps({"config": name, "split": split, "tile": tile, "deal": deal, "world": world, "spp": spp, "max_ms": float(k.max()), "mean_ms": float(k.mean()),
                  "imbalance_max_over_mean": float(k.max() / k.mean()),
                  "scaling_ceiling": float(world * k.mean() / k.max()),
                  "Msamples_per_s_if_parallel": samples / k.max() / 1e3}), flush=True)
