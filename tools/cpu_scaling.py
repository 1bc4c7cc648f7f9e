"""The reference's CPU path (oracle/_ref/ptref: the unmodified reference
sources, RenderBlock-style pool of std::threads) timed on this host:

  1. C1 in full (256x256, 16 spp, depth 4, scene P0) -- BASELINE.md's plan;
  2. the C3 bench sample (hashed pixels of the 1920x1080 frame at 1024 spp) at
     4, 8 and 16 threads -- the linearity that bench.py's
     cpu_baseline.all_host_cpus_projected assumes, measured inside the GPU
     box's per-GPU CPU share (16 threads; more would take other GPUs' shares).

usage: python tools/cpu_scaling.py OUT.json [c3_pixels]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "path-trace_amd"), os.path.join(ROOT, "oracle")]
import oracle_py as O  # noqa: E402
from pathtrace import scenes  # noqa: E402
from pathtrace.scene import to_text  # noqa: E402

out_path = sys.argv[1]
npx = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
share = len(os.sched_getaffinity(0))
omp = os.environ.get("OMP_NUM_THREADS", "")
if omp.isdigit():
    share = min(share, int(omp))
res = {"host_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)), "cpu_share": share,
       "kind": "reference" if O.ref_available() else "port"}
render = O.ref_render if O.ref_available() else None
if render is None:
    sys.exit("needs oracle/_ref/ptref (built by build() in the build container)")

c1 = scenes.CONFIGS["C1"]
txt = to_text(c1.scene(), "/tmp/pt_cpu_scaling_img")
t0 = time.time()
img, info = render(txt, c1.width, c1.height, c1.spp, c1.depth, screen=c1.screen, threads=share, info=True)
res["C1_full_frame"] = {"threads": share, "seconds": info["seconds"], "samples": info["samples"],
                        "Msamples_per_s": info["samples"] / info["seconds"] / 1e6,
                        "queries_per_sample": info["queries"] / info["samples"], "wall_s": time.time() - t0,
                        "image_mean": [float(v) for v in img.mean(axis=0)]}
print(json.dumps(res["C1_full_frame"]), flush=True)

c3 = scenes.CONFIGS["C3"]
txt = to_text(c3.scene(), "/tmp/pt_cpu_scaling_img")
pix = np.sort(np.random.default_rng(0x5EED).choice(c3.width * c3.height, npx, replace=False)).astype(np.int32)
rows = []
for th in (4, 8, 16):
    if th > share:
        continue
    _, info = render(txt, c3.width, c3.height, c3.spp, c3.depth, screen=c3.screen, pixels=pix, threads=th, info=True)
    rows.append({"threads": th, "seconds": info["seconds"], "Msamples_per_s": info["samples"] / info["seconds"] / 1e6,
                 "queries_per_sample": info["queries"] / info["samples"]})
    print(json.dumps(rows[-1]), flush=True)
base = rows[0]
for r in rows:
    r["speedup_vs_%d" % base["threads"]] = r["Msamples_per_s"] / base["Msamples_per_s"]
    r["parallel_efficiency"] = r["speedup_vs_%d" % base["threads"]] * base["threads"] / r["threads"]
res["C3_sample_scaling"] = {"pixels": npx, "spp": c3.spp, "rows": rows,
                            "why_not_beyond_share": "the box gives each GPU job a %d-thread CPU share "
                                                    "(OMP_NUM_THREADS); threads past it would run on the other "
                                                    "GPUs' shares of the %d-CPU host" % (share, os.cpu_count())}
with open(out_path, "w") as f:
    json.dump(res, f, indent=1)
