"""Quick single-GPU probe: render the C3 scene at 1080p with a few spp and
print Msamples/s and the kernel's counters.  usage: perf_probe.py [spp] [order]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "path-trace_amd"))
import pathtrace as pt  # noqa: E402
from pathtrace import scenes  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 4
order = sys.argv[2] if len(sys.argv) > 2 else "fast"
ds = scenes.CONFIGS["C3"].device_scene()  # the bench config's scene and settings
t = time.time()
img, st = pt.render(ds, 1920, 1080, spp, 8, stats=True, order=order)
dt = time.time() - t
ms = st["kernel_ms"]
print(json.dumps({"spp": spp, "order": order, "wall_s": dt, "kernel_ms": ms,
                  "Msamples_per_s": 1920 * 1080 * spp / ms / 1e3,
                  "queries_per_sample": st["queries"] / st["samples"],
                  "Msamples_per_s_waves": 1920 * 1080 * spp / st["wave_ms"] / 1e3 if st.get("wave_ms") else None,
                  **st}))
