"""Same bits under a PT_DEVICE_DEFINES variant?  Renders a hashed pixel subset
of a config with the built-in library and with the variant (one process, the
define toggled between renders) and counts differing values.
usage: bits_ab.py CONFIG NPIX SPP "DEFINES" [order]   ("hdr:PATH" = a PT_DEVICE_HEADER variant)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "path-trace_amd"))
import pathtrace as pt  # noqa: E402
from pathtrace import scenes  # noqa: E402

name, npix, spp, defs = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
order = sys.argv[5] if len(sys.argv) > 5 else "fast"
cfg = scenes.CONFIGS[name]
rng = np.random.default_rng(7)
pix = np.sort(rng.choice(cfg.width * cfg.height, npix, replace=False)).astype(np.int32)
out = []
var = "PT_DEVICE_HEADER" if defs.startswith("hdr:") else "PT_DEVICE_DEFINES"
for d in ("", defs[4:] if defs.startswith("hdr:") else defs):
    if d:
        os.environ[var] = d
    else:
        os.environ.pop(var, None)
    ds = cfg.device_scene()
    img = pt.render(ds, cfg.width, cfg.height, spp, cfg.depth, screen=cfg.screen, pixels=pix, order=order)
    out.append(np.asarray(img).reshape(-1))
bad = int(np.sum(out[0].view(np.uint32) != out[1].view(np.uint32)))
print("%s %d px x %d spp, %s order, %r: %d of %d values differ" % (name, npix, spp, order, defs, bad, out[0].size))
sys.exit(1 if bad else 0)
