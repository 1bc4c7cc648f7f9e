"""C5 reference-order pixels against the unmodified reference's config fixture
(tests/golden/config_C5.npz) and the fast order against the oracle: count of
values that differ in any bit (the spherical sky map's glibc atan2f/asinf)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "path-trace_amd"), os.path.join(ROOT, "oracle")]
import oracle_py as O  # noqa: E402
import pathtrace as pt  # noqa: E402
from pathtrace import scenes  # noqa: E402
from pathtrace.scene import to_text  # noqa: E402

z = np.load(os.path.join(ROOT, "tests", "golden", "config_C5.npz"))
pix, ref = z["pixels"], z["means"]
W, H, spp, depth, seed = [int(v) for v in z["meta"][:5]]
cfg = scenes.CONFIGS["C5"]
ds = cfg.device_scene()
g = pt.render(ds, W, H, spp, depth, screen=cfg.screen, seed=seed, pixels=pix, order="reference")
f = pt.render(ds, W, H, spp, depth, screen=cfg.screen, seed=seed, pixels=pix, order="fast")
o = O.render(to_text(cfg.scene(), "/tmp/pt_c5bits"), W, H, spp, depth, screen=cfg.screen, seed=seed, pixels=pix,
             order=O.ORDER_FAST)
print(json.dumps({"pixels": len(pix), "reference_order_vs_ptref_bad": int(np.sum(g.view(np.uint32) != ref.view(np.uint32))),
                  "fast_vs_oracle_bad": int(np.sum(f.view(np.uint32) != o.view(np.uint32)))}))
