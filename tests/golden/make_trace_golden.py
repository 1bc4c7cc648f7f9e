"""Freezes traceRay fixtures of the UNMODIFIED reference (oracle/_ref/ptref
"rays" mode: PathTrace::traceRay<PtSampleEngine>(ray, it, depth, engine,
strength), include/path-trace.h:58-165, once per (ray, sample) with the
per-(ray, sample) engine of include/pt/pt_engine.h, samples summed in order,
/ spp) for tests/test_trace_rays.py.  Runs only where /root/reference exists.

    python tests/golden/make_trace_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "path-trace_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import oracle_py as O  # noqa: E402
import zoo as T  # noqa: E402
from pathtrace.scene import to_text  # noqa: E402

SEED = 0x5EED
# (name, builder, depth, rays, spp)
CASES = [("p1", "scene_p1", 8, 384, 2), ("csg", "csg_zoo", 6, 384, 2)]


def main():
    if not O.ref_available():
        sys.exit("needs `make -C oracle ref` (/root/reference)")
    for name, builder, depth, n, spp in CASES:
        rays = T.trace_rays_input(n, seed=17)
        txt = to_text(T.build(builder), "/tmp/pt_trace_golden_img")
        ref = O.ref_trace_rays(txt, rays, spp, depth, seed=SEED)
        np.savez_compressed(os.path.join(HERE, "trace_%s.npz" % name), rays=rays, mean=ref,
                            meta=np.array([spp, depth, SEED], dtype=np.int64))
        print(name, rays.shape, "mean", ref.mean(axis=0))


if __name__ == "__main__":
    main()
