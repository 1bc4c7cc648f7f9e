"""Freezes the reference's texture lookups for the boundary's pt_tex_eval
(Texture::getColor / getFloat, include/texture.h:13-18, through the virtuals)
into tests/golden/tex_eval.npz: every texture of the zoo scenes (file order of
to_text) at zoo.texture_points().  Runs only where /root/reference and the
compiled reference driver (oracle/_ref/ptref, "tex" mode) exist."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "path-trace_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle_py as O  # noqa: E402
import zoo as T  # noqa: E402
from pathtrace.scene import to_text  # noqa: E402


def main():
    if not (os.path.isdir("/root/reference") and O.ref_available()):
        sys.exit("needs /root/reference and `make -C oracle ref`")
    pts = T.texture_points()
    out = {"points": pts}
    for name in T.TEX_EVAL_SCENES:
        txt = to_text(T.build(name), "/tmp/pt_golden_img")
        out[name] = O.ref_tex_eval(txt, pts)
    np.savez_compressed(os.path.join(HERE, "tex_eval.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
