"""Freezes outputs of the UNMODIFIED reference (oracle/_ref/ptref, built from
/root/reference/src by oracle/Makefile) into small fixtures in tests/golden/.
Runs only in the survey/build container (needs /root/reference); the GPU box
and the CPU test suite read the committed fixtures.

    python tests/golden/make_golden.py
"""
import os
import shutil
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "path-trace_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import oracle_py as O  # noqa: E402
import zoo as T  # noqa: E402
from pathtrace.scene import to_text  # noqa: E402

REF = "/root/reference"
SEED = 0x5EED


def spans_to_arrays(spans):
    counts = np.array([len(s) for s in spans], dtype=np.int32)
    rows = []
    for s in spans:
        for (a, m0, b, m1) in s:
            rows.append(np.concatenate([a.view(np.uint32), [np.uint32(m0 & 0xFFFFFFFF)], b.view(np.uint32),
                                        [np.uint32(m1 & 0xFFFFFFFF)]]))
    data = np.array(rows, dtype=np.uint32).reshape(-1, 10)
    return counts, data


def main():
    if not (os.path.isdir(REF) and O.ref_available()):
        sys.exit("needs /root/reference and `make -C oracle ref`")
    img_dir = "/tmp/pt_golden_img"
    # 1. engine / vector-math known answers
    np.save(os.path.join(HERE, "kat.npy"), O.ref_kat())
    # 2. full span lists of random rays through CSG scenes (quirks included)
    for name, builder in [("csg", T.csg_zoo), ("p1", None)]:
        root = builder() if builder else T.build("scene_p1")
        txt = to_text(root, img_dir)
        rays = T.random_rays(3000, seed=11)
        counts, data = spans_to_arrays(O.ref_spans(txt, rays))
        np.savez_compressed(os.path.join(HERE, "spans_%s.npz" % name), rays=rays, counts=counts, data=data)
    # 3. per-sample radiance of small frames (tracePixel<E> with the per-sample engine)
    for (name, builder, W, H, spp, depth) in T.RENDER_CASES:
        txt = to_text(T.build(builder), img_dir)
        res, info = O.ref_render(txt, W, H, spp, depth, seed=SEED, per_sample=True, info=True)
        np.savez_compressed(os.path.join(HERE, "render_%s.npz" % name), per_sample=res,
                            meta=np.array([W, H, spp, depth, SEED, info["queries"]], dtype=np.int64))
    # 4. test images hash (fixtures assume numpy's PCG64 stream is unchanged)
    imgs = T.zoo_images()
    np.save(os.path.join(HERE, "test_images_sum.npy"), np.array([float(np.sum(i.data, dtype=np.float64))
                                                                  for i in imgs]))
    # 5. Radiance HDR: the reference's matched 192x108 pair; its decode; writeHDR of synthetic data
    shutil.copy(os.path.join(REF, "image53424F01.hdr"), os.path.join(HERE, "image53424F01.hdr"))
    shutil.copy(os.path.join(REF, "image53424F01.bmp"), os.path.join(HERE, "image53424F01.bmp"))
    px, rewritten = O.ref_hdr(os.path.join(REF, "image53424F01.hdr"))
    with open(os.path.join(REF, "image53424F01.hdr"), "rb") as f:
        assert f.read() == rewritten, "reference writeHDR does not round-trip its own file"
    np.savez_compressed(os.path.join(HERE, "hdr_decode.npz"), rgba=px)
    rng = np.random.default_rng(21)
    cases = []
    for (w, h) in [(40, 3), (130, 2), (8, 5)]:
        rgb = (rng.lognormal(mean=-0.5, sigma=2.0, size=(h, w, 3)) * (rng.uniform(size=(h, w, 1)) > 0.1))
        rgb = rgb.astype(np.float32)
        rgb[0, :w // 2] = rgb[0, 0]  # long runs for the RLE encoder
        cases.append((rgb, O.ref_write_hdr(rgb)))
    np.savez_compressed(os.path.join(HERE, "hdr_write.npz"),
                        **{"rgb%d" % k: c[0] for k, c in enumerate(cases)},
                        **{"bytes%d" % k: np.frombuffer(c[1], dtype=np.uint8) for k, c in enumerate(cases)})
    # 6. Matrix::rotate / invert / concat
    rng = np.random.default_rng(5)
    recs, inputs = [], []
    for k in range(64):
        axis = rng.normal(size=3).astype(np.float32)
        angle = float(rng.uniform(-7, 7))
        m = rng.normal(size=12).astype(np.float32)
        m2 = rng.normal(size=12).astype(np.float32)
        if k == 0:
            m[:] = 0  # singular
        recs.append(axis.tobytes() + b"\0" * 4 + struct.pack("<d", angle) + m.tobytes() + m2.tobytes())
        inputs.append((axis, angle, m, m2))
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        a, b = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        with open(a, "wb") as f:
            f.write(b"".join(recs))
        subprocess.check_call([O.REF_PATH, "matrix", a, b])
        out = np.fromfile(b, dtype=np.float32).reshape(64, 3, 12)
    np.savez_compressed(os.path.join(HERE, "matrix.npz"), axis=np.array([i[0] for i in inputs]),
                        angle=np.array([i[1] for i in inputs]), m=np.array([i[2] for i in inputs]),
                        m2=np.array([i[3] for i in inputs]), out=out)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
