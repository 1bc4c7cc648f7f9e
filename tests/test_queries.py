"""The boundary's query virtuals on the device:

  pt_query_spans  Object::makeSpanIterator() + SpanIterator::init / next
                  (include/object.h:14, include/span.h:129-171): full span lists
                  of random rays through the CSG zoo (every operator, nested
                  transforms, the Difference quirk) and the north-star scene,
                  bit for bit against the UNMODIFIED reference's lists
                  (tests/golden/spans_*.npz, frozen from oracle/_ref/ptref);
  pt_tex_eval     Texture::getColor / getFloat (include/texture.h:13-18) of
                  every texture of the texture zoos at 2048 points, against the
                  reference's lookups (tests/golden/tex_eval.npz): bit for bit
                  for every texture, the transcendental zoo included (atan2f/asinf/
                  logf restated from glibc on the device)."""
import os

import numpy as np
import pytest

import oracle_py as O
import zoo as T
from pathtrace import DeviceScene
from pathtrace.scene import to_text

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_oracle_textures_match_reference(built, tmp_path):
    """CPU: the oracle's texture classes against the reference's own lookups."""
    z = np.load(os.path.join(GOLD, "tex_eval.npz"))
    for name in T.TEX_EVAL_SCENES:
        got = O.tex_eval(to_text(T.build(name), str(tmp_path)), z["points"])
        np.testing.assert_array_equal(got.view(np.uint32), z[name].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["csg", "p1"])
def test_query_spans_match_reference(built, tmp_path, name):
    z = np.load(os.path.join(GOLD, "spans_%s.npz" % name))
    root = T.csg_zoo() if name == "csg" else T.build("scene_p1")
    ds = DeviceScene.from_text(to_text(root, str(tmp_path)))  # material ids = the text's
    ms = int(z["counts"].max())
    counts, spans = ds.query_spans(z["rays"], max_spans=ms)
    np.testing.assert_array_equal(counts, z["counts"])
    rows = np.concatenate([spans[i, :c] for i, c in enumerate(counts)]).view(np.uint32)
    np.testing.assert_array_equal(rows, z["data"])


@pytest.mark.gpu
def test_query_spans_truncates_to_max_spans(built, tmp_path):
    z = np.load(os.path.join(GOLD, "spans_csg.npz"))
    ds = DeviceScene.from_text(to_text(T.csg_zoo(), str(tmp_path)))
    counts, spans = ds.query_spans(z["rays"], max_spans=1)
    np.testing.assert_array_equal(counts, z["counts"])  # counts are the full list lengths
    first = np.cumsum(np.concatenate([[0], z["counts"][:-1]]))
    has = z["counts"] > 0
    np.testing.assert_array_equal(spans[has, 0].view(np.uint32), z["data"][first[has]])


@pytest.mark.gpu
@pytest.mark.parametrize("name", T.TEX_EVAL_SCENES)
def test_tex_eval_matches_reference(built, tmp_path, name):
    z = np.load(os.path.join(GOLD, "tex_eval.npz"))
    want = z[name]
    ds = DeviceScene.from_text(to_text(T.build(name), str(tmp_path)))  # texture ids = file order
    got = np.zeros_like(want)
    for k in range(len(want)):
        rgb, val = ds.tex_eval(k, z["points"])
        got[k, :, :3], got[k, :, 3] = rgb, val
    same = got.view(np.uint32) == want.view(np.uint32)
    # bit for bit, the transcendental zoo too: the spherical maps' atan2f / asinf
    # and the log filter's logf are glibc's algorithms restated (tests/test_libm.py)
    assert same.all(), "%d of %d lookups differ" % ((~same).sum(), same.size)
