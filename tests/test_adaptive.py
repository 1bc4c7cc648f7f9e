"""The reference demo's adaptive image formation (RenderBlock::renderSquare,
reference src/test.cpp:423-507).

CPU: the oracle's depth-first restatement (oracle.cpp AdaptiveBlock) against
an independent pure-Python restatement of the same recursion on small frames,
and against plain per-pixel renders when interpolation is disabled.
GPU: libpt's level-synchronous evaluation (pt_render_adaptive) bit for bit
against the oracle.  The reference's renderSquare lives in src/test.cpp, which
needs SDL and is not compiled here: the policy layer's parity rests on these
restatements (per-pixel values are pinned by the reference goldens)."""
import numpy as np
import pytest

import oracle_py as O
import zoo as T
from pathtrace import scenes
from pathtrace.scene import to_text


def py_adaptive(trace, W, H, block, max_interp, min_delta):
    """Straight Python restatement of RenderBlock for one frame."""
    f32 = np.float32
    img = np.zeros((H, W, 3), dtype=f32)
    mcd2 = f32(min_delta) * f32(min_delta)

    def abs2(a):
        return f32(f32(a[0] * a[0] + a[1] * a[1]) + a[2] * a[2])

    def close(a, b):
        d = (a - b).astype(f32)
        return abs2(d) <= f32(mcd2 * abs2(a))

    for y0 in range(0, H, block):
        for x0 in range(0, W, block):
            buf = {}

            def inb(x, y):
                return not (x < x0 or x - x0 > block) and not (y < y0 or y - y0 > block)

            def setp(x, y, c):
                if inb(x, y):
                    buf[(x, y)] = c

            def calc(x, y):
                if inb(x, y) and (x, y) in buf:
                    return buf[(x, y)]
                c = trace(x, y)
                setp(x, y, c)
                return c

            def square(x, y, size, tl, tr, bl, br):
                if x > W or y > H:
                    return
                if size <= 1:
                    setp(x, y, tl)
                    return
                if (close(tl, tr) and close(tl, bl) and close(tl, br) and close(tr, bl) and close(tr, br)
                        and close(bl, br) and size <= max_interp):
                    for yy in range(size):
                        fy = f32(f32(yy) / f32(size))
                        lc = (tl + (fy * (bl - tl).astype(f32)).astype(f32)).astype(f32)
                        rc = (tr + (fy * (br - tr).astype(f32)).astype(f32)).astype(f32)
                        for xx in range(size):
                            fx = f32(f32(xx) / f32(size))
                            setp(xx + x, yy + y, (lc + (fx * (rc - lc).astype(f32)).astype(f32)).astype(f32))
                    return
                h = size // 2
                cx, cy = x + h, y + h
                tc, cl, cc = calc(cx, y), calc(x, cy), calc(cx, cy)
                cr, bc = calc(x + size, cy), calc(cx, y + size)
                square(x, y, h, tl, tc, cl, cc)
                square(cx, y, h, tc, tr, cc, cr)
                square(x, cy, h, cl, cc, bl, bc)
                square(cx, cy, h, cc, cr, bc, br)

            square(x0, y0, block, calc(x0, y0), calc(x0 + block, y0), calc(x0, y0 + block),
                   calc(x0 + block, y0 + block))
            for (x, y), c in buf.items():
                if x0 <= x < min(x0 + block, W) and y0 <= y < min(y0 + block, H):
                    img[y, x] = c
    return img


def _tracer(txt, W, H, spp, depth, block):
    """tracePixel on the engine grid (gw = ceil(W / block) * block + 1), for every
    grid pixel the frame's blocks can touch."""
    gw = (W + block - 1) // block * block + 1
    rows = (H + block - 1) // block * block + 1
    grid = O.render_gw(txt, W, H, gw, np.arange(gw * rows), spp, depth,
                       order=O.ORDER_FAST).reshape(rows, gw, 3)
    return lambda x, y: grid[y, x].copy()


@pytest.mark.parametrize("W,H,block,max_interp,delta", [(40, 24, 8, 9, 0.003), (33, 19, 16, 9, 0.05),
                                                         (24, 16, 8, 4, 0.3)])
def test_oracle_adaptive_matches_python_restatement(built, tmp_path, W, H, block, max_interp, delta):
    txt = to_text(scenes.scene_p1(), str(tmp_path))
    spp, depth = 2, 4
    got, traced = O.render_adaptive(txt, W, H, spp, depth, block, max_interp, delta, order=O.ORDER_FAST)
    want = py_adaptive(_tracer(txt, W, H, spp, depth, block), W, H, block, max_interp, delta)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    assert 0 < traced


def test_oracle_adaptive_without_interpolation_is_per_pixel(built, tmp_path):
    """max_interp = 1: every square subdivides to single pixels, so the image is
    tracePixel of every pixel on the engine grid."""
    W, H = 37, 21
    gw = 41  # ceil(37 / 8) * 8 + 1
    txt = to_text(T.csg_zoo(), str(tmp_path))
    got, _ = O.render_adaptive(txt, W, H, 2, 4, 8, 1, 0.003, order=O.ORDER_FAST)
    ys, xs = np.mgrid[0:H, 0:W]
    want = O.render_gw(txt, W, H, gw, (ys * gw + xs).ravel(), 2, 4, order=O.ORDER_FAST)
    np.testing.assert_array_equal(got.reshape(-1, 3).view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("builder,W,H,spp,depth,block,max_interp,delta", [
    ("p1", 96, 64, 4, 8, 16, 9, 0.003), ("csg_zoo", 80, 48, 2, 6, 32, 9, 0.01), ("p0", 64, 40, 3, 4, 8, 9, 0.003)])
def test_gpu_adaptive_matches_oracle(built, tmp_path, builder, W, H, spp, depth, block, max_interp, delta):
    import pathtrace as pt
    root = {"p1": scenes.scene_p1, "p0": scenes.scene_p0, "csg_zoo": T.csg_zoo}[builder]()
    img, info = pt.render_adaptive(root, W, H, spp, depth, block_size=block, max_interp=max_interp,
                                   min_delta=delta)
    want, traced = O.render_adaptive(to_text(root, str(tmp_path)), W, H, spp, depth, block, max_interp, delta,
                                     order=O.ORDER_FAST)
    diff = np.nonzero(img.reshape(-1, 3).view(np.uint32) != want.reshape(-1, 3).view(np.uint32))[0]
    assert diff.size == 0, "%d mismatches, first %s" % (diff.size, diff[:4])
    # the GPU traces each distinct pixel once; the oracle once per block that needs it
    assert 0 < info["traced_pixels"] <= traced
    # lookahead batching (the default) and one batch per level: the same bits,
    # the same used points, fewer batches
    img2, info2 = pt.render_adaptive(root, W, H, spp, depth, block_size=block, max_interp=max_interp,
                                     min_delta=delta, exact_batches=True)
    np.testing.assert_array_equal(img2.view(np.uint32), img.view(np.uint32))
    assert info2["traced_pixels"] == info["traced_pixels"] and info2["lookahead_pixels"] == 0
    assert info["levels"] <= info2["levels"]
