"""GPU parity: the HIP megakernel (through the C ABI, libpt.so) against the
reference's own outputs (tests/golden/, produced by the unmodified reference
sources) and the CPU oracle.

Bars (BASELINE.json north_star: per-channel RMSE <= 1e-3 on the float
accumulator before tone mapping) -- checked here much more strictly:
  * PT_ORDER_REFERENCE : pixel means bit-identical to the reference's;
  * PT_ORDER_FAST   : bit-identical to the oracle in the fast order,
                         RMSE vs the reference <= 1e-5.
"""
import os

import numpy as np
import pytest

import oracle_py as O
import pathtrace as pt
import zoo as T
from pathtrace import dist as ptdist
from pathtrace import scenes
from pathtrace.scene import to_text

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
RMSE_BAR = 1e-3


def rmse(a, b):
    return np.sqrt(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2, axis=0))


def golden_means(name):
    z = np.load(os.path.join(GOLD, "render_%s.npz" % name))
    ps = z["per_sample"]
    acc = np.zeros((ps.shape[0], 3), dtype=np.float32)
    for s in range(ps.shape[1]):
        acc = (acc + ps[:, s]).astype(np.float32)
    return (acc / np.float32(ps.shape[1])).astype(np.float32)


def tree32(v):
    """pairwise tree of up to 32 float32 rows (n x 3), missing leaves -0.0f"""
    b = np.full((32,) + v.shape[1:], -0.0, dtype=np.float32)
    b[:len(v)] = v
    w = 1
    while w < 32:
        b[0:32:2 * w] = (b[0:32:2 * w] + b[w:32:2 * w]).astype(np.float32)
        w *= 2
    return b[0]


def block_sum(per):
    """the fast order's pixel sum of per-sample values (npx x n x 3):
    blocks of 32 samples, pairwise tree each, blocks added in order"""
    acc = np.zeros((per.shape[0], 3), dtype=np.float32)
    for s in range(0, per.shape[1], 32):
        acc = (acc + np.stack([tree32(px[s:s + 32]) for px in per])).astype(np.float32)
    return acc


def assert_bits(gpu, ref, what):
    gpu = np.ascontiguousarray(gpu, dtype=np.float32).reshape(-1, 3)
    ref = np.ascontiguousarray(ref, dtype=np.float32).reshape(-1, 3)
    diff = np.nonzero(gpu.view(np.uint32) != ref.view(np.uint32))[0]
    assert diff.size == 0, "%s: %d mismatches, first %s gpu=%s ref=%s" % (
        what, diff.size, diff[:4], gpu[diff[:4]], ref[diff[:4]])


@pytest.mark.parametrize("case", T.EXACT_CASES, ids=[c[0] for c in T.EXACT_CASES])
def test_reference_order_bitexact_vs_reference_goldens(built, case):
    name, builder, W, H, spp, depth = case
    g = pt.render(T.build(builder), W, H, spp, depth, order="reference")
    assert_bits(g, golden_means(name), "reference order vs ptref")


@pytest.mark.parametrize("case", T.EXACT_CASES, ids=[c[0] for c in T.EXACT_CASES])
def test_fast_order_bitexact_vs_oracle_and_within_bar(built, tmp_path, case):
    name, builder, W, H, spp, depth = case
    root = T.build(builder)
    g = pt.render(root, W, H, spp, depth, order="fast")
    o = O.render(to_text(root, str(tmp_path)), W, H, spp, depth, order=O.ORDER_FAST)
    assert_bits(g, o, "fast order vs oracle fast order")
    e = rmse(g.reshape(-1, 3), golden_means(name))
    assert np.all(e <= RMSE_BAR) and np.all(e <= 1e-5), e


@pytest.mark.parametrize("order", ["fast", "reference"])
def test_union_rule_overlaps_and_ties_bitexact(built, tmp_path, order):
    """Union-only scene with overlapping, nested and exactly coincident spans
    (equal starts: the union rule must defer to the pairwise checks / the full
    merge): bit-identical to the oracle in both summation orders."""
    root = T.union_zoo()
    W, H, spp, depth = 48, 32, 4, 6
    g = pt.render(root, W, H, spp, depth, order=order)
    o = O.render(to_text(root, str(tmp_path)), W, H, spp, depth,
                 order=O.ORDER_FAST if order == "fast" else O.ORDER_REFERENCE)
    assert_bits(g, o, "union zoo, %s order vs oracle" % order)


LANE_WALK_CASES = [("csg_zoo", 6, 1), ("csg_zoo", 6, 2), ("scene_p0", 4, 2), ("texture_zoo", 5, 2),
                   ("union_zoo", 6, 3)]


@pytest.mark.parametrize("builder,depth,frames", LANE_WALK_CASES)
def test_lane_walk_bitexact(built, tmp_path, builder, depth, frames):
    """pt_scene_set_lane_walk: lanes walk their own scatter-free ray trees
    (mirror / glass / emitter nodes) with a few register frames and hand
    scatter loops and deeper trees to the wave -- the same bits as the oracle
    (1 frame: most glass trees go back to the wave; 2-3: most finish in lanes)."""
    root = T.build(builder)
    W, H, spp = 40, 24, 3
    g = pt.render(pt.DeviceScene(root, lane_walk=frames), W, H, spp, depth, order="fast")
    o = O.render(to_text(root, str(tmp_path)), W, H, spp, depth, order=O.ORDER_FAST)
    assert_bits(g, o, "lane walk %d, %s vs oracle" % (frames, builder))


def test_lane_walk_c5_same_bits(built):
    """C5 (glass ball, sky box with the spherical sky map, skybox sphere) at its
    depth: the per-lane walk gives the wave walk's bits, transcendental
    textures included."""
    cfg = scenes.CONFIGS["C5"]
    rng = np.random.default_rng(3)
    pix = np.sort(rng.choice(cfg.width * cfg.height, 2048, replace=False)).astype(np.int32)
    disk = (1080 + np.arange(-20, 20)[:, None]) * cfg.width + (2460 + np.arange(-20, 20)[None, :])
    pix = np.unique(np.concatenate([pix, disk.ravel().astype(np.int32)]))
    imgs = []
    for frames in (0, cfg.lane_walk or 2):
        ds = pt.DeviceScene(cfg.scene(), workgroups_per_cu=cfg.wg_per_cu, fast_spine=cfg.fast_spine, lane_walk=frames)
        imgs.append(pt.render(ds, cfg.width, cfg.height, 16, cfg.depth, screen=cfg.screen, pixels=pix))
    assert_bits(imgs[1], imgs[0], "C5 lane walk vs wave walk")


@pytest.mark.parametrize("spp", [2, 64])
def test_split_launch_same_bits(built, spp):
    """Split launches (pt_scene_set_split, on by default in lane-walk scenes):
    the light kernel finishes the chunks whose lanes decide every query and
    leaves the rest, whole, to the full kernel -- the same bits and the same
    query counts as every chunk through the full kernel, on C5's hashed pixels
    plus a disk on the glass ball (where the light kernel gives chunks back),
    sample-major (2 spp) and block-staged (64 spp) launches."""
    cfg = scenes.CONFIGS["C5"]
    rng = np.random.default_rng(5)
    pix = np.sort(rng.choice(cfg.width * cfg.height, 4096, replace=False)).astype(np.int32)
    disk = (1080 + np.arange(-24, 24)[:, None]) * cfg.width + (2460 + np.arange(-24, 24)[None, :])
    pix = np.unique(np.concatenate([pix, disk.ravel().astype(np.int32)]))
    out = []
    for split in (True, False):
        ds = pt.DeviceScene(cfg.scene(), workgroups_per_cu=cfg.wg_per_cu, fast_spine=cfg.fast_spine,
                            lane_walk=cfg.lane_walk, split=split)
        out.append(pt.render(ds, cfg.width, cfg.height, spp, cfg.depth, screen=cfg.screen, pixels=pix, stats=True))
    (a, sa), (b, sb) = out
    assert_bits(a, b, "C5 split vs full-kernel launch")
    for k in ("samples", "queries", "shaded"):
        if k in sa:
            assert sa[k] == sb[k], (k, sa[k], sb[k])


# (builder, depth) of the poisoned-LDS test build (test_lds_poison_bitexact)
POISON_CASES = [("scene_p1", 8), ("csg_zoo", 6)]

# (builder, depth) of the lane scatter walk tests
LANE_SCATTER_CASES = [("scatter_zoo", 6), ("csg_zoo", 6), ("union_zoo", 6)]


@pytest.mark.parametrize("order", ["fast", "reference"])
@pytest.mark.parametrize("builder,depth", LANE_SCATTER_CASES)
def test_lane_scatter_bitexact(built, tmp_path, builder, depth, order):
    """pt_scene_set_lane_scatter: lanes walk whole trees, scatter loops
    included (their own engine's draws one attempt after another, the fast
    order's run of <= 64 terms as a binary counter of the pairwise tree): the
    oracle's bits in both orders.  scatter_zoo has loops of 1..64 children that
    recurse, a bright diffuse sphere and zero terms among the non-zero ones."""
    root = T.build(builder)
    W, H, spp = 48, 32, 2
    g, st = pt.render(pt.DeviceScene(root, lane_scatter=True), W, H, spp, depth, order=order, stats=True)
    o = O.render(to_text(root, str(tmp_path)), W, H, spp, depth,
                 order=O.ORDER_FAST if order == "fast" else O.ORDER_REFERENCE)
    assert_bits(g, o, "lane scatter, %s %s order vs oracle" % (builder, order))
    if builder == "scatter_zoo":
        # lanes finished scatter loops: fewer leaf children went through the wave's
        # bursts (the dim floor's plain bursts, ~5 000 leaves a sample, stay there)
        _, st0 = pt.render(pt.DeviceScene(root), W, H, spp, depth, order=order, stats=True)
        assert st["leaf_queries"] < 0.97 * st0["leaf_queries"], (st["leaf_queries"], st0["leaf_queries"])


def test_lane_scatter_run_cap_same_bits(built, tmp_path, monkeypatch):
    """PT_LANE_RUN_CAP=3 (test hook): a lane hands its sample back to the wave
    at the 4th non-zero term of a run, mid-walk, after drawing numbers and
    pushing frames; the wave walks it again from its seed -- the same bits."""
    monkeypatch.setenv("PT_DEVICE_DEFINES", "PT_LANE_RUN_CAP=3")
    root = T.scatter_zoo()
    W, H, spp, depth = 48, 32, 2, 6
    g = pt.render(pt.DeviceScene(root, lane_scatter=True), W, H, spp, depth, order="fast")
    o = O.render(to_text(root, str(tmp_path)), W, H, spp, depth, order=O.ORDER_FAST)
    assert_bits(g, o, "lane scatter, run cap 3")


def c2_bright_pixels(cfg, n, seed):
    """hashed pixels plus pixels on the matBrightDiffuseWhite sphere (the
    fourth sphere, centred near pixel (429, 397) at 1280x720)"""
    rng = np.random.default_rng(seed)
    pix = rng.choice(cfg.width * cfg.height, n, replace=False)
    a, rr = rng.uniform(0, 2 * np.pi, n), 30 * np.sqrt(rng.uniform(0, 1, n))
    disk = (397 + rr * np.sin(a)).astype(np.int64) * cfg.width + (429 + rr * np.cos(a)).astype(np.int64)
    return np.unique(np.concatenate([pix, disk])).astype(np.int32)


@pytest.mark.parametrize("order", ["fast", "reference"])
def test_c2_full_mix_bitexact(built, tmp_path, order):
    """C2 with the reference's full material mix (matBrightDiffuseWhite, src/
    test.cpp:115) at its depth 16, lanes walking the bright sphere's trees
    (the config's setting): bright-sphere and hashed pixels bit for bit against
    the oracle in both orders."""
    cfg = scenes.C2_FULL
    assert cfg.lane_scatter
    root = cfg.scene()
    pix = c2_bright_pixels(cfg, 24, 5)
    g, st = pt.render(cfg.device_scene(), cfg.width, cfg.height, 1, cfg.depth, screen=cfg.screen, pixels=pix,
                      order=order, stats=True)
    o = O.render(to_text(root, str(tmp_path)), cfg.width, cfg.height, 1, cfg.depth, screen=cfg.screen, pixels=pix,
                 order=O.ORDER_FAST if order == "fast" else O.ORDER_REFERENCE)
    assert_bits(g, o, "C2 full mix, %s order vs oracle" % order)
    assert st["queries"] / st["samples"] > 5000  # the bright sphere's samples: ~27 000 queries each


def test_c2_lane_scatter_same_bits_as_wave(built):
    """C2 full mix: the lanes' walk gives the wave walk's bits (4 spp on the
    bright sphere and hashed pixels)."""
    cfg = scenes.C2_FULL
    pix = c2_bright_pixels(cfg, 16, 6)
    imgs = []
    for ls in (False, True):
        ds = pt.DeviceScene(cfg.scene(), workgroups_per_cu=cfg.wg_per_cu, fast_spine=cfg.fast_spine,
                            lane_scatter=ls)
        imgs.append(pt.render(ds, cfg.width, cfg.height, 4, cfg.depth, screen=cfg.screen, pixels=pix))
    assert_bits(imgs[1], imgs[0], "C2 lane scatter vs wave walk")


@pytest.mark.parametrize("builder,depth", [("csg_zoo", 6), ("scene_p1", 8), ("union_zoo", 6)])
def test_fast_spine_bitexact(built, tmp_path, builder, depth):
    """pt_scene_set_fast_spine: wave-walked queries take every span and the
    fast checks first (lazy merge only where they cannot decide): the same
    bits as the oracle on CSG with Difference/Intersection/transforms."""
    root = T.build(builder)
    W, H, spp = 40, 24, 3
    g = pt.render(pt.DeviceScene(root, fast_spine=True), W, H, spp, depth, order="fast")
    o = O.render(to_text(root, str(tmp_path)), W, H, spp, depth, order=O.ORDER_FAST)
    assert_bits(g, o, "fast spine, %s vs oracle" % builder)


def test_full_1080p_frame_on_sampled_pixels(built, tmp_path):
    """BASELINE's full frame size (C3 scene, 1920x1080) at 2 spp: the GPU renders
    every pixel; the oracle checks 1500 hashed pixels bit for bit."""
    cfg = scenes.CONFIGS["C3"]
    root = cfg.scene()
    img, st = pt.render(cfg.device_scene(root=root), cfg.width, cfg.height, 2, cfg.depth, screen=cfg.screen, stats=True)
    rng = np.random.default_rng(7)
    pix = np.sort(rng.choice(cfg.width * cfg.height, 1500, replace=False)).astype(np.int32)
    o = O.render(to_text(root, str(tmp_path)), cfg.width, cfg.height, 2, cfg.depth, screen=cfg.screen,
                 pixels=pix, order=O.ORDER_FAST)
    assert_bits(img.reshape(-1, 3)[pix], o, "1080p sample")
    assert st["samples"] == cfg.width * cfg.height * 2
    assert 300 < st["queries"] / st["samples"] < 2000


@pytest.mark.parametrize("name,spp,npix", [("C1", 4, 2000), ("C2", 2, 300), ("C5", 2, 2000)])
def test_benchmark_configs_on_sampled_pixels(built, tmp_path, name, spp, npix):
    """The other benchmark workloads: C1 (P0), C2 (mirror-ball
    env, depth 16, overlapping half-space sky box: the union rule) and
    C5 (demo world, lens = Intersection, TransformedTexture, skybox, 4K):
    the full frame on the GPU, hashed pixels bit for bit against the oracle."""
    cfg = scenes.CONFIGS[name]
    root = cfg.scene()
    img, st = pt.render(cfg.device_scene(root=root), cfg.width, cfg.height, spp, cfg.depth, screen=cfg.screen, stats=True)
    assert st["samples"] == cfg.width * cfg.height * spp
    rng = np.random.default_rng(11)
    pix = np.sort(rng.choice(cfg.width * cfg.height, npix, replace=False)).astype(np.int32)
    o = O.render(to_text(root, str(tmp_path)), cfg.width, cfg.height, spp, cfg.depth, screen=cfg.screen,
                 pixels=pix, order=O.ORDER_FAST)
    assert_bits(img.reshape(-1, 3)[pix], o, "%s sample" % name)


def test_multipass_equals_single_pass(built):
    """Sample passes bounded by max_buffer_bytes carry the running sums exactly."""
    root = scenes.scene_p1()
    a = pt.render(root, 40, 30, 200, 8)
    b, st = pt.render(root, 40, 30, 200, 8, max_buffer_bytes=40 * 30 * 64 * 12, stats=True)
    assert st["launches"] >= 3
    assert_bits(a, b, "multi-pass")


def test_virtual_ranks_on_one_gpu_sum_to_full_frame(built):
    """Disjoint tile sets rendered separately and summed == the full frame."""
    root = scenes.scene_p0()
    W, H, spp, depth = 70, 45, 3, 4
    full = pt.render(root, W, H, spp, depth).reshape(-1, 3)
    acc = np.zeros_like(full)
    for r in range(3):
        pix = ptdist.rank_pixels(W, H, r, 3, tile=16)
        part = pt.render(root, W, H, spp, depth, pixels=pix)
        frame = np.zeros_like(full)
        frame[pix] = part
        acc = (acc + frame).astype(np.float32)
    assert_bits(acc, full, "3 virtual ranks")


@pytest.mark.parametrize("W,H,spp,depth", [(1, 1, 1, 8), (17, 3, 5, 0), (9, 7, 1, 1), (33, 5, 65, 3)])
def test_edge_shapes_and_depths(built, tmp_path, W, H, spp, depth):
    root = T.csg_zoo()
    g = pt.render(root, W, H, spp, depth)
    o = O.render(to_text(root, str(tmp_path)), W, H, spp, depth, order=O.ORDER_FAST)
    assert_bits(g, o, "edge %dx%d spp %d depth %d" % (W, H, spp, depth))


@pytest.mark.parametrize("npix", [127, 128, 210, 2310, 4096])
def test_sample_major_slot_permutation(built, tmp_path, npix):
    """Launches of <= 64 samples per pixel take their slots in a multiplicative
    permutation (runtime.cpp slot_permutation: a prime near n/phi that does not
    divide n; none below 128 slots).  Pixel-list sizes around the threshold
    and with many small prime factors (210, 2310): every slot rendered once,
    the oracle's bits in both orders."""
    root = T.csg_zoo()
    W, H = 80, 60
    pix = np.sort(np.random.default_rng(npix).choice(W * H, npix, replace=False)).astype(np.int32)
    txt = to_text(root, str(tmp_path))
    ds = pt.DeviceScene(root)
    for order, oo in (("fast", O.ORDER_FAST), ("reference", O.ORDER_REFERENCE)):
        g, st = pt.render(ds, W, H, 3, 6, pixels=pix, order=order, stats=True)
        assert st["samples"] == npix * 3
        assert_bits(g, O.render(txt, W, H, 3, 6, pixels=pix, order=oo), "%d slots, %s" % (npix, order))


def test_empty_pixel_list(built):
    out = pt.render(scenes.scene_p0(), 8, 8, 2, 4, pixels=np.zeros(0, dtype=np.int32))
    assert out.shape == (0, 3)


def test_device_path_with_torch_stream(built):
    import torch
    root = scenes.scene_p1()
    W, H, spp, depth = 32, 20, 4, 8
    ds = pt.DeviceScene(root)
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    s = torch.cuda.Stream()
    params, keep = pt.make_params(W, H, spp, depth)
    pt.prepare(ds, params)
    with torch.cuda.stream(s):
        st = pt.render_device(ds, params, fb.data_ptr(), s.cuda_stream, stats=True)
    s.synchronize()
    assert st["kernel_ms"] > 0 and st["samples"] == W * H * spp
    assert_bits(fb.cpu().numpy(), pt.render(ds, W, H, spp, depth), "device path")


def test_deterministic_across_runs(built):
    root = scenes.scene_p1()
    a = pt.render(root, 48, 32, 8, 8)
    b = pt.render(root, 48, 32, 8, 8)
    assert_bits(a, b, "rerun")


def test_fast_math_paths_bitexact(built):
    """csqrt/cdiv/cnormalize are bit-identical to the compiler's correctly
    rounded sqrtf and '/' (2^28 hashed inputs)."""
    from pathtrace import _lib
    bad = _lib.selftest_math(n=1 << 28, seed=12345)
    assert bad == {"sqrt": 0, "div": 0, "normalize": 0}, bad


@pytest.mark.parametrize("cap", [3, 40])
def test_round_cut_paths_bitexact(built, tmp_path, monkeypatch, cap):
    """A generation round normally takes all 512 of its attempts at once (the
    whole-round path); the per-half replay handles rounds that stop early.
    PT_ROOM_CAP caps the free ring slots a round may fill, so nearly every
    round ends at a ring cut and runs the general replay: the pixels stay
    bit-identical to the oracle."""
    monkeypatch.setenv("PT_DEVICE_DEFINES", "PT_ROOM_CAP=%d" % cap)
    root = scenes.scene_p1()
    W, H, spp, depth = 40, 24, 6, 8
    g = pt.render(root, W, H, spp, depth)
    o = O.render(to_text(root, str(tmp_path)), W, H, spp, depth, order=O.ORDER_FAST)
    assert_bits(g, o, "PT_ROOM_CAP=%d" % cap)


@pytest.mark.parametrize("builder,depth", POISON_CASES)
def test_lds_poison_bitexact(built, tmp_path, monkeypatch, builder, depth):
    """PT_POISON_LDS (test build): every LDS word starts all-ones, so any read
    of LDS state the launch has not written (round 2's j3 failure: kept-only
    position flags read stale flags left by an earlier launch or by a round's
    speculative writes) changes the bits.  Small pixel-list launches -- the
    adaptive caller's shape -- with forced early round ends (PT_ROOM_CAP=3)
    and whole frames, fast and reference order, against the oracle."""
    monkeypatch.setenv("PT_DEVICE_DEFINES", "PT_POISON_LDS=1 PT_ROOM_CAP=3")
    root = T.build(builder)
    txt = to_text(root, str(tmp_path))
    W, H = 40, 28
    rng = np.random.default_rng(3)
    ds = pt.DeviceScene(root)
    for order, oo in (("fast", O.ORDER_FAST), ("reference", O.ORDER_REFERENCE)):
        g = pt.render(ds, W, H, 3, depth, order=order)
        assert_bits(g, O.render(txt, W, H, 3, depth, order=oo), "poisoned LDS, %s frame" % order)
        for n in (1, 7, 70):  # launches far smaller than the grid
            pix = np.sort(rng.choice(W * H, n, replace=False)).astype(np.int32)
            g = pt.render(ds, W, H, 5, depth, pixels=pix, order=order)
            assert_bits(g, O.render(txt, W, H, 5, depth, pixels=pix, order=oo),
                        "poisoned LDS, %s, %d pixels" % (order, n))


def test_c4_eight_shards_on_one_gpu(built, tmp_path):
    """C4's per-rank work: the C3 frame at 1920x1080 cut into the
    8 ranks' hashed 16x16 tile sets (pathtrace.dist.rank_pixels), each shard
    rendered through `pixels=` as its rank would, the zero-filled per-rank
    frames summed as the RCCL reduce does.  Bit-identical to the full frame,
    and the shards' pixels bit-identical to the oracle on hashed pixels
    (replaces the reference's block farm, src/test.cpp:520-778)."""
    cfg = scenes.CONFIGS["C4"]
    root = cfg.scene()
    ds = cfg.device_scene(root=root)
    W, H, spp = cfg.width, cfg.height, 2
    full = pt.render(ds, W, H, spp, cfg.depth, screen=cfg.screen).reshape(-1, 3)
    acc = np.zeros_like(full)
    owner = np.full(W * H, -1)
    for r in range(8):
        pix = ptdist.rank_pixels(W, H, r, 8)
        owner[pix] = r
        part = pt.render(ds, W, H, spp, cfg.depth, screen=cfg.screen, pixels=pix).reshape(-1, 3)
        frame = np.zeros_like(full)
        frame[pix] = part
        acc = (acc + frame).astype(np.float32)
    assert (owner >= 0).all()
    assert_bits(acc, full, "8 shards summed vs full frame")
    rng = np.random.default_rng(44)
    pix = np.sort(rng.choice(W * H, 800, replace=False)).astype(np.int32)
    o = O.render(to_text(root, str(tmp_path)), W, H, spp, cfg.depth, screen=cfg.screen, pixels=pix,
                 order=O.ORDER_FAST)
    assert_bits(acc[pix], o, "8 shards vs oracle")


def test_sample_split_sums(built, tmp_path):
    """bench.py's N-GPU sample split: a call renders samples sample_begin ..
    sample_begin + spp - 1 of every pixel and (sum_only) writes their sum in
    the fast order's pixel order (blocks of 32 from the call's first
    sample, pairwise tree each, blocks in order); the oracle's per-sample
    values summed the same way match bit for bit, and the ranks' sums added
    and divided by the total spp stay within float rounding of the
    single-call frame."""
    root = scenes.scene_p1()
    W, H, S, depth = 40, 24, 12, 8
    per = O.render(to_text(root, str(tmp_path)), W, H, S, depth, order=O.ORDER_FAST, per_sample=True)
    ds = pt.DeviceScene(root)
    total = np.zeros((W * H, 3), dtype=np.float32)
    for b, c in [(0, 5), (5, 4), (9, 3)]:
        g = pt.render(ds, W, H, c, depth, sample_begin=b, sum_only=True).reshape(-1, 3)
        want = block_sum(per[:, b:b + c])
        assert_bits(g, want, "samples %d..%d" % (b, b + c - 1))
        total = (total + g).astype(np.float32)
    full = pt.render(ds, W, H, S, depth).reshape(-1, 3)
    e = rmse(total / np.float32(S), full)
    assert np.all(e <= 1e-6), e


def test_sample_split_block_path(built, tmp_path):
    """The sample split's real shape: shares of more than 64 samples, a
    multiple of 32, the second at a nonzero sample_begin -- the block-staged
    path (one launch, 32-sample block partials in the kernel, reduce mode 2),
    not the per-sample staging of small shares.  Each share's sums equal the
    oracle's per-sample values summed in the fast order's blocks bit for bit."""
    root = scenes.scene_p1()
    W, H, S, depth = 16, 8, 256, 8
    per = O.render(to_text(root, str(tmp_path)), W, H, S, depth, order=O.ORDER_FAST, per_sample=True)
    ds = pt.DeviceScene(root)
    for b, c in [(0, 128), (128, 128)]:
        g, st = pt.render(ds, W, H, c, depth, sample_begin=b, sum_only=True, stats=True)
        assert st["launches"] == 1
        assert_bits(g.reshape(-1, 3), block_sum(per[:, b:b + c]), "samples %d..%d" % (b, b + c - 1))


def test_c4_rank_share_block_path(built):
    """C4's real rank share: the C3 scene at
    1920x1080, ranks 0 and 1 of 8 rendering samples r*512 .. r*512+511 of 1536
    hashed pixels -- enough that the launch takes 32-sample block chunks as a
    whole-frame share does (one launch, block partials in the kernel) -- each
    share's per-pixel sums bit for bit against the oracle's per-sample values
    summed in the fast order's blocks (tests/golden/c4_shares.npz, frozen by
    make_c4_share_golden.py: 1.6 M oracle samples, ~2 min on 8 cores); the two
    shares added within 1e-6 of the 1024-sample sum (association only)."""
    z = np.load(os.path.join(GOLD, "c4_shares.npz"))
    pix = z["pixels"]
    W, H, share, depth, seed = [int(v) for v in z["meta"]]
    cfg = scenes.CONFIGS["C4"]
    assert (W, H, share, depth) == (cfg.width, cfg.height, cfg.spp // 8, cfg.depth)
    ds = cfg.device_scene()
    sums = []
    for r in (0, 1):
        g, st = pt.render(ds, W, H, share, depth, screen=cfg.screen, seed=seed, pixels=pix, sample_begin=r * share,
                          sum_only=True, stats=True)
        assert st["launches"] == 1 and st["samples"] == len(pix) * share
        assert_bits(g, z["sums"][r], "C4 rank %d share" % r)
        sums.append(g)
    both = (sums[0] + sums[1]).astype(np.float32)
    e = rmse(both / np.float32(2 * share), z["both"] / np.float32(2 * share))
    assert np.all(e <= 1e-6), e


@pytest.mark.parametrize("order", ["fast", "reference"])
def test_c2_full_mix_wide_bitexact(built, tmp_path, order):
    """C2's full material mix (matBrightDiffuseWhite, src/test.cpp:115; the
    lane_walk_sc mode) on 128 pixels -- half on the bright sphere -- at 4 spp,
    in both orders, bit for bit against the oracle."""
    cfg = scenes.C2_FULL
    root = cfg.scene()
    pix = c2_bright_pixels(cfg, 64, 8)[:128]
    g = pt.render(cfg.device_scene(), cfg.width, cfg.height, 4, cfg.depth, screen=cfg.screen, pixels=pix,
                  order=order)
    o = O.render(to_text(root, str(tmp_path)), cfg.width, cfg.height, 4, cfg.depth, screen=cfg.screen, pixels=pix,
                 order=O.ORDER_FAST if order == "fast" else O.ORDER_REFERENCE)
    assert_bits(g, o, "C2 full mix 128 px x 4 spp, %s order vs oracle" % order)


@pytest.mark.parametrize("name", ["C3", "C2", "C5"])
def test_config_scale_vs_reference(built, name, tmp_path):
    """Each benchmark config at its real spp and depth against the UNMODIFIED
    reference (tests/golden/config_*.npz, frozen by make_config_golden.py):
    hashed pixels (C5: half on the skybox sphere), reference order bit for bit
    (C5 included: its spherical sky map's glibc atan2f/asinf are restated on
    the device), fast order within RMSE 1e-5 -- except C5, whose 8192-sample
    pixel sums the reference adds sequentially: there the reference itself is
    3.9e-5 RMSE from the float64 mean and the fast order's 32-sample blocks
    5e-7, so the fast order is held to the oracle's fast order
    bit for bit and to the reference at 1e-4 (the north star's bar is 1e-3)."""
    z = np.load(os.path.join(GOLD, "config_%s.npz" % name))
    pix, ref = z["pixels"], z["means"]
    W, H, spp, depth, seed = [int(v) for v in z["meta"][:5]]
    # config_C2.npz holds the benchmarked C2 (no matBrightDiffuseWhite); the
    # full mix is checked against the oracle (test_c2_full_mix_bitexact)
    cfg = scenes.CONFIGS[name]
    ds = cfg.device_scene()
    g = pt.render(ds, W, H, spp, depth, screen=cfg.screen, seed=seed, pixels=pix, order="reference")
    # C5's spherical sky map calls glibc's atan2f / asinf, restated on the
    # device (pt_device.h libm_atan2f / libm_asinf): bits here too
    assert_bits(g, ref, "%s reference order vs ptref" % name)
    f = pt.render(ds, W, H, spp, depth, screen=cfg.screen, seed=seed, pixels=pix, order="fast")
    bar = 1e-5
    if name == "C5":
        o = O.render(to_text(cfg.scene(), str(tmp_path)), W, H, spp, depth, screen=cfg.screen, seed=seed, pixels=pix,
                     order=O.ORDER_FAST)
        assert_bits(f, o, "C5 fast order vs oracle")
        bar = 1e-4
    e = rmse(f, ref)
    assert np.all(e <= bar), e


def test_block_staged_pixel_sums(built, tmp_path):
    """Slot-major launches of whole 32-sample blocks (chunks of 32, >= 4 per
    resident wave) stage one partial per block, the chunk's 32 samples summed
    by the DPP tree; passes of 64 samples stage per-sample values and pt_reduce
    forms the blocks.  Both bit-identical to each other on every pixel and to
    the oracle's fast order (and a numpy restatement of the pixel sum) on
    hashed pixels."""
    root = scenes.scene_p1()
    W, H, spp, depth = 256, 160, 128, 8
    ds = pt.DeviceScene(root)
    one, st1 = pt.render(ds, W, H, spp, depth, stats=True)
    # a budget of 2 floats x 3 per pixel = 64 samples per pass under block staging
    passes, st2 = pt.render(ds, W, H, spp, depth, max_buffer_bytes=W * H * 12 * 2, stats=True)
    assert st1["launches"] == 1 and st2["launches"] == 2
    assert_bits(one, passes, "block-staged vs per-sample passes")
    rng = np.random.default_rng(3)
    pix = np.sort(rng.choice(W * H, 300, replace=False)).astype(np.int32)
    txt = to_text(root, str(tmp_path))
    o = O.render(txt, W, H, spp, depth, pixels=pix, order=O.ORDER_FAST)
    per = O.render(txt, W, H, spp, depth, pixels=pix, order=O.ORDER_FAST, per_sample=True)
    assert_bits(block_sum(per) / np.float32(spp), o, "numpy block sums vs oracle")
    assert_bits(one.reshape(-1, 3)[pix], o, "block-staged vs oracle")


@pytest.mark.gpu
def test_pixel_list_duplicates_and_order(built):
    """A pixel list in any order, with repeats (a caller's blocks overlapping
    at their corners, src/test.cpp:466-499): every entry gets its pixel's
    frame value bit for bit -- the engine is keyed by the pixel, not the slot."""
    W, H, spp, depth = 40, 24, 4, 8
    ds = pt.DeviceScene(scenes.scene_p1())
    frame = pt.render(ds, W, H, spp, depth).reshape(-1, 3)
    pix = np.array([5, 939, 5, 0, 477, 939, 939, 12, W * H - 1, 0], np.int32)
    got = pt.render(ds, W, H, spp, depth, pixels=pix)
    np.testing.assert_array_equal(got.view(np.uint32), frame[pix].view(np.uint32))
