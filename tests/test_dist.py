"""Multi-GPU sharding (pathtrace.dist) on CPU: the tile partition covers every
pixel exactly once, and a world-size-2 gloo run (each rank renders its tiles,
then one sum-reduce) reproduces the single-process frame bit for bit.  The
per-rank renderer here is the CPU oracle (no GPU in this container); the
reduce is the exact call bench.py makes over RCCL."""
import os
import socket

import numpy as np
import pytest

from pathtrace import dist as ptdist


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_partition_is_exact_cover(world):
    W, H = 100, 37
    parts = [ptdist.rank_pixels(W, H, r, world) for r in range(world)]
    allpix = np.concatenate(parts)
    assert len(allpix) == W * H
    assert len(np.unique(allpix)) == W * H
    if world > 1:
        sizes = [len(p) for p in parts]
        assert min(sizes) > 0


def test_partition_balance_1080p():
    sizes = [len(ptdist.rank_pixels(1920, 1080, r, 8)) for r in range(8)]
    assert max(sizes) / min(sizes) < 1.1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, txt, W, H, spp, depth, out_path):
    import torch
    import torch.distributed as dist
    import oracle_py as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pix = ptdist.rank_pixels(W, H, rank, world, tile=4)
    fb = torch.zeros(W * H * 3, dtype=torch.float32)
    vals = O.render(txt, W, H, spp, depth, pixels=pix, threads=2, order=O.ORDER_FAST)
    fb.view(-1, 3)[torch.from_numpy(pix.astype(np.int64))] = torch.from_numpy(vals)
    ptdist.reduce_frame(fb)
    if rank == 0:
        np.save(out_path, fb.numpy())
    dist.destroy_process_group()


def test_gloo_two_ranks_bitexact(built, tmp_path):
    import torch.multiprocessing as mp
    import oracle_py as O
    from pathtrace import scenes
    from pathtrace.scene import to_text
    W, H, spp, depth = 24, 16, 2, 8
    txt = to_text(scenes.scene_p1(), str(tmp_path))
    out = str(tmp_path / "fb.npy")
    mp.spawn(_worker, args=(2, _free_port(), txt, W, H, spp, depth, out), nprocs=2, join=True)
    got = np.load(out).reshape(-1, 3)
    want = O.render(txt, W, H, spp, depth, order=O.ORDER_FAST)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


def _split_worker(rank, world, port, txt, W, H, spp, depth, out_path):
    import torch
    import torch.distributed as dist
    import oracle_py as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, e = rank * spp // world, (rank + 1) * spp // world
    per = O.render(txt, W, H, spp, depth, threads=2, order=O.ORDER_FAST, per_sample=True)[:, b:e]
    acc = np.zeros((W * H, 3), dtype=np.float32)
    for s in range(per.shape[1]):  # this rank's samples, summed in sample order (sum_only)
        acc = (acc + per[:, s]).astype(np.float32)
    fb = torch.from_numpy(acc.reshape(-1).copy())
    ptdist.reduce_frame(fb)
    if rank == 0:
        fb.div_(float(spp))
        np.save(out_path, fb.numpy())
    dist.destroy_process_group()


def test_gloo_sample_split_two_ranks(built, tmp_path):
    """bench.py's default N>1 split: every rank renders all pixels for its
    share of the samples and sends per-pixel sums; rank 0 divides the reduced
    sums by spp.  Equals the single-process frame within float rounding of the
    changed summation order (RMSE far below the 1e-3 bar)."""
    import torch.multiprocessing as mp
    import oracle_py as O
    from pathtrace import scenes
    from pathtrace.scene import to_text
    W, H, spp, depth = 24, 16, 6, 8
    txt = to_text(scenes.scene_p1(), str(tmp_path))
    out = str(tmp_path / "fb.npy")
    mp.spawn(_split_worker, args=(2, _free_port(), txt, W, H, spp, depth, out), nprocs=2, join=True)
    got = np.load(out).reshape(-1, 3).astype(np.float64)
    want = O.render(txt, W, H, spp, depth, order=O.ORDER_FAST).astype(np.float64)
    rmse = np.sqrt(np.mean((got - want) ** 2, axis=0))
    assert np.all(rmse < 1e-6), rmse
    assert np.abs(got - want).max() <= 1e-6 * max(1.0, np.abs(want).max())


@pytest.mark.parametrize("world", [2, 3, 8])
def test_lattice_rows_are_stratified(world):
    """the lattice deal: any `world` consecutive tiles of a tile row have `world` different owners"""
    own = ptdist.tile_owners(1920, 1080, world, ptdist.TILE, "lattice")
    for row in own[:: max(1, own.shape[0] // 17)]:
        for x in range(0, own.shape[1] - world + 1, 7):
            assert len(set(row[x:x + world].tolist())) == world


def test_lattice_balances_a_clustered_cost_map():
    """tile cost clustered in space (a few bright disks on a cheap sky, the
    shape of C3's frame): the 4x4 lattice balances 8 ranks far better than
    16x16 hashed tiles (measured on the GPU: C3 1.030 vs 1.158,
    profiles/round6/shards_*.jsonl)"""
    W, H = 1920, 1080
    ys, xs = np.mgrid[0:H, 0:W]
    cost = np.ones((H, W))
    for cx, cy, r in [(700, 540, 180), (1250, 560, 200), (960, 700, 90)]:
        cost += 900.0 * (((xs - cx) ** 2 + (ys - cy) ** 2) < r * r)
    flat = cost.reshape(-1)

    def imbalance(deal, tile):
        work = [flat[ptdist.rank_pixels(W, H, r, 8, tile=tile, deal=deal)].sum() for r in range(8)]
        return max(work) / np.mean(work)

    lat, hashed = imbalance("lattice", 4), imbalance("hashed", 16)
    assert lat < 1.01 and lat < hashed, (lat, hashed)


@pytest.mark.parametrize("W,H,world,tile", [(1920, 1080, 8, 4), (100, 37, 3, 4), (64, 40, 2, 1), (33, 17, 5, 8)])
def test_c_abi_partition_equals_python(built, W, H, world, tile):
    """pt_rank_pixels (the C hosts' partition) is pathtrace.dist.rank_pixels' lattice deal"""
    import ctypes
    from pathtrace import _lib
    L = _lib.lib()
    for r in range(world):
        n = ctypes.c_int64(0)
        _lib.check(L.pt_rank_pixels(W, H, r, world, tile, None, 0, ctypes.byref(n)))
        out = np.zeros(max(1, n.value), np.int32)
        _lib.check(L.pt_rank_pixels(W, H, r, world, tile, out.ctypes.data, n.value, ctypes.byref(n)))
        np.testing.assert_array_equal(out[:n.value], ptdist.rank_pixels(W, H, r, world, tile=tile))
