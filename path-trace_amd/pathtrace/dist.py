"""Multi-GPU sharding of one frame.

The frame is cut into square tiles and every tile has exactly one owner.  Each
pixel's samples are seeded by its global index, so each rank writes its own
pixels into a zero-initialised full-frame float3 buffer and one sum-reduce over
RCCL/xGMI (or gloo on CPU) assembles a frame that is bit-identical to a
single-GPU render (x + 0.0 == x).  This replaces the reference's TCP block farm
(src/test.cpp:520-778), whose text protocol also moved each pixel exactly once.

Two deals of the tile grid:

* "lattice" (default, 4x4 tiles): tile (tx, ty) -> rank (tx + LATTICE_STEP * ty)
  mod N.  Any N consecutive tiles of a tile row belong to N different ranks, so
  every rank holds the same share of every region wider than N tiles.  Tile
  cost varies by ~10^3 between sky and diffuse regions but is smooth in space,
  so this stratified deal balances the ranks' work to the cost of a tile edge
  (tools/shard_times.py, profiles/round6/).
* "hashed" (the round-2..5 partition, 16x16 tiles): tiles dealt round-robin in
  a splitmix64-hashed order -- interleaved, but the count of expensive tiles a
  rank receives is binomial: 1.19 max/mean on C4 at 8 ranks
  (profiles/round4/shards_c4_8ranks_tiles.jsonl).
"""
from __future__ import annotations

import numpy as np

TILE = 4            # default tile edge (pixels) of the lattice deal
HASHED_TILE = 16    # the hashed deal's tile edge (rounds 2-5)
LATTICE_STEP = 3    # rank offset between tile rows: odd, so rows shift by a unit coprime to 2^k


def tile_owner(tile_index: np.ndarray, world: int) -> np.ndarray:
    """Deterministic hash of the tile index (splitmix64 finaliser) mod world."""
    z = (np.asarray(tile_index, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15))
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z % np.uint64(world)).astype(np.int64)


def tile_owners(width: int, height: int, world: int, tile: int, deal: str) -> np.ndarray:
    """owner rank of every tile, shape (tiles_y, tiles_x)"""
    tx = (width + tile - 1) // tile
    ty = (height + tile - 1) // tile
    if deal == "lattice":
        xs = np.arange(tx, dtype=np.int64)[None, :]
        ys = np.arange(ty, dtype=np.int64)[:, None]
        return (xs + LATTICE_STEP * ys) % world
    if deal != "hashed":
        raise ValueError("deal must be 'lattice' or 'hashed'")
    # deal tiles round-robin in hashed order: spatially scattered, counts equal to +-1
    order = np.argsort(tile_owner(np.arange(tx * ty), 1 << 30), kind="stable")
    owners = np.empty(tx * ty, dtype=np.int64)
    owners[order] = np.arange(tx * ty) % world
    return owners.reshape(ty, tx)


def rank_pixels(width: int, height: int, rank: int, world: int, tile: int = 0, deal: str = "lattice") -> np.ndarray:
    """Global pixel indices (y * width + x) owned by `rank`, in raster order.
    tile 0 = the deal's default edge (lattice 4, hashed 16)."""
    if world == 1:
        return np.arange(width * height, dtype=np.int32)
    if tile <= 0:
        tile = TILE if deal == "lattice" else HASHED_TILE
    owners = tile_owners(width, height, world, tile, deal)
    ys, xs = np.mgrid[0:height, 0:width]
    mine = owners[ys // tile, xs // tile] == rank
    return (ys * width + xs)[mine].astype(np.int32)


def reduce_frame(fb, group=None):
    """Sum-reduce the per-rank frame buffers to rank 0 (torch.distributed)."""
    import torch.distributed as dist
    dist.reduce(fb, dst=0, op=dist.ReduceOp.SUM, group=group)
    return fb


class RankFrame:
    """One rank's share of a frame, as bench.py renders it (the per-rank step
    of the multi-GPU run; tests/test_dist_gpu.py drives the same object).

    split "samples": the rank renders every pixel (or `subset`) for samples
    [r*spp/N, (r+1)*spp/N) and writes per-pixel sums (sample_begin / sum_only);
    after the sum-reduce rank 0 divides by spp -- tracePixel's mean with the
    ranks' partial sums added in rank order.  split "tiles" (the default since
    round 6): the rank renders the tiles it owns (rank_pixels: `deal`, `tile`)
    as means; the disjoint frames sum-reduce to the single-GPU frame bit for
    bit.  One rank is the plain full render."""

    def __init__(self, ds, width, height, spp, depth, rank=0, world=1, split="tiles", screen=None,
                 subset=None, order="fast", device=0, max_buffer_bytes=0, seed=0x5EED, force_split=False,
                 tile=0, deal="lattice"):
        from . import make_params
        if split not in ("samples", "tiles"):
            raise ValueError("split must be 'samples' or 'tiles'")
        self.ds, self.rank, self.world, self.spp, self.device = ds, rank, world, spp, device
        self.tile = tile if tile > 0 else (TILE if deal == "lattice" else HASHED_TILE)
        # force_split: take the N > 1 path even for one rank (per-pixel sums +
        # the reduce + rank 0's division), e.g. bench.py --force-dist
        self.by_samples = (world > 1 or force_split) and split == "samples"
        mine = rank_pixels(width, height, rank, 1 if self.by_samples else world, tile=tile, deal=deal)
        if subset is not None:
            mine = np.intersect1d(mine, np.asarray(subset)).astype(np.int32)
        self.pixels = mine
        if self.by_samples:
            self.sample_begin = rank * spp // world
            self.sample_count = (rank + 1) * spp // world - self.sample_begin
        else:
            self.sample_begin, self.sample_count = 0, spp
        full = (world == 1 or self.by_samples) and subset is None
        self.params, self._keep = make_params(width, height, self.sample_count, depth, screen=screen, seed=seed,
                                              order=order, device=device, pixels=None if full else mine,
                                              max_buffer_bytes=max_buffer_bytes, sample_begin=self.sample_begin,
                                              sum_only=self.by_samples)

    def prepare(self):
        from . import prepare
        prepare(self.ds, self.params)

    def render(self, fb_ptr, stream_ptr=0, stats=True):
        """this rank's contribution into the zeroed device frame at fb_ptr"""
        from . import render_device
        return render_device(self.ds, self.params, fb_ptr, stream_ptr, stats=stats)

    def render_async(self, fb_ptr, stream_ptr=0):
        """render() queued on the stream without a host wait; collect() sums
        the timings and counters of every render_async since the last one"""
        from . import render_device_timed
        render_device_timed(self.ds, self.params, fb_ptr, stream_ptr)

    def collect(self):
        from . import render_collect
        return render_collect(self.ds, self.device)

    def finish(self, fb):
        """after the sum-reduce to rank 0: the frame of means (torch tensor, in place)"""
        if self.by_samples and self.rank == 0:
            fb.div_(float(self.spp))
        return fb
