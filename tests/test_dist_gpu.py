"""The multi-GPU step through the HIP kernel, on one GPU: two ranks (gloo,
both on cuda:0) run bench.py's own per-rank step (pathtrace.dist.RankFrame:
render_device into a zeroed device frame, sample split with sum_only or hashed
tiles), reduce host copies of their frames to rank 0, which finishes the frame
as bench.py does.  Against the one-rank frame of the same kernel: tiles bit for
bit, samples within RMSE 1e-6 (the ranks' partial sums add in another order).
Each rank's sample share is 128 of 256 spp, so the sample split runs the
block-staged path (32-sample block partials, sample_begin 128 on rank 1)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, SPP, DEPTH = 64, 40, 256, 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, split, out_path):
    import torch
    import torch.distributed as dist
    import pathtrace as pt
    from pathtrace import dist as ptdist
    from pathtrace import scenes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    ds = pt.DeviceScene(scenes.scene_p1())
    share = ptdist.RankFrame(ds, W, H, SPP, DEPTH, rank=rank, world=world, split=split)
    share.prepare()
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    st = share.render(fb.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    host = fb.cpu()
    ptdist.reduce_frame(host)
    share.finish(host)
    if rank == 0:
        np.save(out_path, host.numpy())
    np.save(out_path + ".%d.npy" % rank, np.array([st["launches"], share.sample_begin, share.sample_count,
                                                   len(share.pixels)]))
    dist.destroy_process_group()


@pytest.mark.parametrize("split", ["samples", "tiles"])
def test_two_ranks_through_the_hip_kernel(built, tmp_path, split):
    import torch.multiprocessing as mp
    import pathtrace as pt
    from pathtrace import scenes
    out = str(tmp_path / "fb.npy")
    mp.spawn(_rank, args=(2, _free_port(), split, out), nprocs=2, join=True)
    got = np.load(out).reshape(-1, 3)
    one = pt.render(pt.DeviceScene(scenes.scene_p1()), W, H, SPP, DEPTH).reshape(-1, 3)
    info = [np.load(out + ".%d.npy" % r) for r in range(2)]
    if split == "tiles":
        np.testing.assert_array_equal(got.view(np.uint32), one.view(np.uint32))
        assert sum(int(i[3]) for i in info) == W * H
    else:
        assert [int(i[1]) for i in info] == [0, SPP // 2] and all(int(i[2]) == SPP // 2 for i in info)
        assert all(int(i[0]) == 1 for i in info)  # one block-staged launch per rank
        e = np.sqrt(np.mean((got.astype(np.float64) - one) ** 2, axis=0))
        assert np.all(e <= 1e-6), e
