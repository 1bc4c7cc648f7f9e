"""bench.py's N > 1 code path rehearsed on one GPU (tests for VERDICT r3 #4):
two ranks under torch.distributed.run with the gloo backend (the frame
reduced through host memory) run exactly the multi-GPU step -- RankFrame's
share, the asynchronous timed render, the reduce, rank 0's division by spp,
the max-over-ranks timing, the roofline divided over ranks, the CPU leg on
rank 0 -- and the reduced frame equals the one-rank frame."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _bench(args, nproc, tmp_path, name, env_extra=None, torchrun=True):
    frame = str(tmp_path / (name + ".npy"))
    cmd = [sys.executable, "-u"]
    if nproc > 1 and torchrun:
        cmd += ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port())]
    cmd += [os.path.join(ROOT, "bench.py"), "--gpus", str(nproc)] + args + ["--dump-frame", frame]
    env = dict(os.environ, OMP_NUM_THREADS="4", **(env_extra or {}))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints one JSON line
    return json.loads(lines[0]), np.load(frame)


@pytest.mark.gpu
@pytest.mark.parametrize("split", ["samples", "tiles"])
def test_bench_two_ranks_gloo(tmp_path, split):
    # 256 spp: each of the two ranks renders 128 samples per pixel, so it takes the
    # block-staged path (whole 32-sample blocks) a real rank share takes
    common = ["--config", "C3", "--spp", "256", "--steps", "1", "--warmup", "0", "--cpu-pixels", "16"]
    one, f1 = _bench(common + ["--no-cpu"], 1, tmp_path, "one")
    two, f2 = _bench(common + ["--backend", "gloo", "--split", split, "--cpu-at-n"], 2, tmp_path, "two")
    assert two["n_gpus"] == 2 and two["steps"] == 1
    assert "gloo reduce" in two["config"]["sharding"]
    assert ("spp split" in two["config"]["sharding"]) == (split == "samples")
    assert two["samples_per_step"] == one["samples_per_step"] == 1920 * 1080 * 256
    rk = two["ranks"]  # each rank's own numbers, as the driver's N-GPU line carries them
    assert len(rk["kernel_ms_per_launch"]) == 2 and rk["kernel_imbalance_max_over_mean"] >= 1.0
    assert sum(rk["pixels"]) == (1920 * 1080 * (2 if split == "samples" else 1))
    assert sum(rk["queries"]) == pytest.approx(two["queries_per_sample"] * two["samples_per_step"], rel=1e-4)
    # the same frame: the same span queries in total, split over the ranks
    assert two["queries_per_sample"] == pytest.approx(one["queries_per_sample"], rel=1e-9)
    # roofline: each rank's launches carry half the work; the kernel time is the max over ranks
    rf = two["roofline"]
    assert rf["kernel"] == "pt_render_fast" and rf["avg_launch_ms"] > 0
    ops_launch = rf["ops_per_query"] * two["queries_per_sample"] * two["samples_per_step"] / 2
    assert rf["achieved"] == pytest.approx(ops_launch / (rf["avg_launch_ms"] * 1e-3) / 1e12, rel=2e-3)
    # rank 0 ran the CPU leg after the timed region, on the reduced frame
    assert two["cpu_baseline"]["kind"] in ("reference", "port") and two["cpu_baseline"]["value"] > 0
    assert max(two["rmse_vs_cpu_ref"]) < 1e-3
    if split == "tiles":  # disjoint tiles: x + 0.0 == x
        np.testing.assert_array_equal(f2.view(np.uint32), f1.view(np.uint32))
    else:  # the ranks' partial sums change the association only
        rmse = np.sqrt(np.mean((f2.astype(np.float64) - f1) ** 2, axis=(0, 1)))
        assert rmse.max() <= 1e-6, rmse


@pytest.mark.gpu
def test_bench_force_dist_rccl_world1(tmp_path):
    """the RCCL leg of bench.py executed -- init_process_group("nccl",
    device_id=...), the device dist.reduce of the frame, the CUDA-tensor MAX / SUM
    all-reduces and rank 0's division -- as a one-rank group on one GPU.  The
    rank renders per-pixel sums (sum_only) and the frame after the reduce and the
    division by spp is the plain one-GPU frame bit for bit (the kernel's mean is
    the same sum divided by the same spp)."""
    common = ["--config", "C3", "--spp", "64", "--steps", "2", "--warmup", "1", "--no-cpu"]
    one, f1 = _bench(common, 1, tmp_path, "plain")
    d, f2 = _bench(common + ["--force-dist"], 1, tmp_path, "rccl")
    assert d["n_gpus"] == 1 and d["steps"] == 2
    assert "RCCL reduce" in d["config"]["sharding"] and "force-dist" in d["config"]["sharding"]
    assert d["samples_per_step"] == one["samples_per_step"]
    assert d["queries_per_sample"] == pytest.approx(one["queries_per_sample"], rel=1e-9)
    assert d["roofline"]["traffic"] is None and "default one-GPU command" in d["roofline"]["traffic_note"]
    np.testing.assert_array_equal(f2.view(np.uint32), f1.view(np.uint32))


@pytest.mark.gpu
def test_bench_gpus_two_without_torchrun(tmp_path):
    """`bench.py --gpus 2` with no torchrun starts the two ranks
    itself (here over gloo, both on the box's one GPU) and reports n_gpus 2;
    the default partition (4x4 tiles, lattice deal) reduces to the one-rank
    frame bit for bit."""
    common = ["--config", "C3", "--spp", "64", "--steps", "1", "--warmup", "0", "--no-cpu"]
    one, f1 = _bench(common, 1, tmp_path, "one")
    two, f2 = _bench(common + ["--backend", "gloo"], 2, tmp_path, "two", torchrun=False)
    assert two["n_gpus"] == 2
    assert "4x4 tiles, lattice deal" in two["config"]["sharding"]
    assert two["samples_per_step"] == one["samples_per_step"]
    np.testing.assert_array_equal(f2.view(np.uint32), f1.view(np.uint32))


@pytest.mark.gpu
def test_bench_more_gpus_than_the_box_has(tmp_path):
    """--gpus 3 over RCCL on a one-GPU box exits non-zero without a line"""
    import torch
    n = torch.cuda.device_count() + 2
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--no-cpu"],
                       capture_output=True, text=True, timeout=120, cwd=ROOT,
                       env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert r.returncode != 0 and "GPU(s) visible" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
