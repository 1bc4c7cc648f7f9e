"""bench.py's launcher: `bench.py --gpus N` without torchrun
starts N ranks itself -- the driver's scaling run can never print a one-rank
line for N GPUs -- and a mismatch between the ranks launched, --gpus and the
visible GPUs exits non-zero.  On CPU the ranks run --dry-run (process group,
barrier, max over ranks, rank 0's JSON line; no render)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=300):
    env = dict(os.environ, OMP_NUM_THREADS="2", **(env_extra or {}))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        if not env_extra or k not in env_extra:
            env.pop(k, None)
    return subprocess.run([sys.executable, "-u", BENCH] + args, capture_output=True, text=True, timeout=timeout,
                          cwd=ROOT, env=env)


def _line(r):
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout + r.stderr[-3000:]
    return json.loads(lines[0])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--backend", "gloo", "--no-cpu", "--dry-run"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r)
    assert out["dry_run"] is True and out["value"] is None
    assert out["n_gpus"] == n and out["ranks_joined"] == n
    assert out["split"] == "tiles" and out["deal"] == "lattice"  # the default partition


def test_gpus_one_is_a_plain_rank():
    out = _line(_run(["--gpus", "1", "--backend", "gloo", "--dry-run"]))
    assert out["n_gpus"] == 1 and out["ranks_joined"] == 1


def test_world_size_must_equal_gpus():
    """under torchrun, a WORLD_SIZE other than --gpus is refused before any work"""
    env = {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
           "MASTER_PORT": str(_free_port())}
    r = _run(["--gpus", "8", "--dry-run"], env_extra=env, timeout=60)
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 8" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_more_gpus_than_visible_exits_nonzero():
    """--gpus above the visible GPUs over RCCL: non-zero, no line (this container has none;
    on the one-GPU box tests/test_bench_dist.py checks --gpus 3)"""
    import torch
    n = torch.cuda.device_count() + 1
    r = _run(["--gpus", str(n), "--no-cpu"], timeout=60)
    assert r.returncode != 0 and "GPU(s) visible" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_split_env_parsed_like_the_runtime():
    """PT_SPLIT is read with the runtime's atoi rule (runtime.cpp split_launches)"""
    sys.path.insert(0, ROOT)
    import bench
    for v, on in [("", True), ("0", False), ("1", True), ("false", False), ("off", False), ("00", False),
                  (" 2x", True), ("-0", False)]:
        os.environ["PT_SPLIT"] = v
        try:
            assert bench.split_launches_env() is on, v
        finally:
            del os.environ["PT_SPLIT"]
