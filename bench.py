"""bench.py -- BASELINE.json's headline metric on MI355X:
Msamples/s at 1920x1080x1024spp (config C3: 6-sphere union/difference CSG +
sky wall, depth 8), with the per-channel RMSE of the GPU frame against the
reference CPU renderer on a hashed pixel subset.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU)

Launch.  Without torchrun (no WORLD_SIZE in the environment) and --gpus N > 1,
this process starts N rank processes itself (a torch.distributed.run child on
127.0.0.1) and exits with their status; it decides that before any GPU call and
never runs a rank itself.  Under torchrun WORLD_SIZE must equal --gpus, and
over RCCL --gpus may not exceed the visible GPUs: either mismatch exits
non-zero, never falling back to fewer ranks.

One step = one full frame.  N = 1: the HIP megakernel (libpt.so, C ABI)
renders every pixel into a device frame buffer.  N > 1 (--split tiles, the
default): every rank renders the 4x4 tiles it owns in the lattice deal
(pathtrace.dist: any N consecutive tiles of a row go to N different ranks),
and the disjoint frames are sum-reduced to rank 0 over RCCL -- bit-identical to
the one-GPU frame; --split samples: every rank renders every pixel for its
share of the samples (sample_begin / sum_only), the per-pixel sums are reduced
and divided by spp.  The timed region is bracketed by barrier + device
synchronise and the max over ranks is reported.  Inputs (the scene) are
resident before timing.

Extra fields: `roofline` (VALU-bound: the SURVEY.md s8(d) FP32 op model per
root query x the kernel's exact query count / HIP-event kernel time, against
78.6 T non-FMA FP32 op/s) and `cpu_baseline` (the unmodified reference sources,
oracle/_ref/ptref, on the GPU box's host cores over a bounded pixel sample of
the same frame, rank 0 only).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "path-trace_amd"), os.path.join(ROOT, "oracle")]

VALU_PEAK_TOPS = 78.6  # 256 CU x 128 FP32 lanes/clk x 2.4 GHz, no FMA (contraction off for parity)
# SURVEY.md s8(d) op model calibrated by tools/calibrate_ops.py (oracle event
# counts on hashed pixels): C3 8192 px x 32 spp, C2 512 px x 4 spp, C5 8192 px x 64 spp.
# Since round 6 it counts the texture maps' work too (one weight per texture
# evaluation by class, calibrate_ops.TEX_W): C2's mirror-ball sky 37.19 ops per
# query, C5's spherical sky + skybox 125.65; C3 has constant textures only.
OPS_PER_QUERY = {"C3": 438.75, "C4": 438.75, "C2": 651.97, "C5": 679.78}
# Counter evidence of this same command (tools/evidence.sh -> tools/pmc_bench.sh:
# rocprofv3 --pmc passes of bench.py; VALUBusy, HBM bytes = FETCH_SIZE x 2 +
# WRITE_SIZE).  Each file records the code-object key of the kernel its passes
# ran; the line attaches it only when that key is the key of the kernel it timed.
PMC_JSON = os.path.join(ROOT, "profiles", "round6", "pmc_bench_%s.json")
# bounded CPU samples at full spp on the box's per-GPU CPU share (16 threads):
# BASELINE.md's 4096 hashed pixels (C3: ~60 s), fewer where a pixel costs more
CPU_PIXELS = {"C1": 4096, "C2": 512, "C3": 4096, "C4": 1024, "C5": 32768}
# C5 (3840x2160 x 8192 spp, 68 G samples) is timed on one GPU on a hashed pixel
# subset at its full spp and depth: at that size the reference camera
# (|d| = 4320) hides everything nearer than 4.32 units, so the frame is the sky
# box, the skybox sphere and the far side of the glass ball (~6 % of pixels,
# ~60x the cost of a sky pixel); a hashed subset of 65536 pixels holds the same
# mix.  On N > 1 GPUs the whole frame is rendered.
SUBSET_1GPU = {"C5": 65536}


def pmc_evidence(cfg_name: str, kernel_key: str):
    """(PMC summary, None) when profiles/.../pmc_bench_<cfg>.json was collected
    on the code object just timed, else (None, why not)."""
    path = PMC_JSON % cfg_name
    try:
        with open(path) as f:
            ev = json.load(f)
    except (OSError, ValueError):
        return None, "no counter file %s" % os.path.relpath(path, ROOT)
    if ev.get("kernel_key") != kernel_key:
        return None, "%s was collected on code object %s, not on the timed %s" % (
            os.path.relpath(path, ROOT), ev.get("kernel_key"), kernel_key)
    return ev, None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=0)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--spp", type=int, default=0, help="override (for quick local probes only; invalid metric)")
    ap.add_argument("--cpu-pixels", type=int, default=0, help="0 = the config's bounded sample (CPU_PIXELS)")
    ap.add_argument("--subset", type=int, default=-1,
                    help="render only this many hashed pixels at full spp (-1 = config default: a subset for C5 on "
                         "one GPU, else the whole frame; 0 = whole frame)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = the CPUs this process may run on (sched_getaffinity), capped by OMP_NUM_THREADS "
                         "when set (the GPU box exports its per-GPU CPU share there)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-at-n", action="store_true",
                    help="N > 1: also run the CPU baseline and the RMSE on rank 0 (default: the N = 1 line only)")
    ap.add_argument("--dump-frame", default="", help="rank 0: save the reduced frame (H x W x 3 f32 .npy)")
    ap.add_argument("--order", default="fast")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="N>1: RCCL over xGMI (nccl), or gloo with the frame reduced through host memory -- "
                         "rehearses the N>1 code path with several ranks on one GPU")
    ap.add_argument("--force-dist", action="store_true",
                    help="take the N > 1 step at any world size: torch.distributed over RCCL (a one-rank group "
                         "when launched without torchrun), per-pixel sums, the device reduce, rank 0's division")
    ap.add_argument("--split", choices=["samples", "tiles"], default="tiles",
                    help="N>1: each rank renders the tiles it owns (bit-identical to 1 GPU), or every pixel for "
                         "its share of the samples (per-pixel sums, ~1e-7 relative reassociation)")
    ap.add_argument("--deal", choices=["lattice", "hashed"], default="lattice",
                    help="--split tiles: tile (tx, ty) -> rank (tx + 3 ty) mod N, or round-robin in hashed order")
    ap.add_argument("--tile", type=int, default=0, help="tile edge in pixels (0 = the deal's default: 4 / 16)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch and rank plumbing only (process group, barrier, max over ranks, rank 0's line) "
                         "with no render: prints a line with value null and dry_run true")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def visible_gpus() -> int:
    """GPUs this process could use (torch.cuda.device_count does not initialise HIP)."""
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:
        return 0


def launch_check(args):
    """Decide, before any GPU call, whether this process is a rank or the
    launcher of --gpus ranks.  Returns None for a rank, else an exit status."""
    env_world = os.environ.get("WORLD_SIZE")
    need_gpus = not args.dry_run and args.backend == "nccl"
    if env_world is not None:  # launched by torch.distributed.run (the driver's N > 1 form, or ours)
        if int(env_world) != args.gpus:
            print("bench.py: WORLD_SIZE=%s but --gpus %d: refusing to report a %s-rank run as %d GPUs" % (
                env_world, args.gpus, env_world, args.gpus), file=sys.stderr)
            return 2
        if need_gpus and int(os.environ.get("LOCAL_RANK", "0")) >= visible_gpus():
            print("bench.py: LOCAL_RANK %s has no GPU (%d visible)" % (os.environ.get("LOCAL_RANK"),
                                                                      visible_gpus()), file=sys.stderr)
            return 2
        return None
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        return 2
    if need_gpus and args.gpus > visible_gpus():
        print("bench.py: --gpus %d but %d GPU(s) visible" % (args.gpus, visible_gpus()), file=sys.stderr)
        return 2
    if args.gpus == 1:
        return None
    # N > 1 without torchrun: start N ranks (fresh processes: this one has not touched the GPU)
    env = dict(os.environ)
    if "OMP_NUM_THREADS" not in env:  # torchrun would pin it to 1 and starve rank 0's CPU leg
        env["OMP_NUM_THREADS"] = str(len(os.sched_getaffinity(0)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    rc = subprocess.call(cmd, env=env)
    return rc if rc >= 0 else 128 - rc  # a rank launcher killed by a signal: the shell's 128 + signal


def _atoi(text: str) -> int:
    """C atoi: leading blanks, an optional sign, the leading digits; 0 if none"""
    import re
    m = re.match(r"\s*([+-]?\d+)", text)
    return int(m.group(1)) if m else 0


def split_launches_env() -> bool:
    """the runtime's split_launches() (runtime.cpp): PT_SPLIT unset or empty = on, else atoi != 0"""
    v = os.environ.get("PT_SPLIT", "")
    return True if not v else _atoi(v) != 0


def dry_run(args):
    """--dry-run: the rank plumbing of main() without the GPU (CPU tests of the launcher)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if "MASTER_ADDR" not in os.environ:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1")
    dist.init_process_group("gloo")
    dist.barrier()
    t0 = time.perf_counter()
    dist.barrier()
    elapsed = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    ranks = torch.tensor([1.0])
    dist.all_reduce(ranks, op=dist.ReduceOp.SUM)
    if rank == 0:
        print(json.dumps({"metric": "Msamples/sec at 1920x1080x1024spp; per-channel RMSE vs CPU ref",
                          "value": None, "dry_run": True, "n_gpus": world, "ranks_joined": int(ranks[0]),
                          "steps": args.steps, "warmup": args.warmup, "split": args.split, "deal": args.deal}),
              flush=True)
    dist.destroy_process_group()


def cpu_threads(requested: int) -> int:
    """Host threads for the CPU baseline: the CPUs this process may use, capped
    by OMP_NUM_THREADS (the GPU box's per-GPU CPU share) when that is set."""
    if requested > 0:
        return requested
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(cfg, txt, spp, npix, threads, frame_qps, within=None):
    """The reference's own hot path (tracePixel per (pixel, sample), src/test.cpp:450;
    one std::thread per host core as RenderBlock's pool, src/test.cpp:204) over a
    hashed pixel subset of the same frame.  Per-sample cost is bimodal (sky vs
    diffuse pixels), so the subset's queries/sample is reported beside the
    frame's and the rate is also given rescaled by their ratio (CPU time is
    proportional to span queries)."""
    import oracle_py as O
    rng = np.random.default_rng(0x5EED)
    pool = cfg.width * cfg.height if within is None else np.asarray(within)
    pix = np.sort(rng.choice(pool, min(npix, len(pool) if within is not None else npix), replace=False))
    pix = pix.astype(np.int32)
    npix = len(pix)
    qps = None
    if O.ref_available():
        kind = "reference"
        res, info = O.ref_render(txt, cfg.width, cfg.height, spp, cfg.depth, screen=cfg.screen, pixels=pix,
                                 threads=threads, info=True)
        secs = info["seconds"]
        qps = info["queries"] / (npix * spp)
    else:  # restated oracle (same arithmetic, pinned to the reference by tests/golden)
        kind = "port"
        t0 = time.time()
        res, st = O.render(txt, cfg.width, cfg.height, spp, cfg.depth, screen=cfg.screen, pixels=pix,
                           threads=threads, stats=True)
        secs = time.time() - t0
        qps = st["queries"] / (npix * spp)
    value = npix * spp / secs / 1e6
    host = len(os.sched_getaffinity(0))
    out = {"value": round(value, 5), "unit": "Msamples/s", "cores": threads, "kind": kind,
           "host_cpus": os.cpu_count(), "affinity_cpus": host,
           "sample": "%d hashed pixels x %d spp of the same frame (%.1f s)" % (npix, spp, secs),
           "sample_queries_per_sample": round(qps, 2)}
    scal = None
    try:  # the measured thread scaling of this baseline (tools/cpu_scaling.py on a GPU box)
        with open(os.path.join(ROOT, "profiles", "round6", "cpu_scaling.json")) as f:
            rows = json.load(f)["C3_sample_scaling"]["rows"]
        scal = {"threads": [r["threads"] for r in rows],
                "parallel_efficiency": [round(r["parallel_efficiency"], 3) for r in rows],
                "file": "profiles/round6/cpu_scaling.json"}
    except (OSError, ValueError, KeyError):
        pass
    if scal:
        out["thread_scaling_measured"] = scal
    if host > threads:
        # the reference pool spawns hardware_concurrency() threads (src/test.cpp:204); the
        # GPU box asks for its per-GPU CPU share only, so the whole host is a projection
        # (pixels are independent: linear is an upper bound -- the measured 8 -> 16 step
        # is below it, thread_scaling_measured)
        out["all_host_cpus_projected"] = {
            "value": round(value * host / threads, 5), "cores": host,
            "how": "linear from the measured %d threads (not measured; an upper bound)" % threads,
            "why_not_measured": "the GPU box gives each GPU job a %d-thread CPU share (OMP_NUM_THREADS); the "
                                "reference pool's hardware_concurrency() threads (src/test.cpp:204) would take the "
                                "other GPUs' shares of this %d-CPU host" % (threads, host)}
    if frame_qps:
        out["frame_queries_per_sample"] = round(frame_qps, 2)
        out["value_rescaled_to_frame"] = round(value * qps / frame_qps, 5)
    return pix, res, out


def main():
    args = parse()
    status = launch_check(args)
    if status is not None:
        sys.exit(status)
    if args.dry_run:
        dry_run(args)
        return
    import torch
    import pathtrace as pt
    from pathtrace import dist as ptdist
    from pathtrace import scenes
    from pathtrace.scene import to_text

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_dist = world > 1 or args.force_dist
    gloo = use_dist and args.backend == "gloo"
    if gloo:  # rehearsal: ranks may share a GPU
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if use_dist:
        import torch.distributed as dist
        if "MASTER_ADDR" not in os.environ:  # --force-dist without torchrun: a one-rank group
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1")
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist = None

    cfg = scenes.CONFIGS[args.config]
    spp = args.spp or cfg.spp
    W, H = cfg.width, cfg.height
    root = cfg.scene()
    ds = cfg.device_scene(root=root)
    subset = (SUBSET_1GPU.get(cfg.name, 0) if world == 1 else 0) if args.subset < 0 else args.subset
    keep = None
    if subset:
        rng = np.random.default_rng(0x5EED)
        keep = np.sort(rng.choice(W * H, subset, replace=False)).astype(np.int32)
    # this rank's share (pathtrace.dist.RankFrame, also driven by tests/test_dist_gpu.py)
    share = ptdist.RankFrame(ds, W, H, spp, cfg.depth, rank=rank, world=world, split=args.split,
                             screen=cfg.screen, subset=keep, order=args.order, device=local,
                             max_buffer_bytes=40 << 30, force_split=use_dist, tile=args.tile, deal=args.deal)
    kernel_key = ds.kernel_key(cfg.depth)
    # lane-walk scenes render in split launches (runtime.cpp: pt_render_light over every chunk, then
    # pt_render_fast over the chunks it left; PT_SPLIT=0 turns them off); one render = one "launch" here
    split = cfg.lane_walk and args.order == "fast" and split_launches_env()
    render_kernels = "pt_render_light + pt_render_fast" if split else "pt_render_fast"
    by_samples, mine = share.by_samples, share.pixels
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream()
    # untimed: load the code object, upload the scene, allocate every buffer
    share.prepare()
    torch.cuda.synchronize()

    def reduce_frame():
        if gloo:  # through host memory
            h = fb.cpu()
            dist.reduce(h, dst=0, op=dist.ReduceOp.SUM)
            if rank == 0:
                fb.copy_(h)
        else:
            dist.reduce(fb, dst=0, op=dist.ReduceOp.SUM)

    def step():
        # the render is queued without a host wait (its HIP-event timings are
        # collected after the timed region): the reduce follows it on the stream
        fb.zero_()
        share.render_async(fb.data_ptr(), stream.cuda_stream)
        if dist is not None:
            reduce_frame()
            share.finish(fb)  # rank 0, sample split: the ranks' sums over spp

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    share.collect()  # drop the warm-up timings
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = share.collect()
    kernel_ms = st["kernel_ms"] / max(1, st["launches"])
    launches_per_step = st["launches"] // max(1, args.steps)
    queries = st["queries"]
    per_rank = None
    if dist is not None:  # RCCL: CUDA tensors; gloo: host tensors
        dev = "cpu" if gloo else "cuda"
        # every rank's own numbers first (the line reports the spread), then the max / sum
        mine_t = torch.tensor([elapsed, kernel_ms, float(len(mine)), float(queries)], dtype=torch.float64, device=dev)
        gathered = [torch.zeros_like(mine_t) for _ in range(world)]
        dist.all_gather(gathered, mine_t)
        per_rank = [[float(v) for v in g.cpu()] for g in gathered]
        t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(t[0]), float(t[1])
        q = torch.tensor([queries], dtype=torch.float64, device=dev)
        dist.all_reduce(q, op=dist.ReduceOp.SUM)
        queries = int(q[0])

    if rank == 0:
        npix_total = subset if subset else W * H
        samples = npix_total * spp * args.steps
        value = samples / elapsed / 1e6
        frame = fb.view(H, W, 3).cpu().numpy()
        if args.dump_frame:
            np.save(args.dump_frame, frame)
        out = {
            "metric": "Msamples/sec at 1920x1080x1024spp; per-channel RMSE vs CPU ref",
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 1), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "kernel_key": kernel_key,
            "config": {"workload": "%s: %dx%d, %d spp, depth %d, %s%s" % (
                cfg.name, W, H, spp, cfg.depth, cfg.note,
                ("; timed on %d hashed pixels at full spp" % subset) if subset else ""),
                       "order": args.order,
                       "sharding": (("one GPU renders every pixel" if not subset else
                                     "one GPU renders %d hashed pixels of the frame" % subset) if not use_dist else
                                    ("every pixel, spp split over ranks, per-pixel sums" if by_samples
                                     else "%dx%d tiles, %s deal over ranks" % (
                                         share.tile, share.tile, args.deal)) +
                                    (" + gloo reduce through host memory (rehearsal: %d ranks on %d GPU(s))" %
                                     (world, torch.cuda.device_count()) if gloo else " + RCCL reduce")) +
                                   (" (--force-dist: the N > 1 step at world size %d)" % world
                                    if args.force_dist else "")},
            "samples_per_step": npix_total * spp,
            **({"ranks": {"kernel_ms_per_launch": [round(r[1], 2) for r in per_rank],
                          "step_ms": [round(r[0] / args.steps * 1e3, 1) for r in per_rank],
                          "pixels": [int(r[2]) for r in per_rank],
                          "queries": [int(r[3]) for r in per_rank],
                          "kernel_imbalance_max_over_mean": round(
                              max(r[1] for r in per_rank) / max(1e-9, sum(r[1] for r in per_rank) / world), 4)}}
               if per_rank and world > 1 else {}),
            "queries_per_sample": round(queries / samples, 2),
        }
        opq = OPS_PER_QUERY.get(cfg.name)
        if opq:
            ops_per_launch = opq * queries / (args.steps * launches_per_step * world)
            achieved = ops_per_launch / (kernel_ms * 1e-3) / 1e12
            # the PMC passes ran this same command at N = 1 (config defaults: C5's subset, fast order)
            same = world == 1 and args.subset < 0 and not args.spp and args.order == "fast" and not use_dist
            ev, why = pmc_evidence(cfg.name, kernel_key) if same else (
                None, "counters are collected on the default one-GPU command only")
            out["roofline"] = {"bound": "valu", "achieved": round(achieved, 3), "peak": VALU_PEAK_TOPS,
                               "unit": "TFLOP/s", "frac": round(achieved / VALU_PEAK_TOPS, 4),
                               "traffic": round(ev["hbm_bytes_per_launch"]) if ev else None,
                               "kernel": render_kernels, "kernel_key": kernel_key,
                               "avg_launch_ms": round(kernel_ms, 2), "ops_per_query": opq}
            if not ev:
                out["roofline"]["traffic_note"] = why
            else:
                out["roofline"].update({
                    "traffic_unit": "HBM bytes/launch (PMC FETCH_SIZE x2 + WRITE_SIZE, %s)" %
                                    os.path.relpath(PMC_JSON % cfg.name, ROOT),
                    # issue rate against the wave64 VALU ceiling of one instruction per 2 SIMD-cycles
                    # (rocprof's VALUBusy sums in-flight cycles over waves and exceeds 1 here)
                    "valu_insts_per_simd_cycle": round(ev.get("valu_insts_per_simd_cycle", 0), 4),
                    "valu_issue_frac": round(ev.get("valu_insts_per_simd_cycle", 0) / 0.5, 4),
                    "salu_insts_per_simd_cycle": round(ev.get("salu_insts_per_simd_cycle", 0), 4),
                    "valu_busy_rocprof": round(ev["valu_busy"], 4),
                    "hbm_GBps": round(ev["hbm_GBps"], 2), "hbm_peak_GBps": 8000.0})
        if world > 1 and not args.no_cpu and not args.cpu_at_n:
            # the CPU baseline is the N = 1 line's (rank 0 at N = 1 only); an N-rank frame is the
            # one-GPU frame bit for bit (tiles) or within ~1e-7 (sample split), tests/test_bench_dist.py
            out["cpu_baseline"] = {"note": "reported on the N = 1 line (bench.py --gpus 1); --cpu-at-n adds it here"}
        elif not args.no_cpu:  # rank 0, after the timed region (the other ranks are done)
            try:
                npx = args.cpu_pixels or CPU_PIXELS.get(cfg.name, 512)
                pix, ref, cb = cpu_baseline(cfg, to_text(root, "/tmp/pt_bench_img"), spp, npx,
                                            cpu_threads(args.cpu_threads), queries / samples,
                                            mine if subset else None)
                gpu = frame.reshape(-1, 3)[pix]
                out["rmse_vs_cpu_ref"] = [float(v) for v in
                                          np.sqrt(np.mean((gpu.astype(np.float64) - ref) ** 2, axis=0))]
                out["cpu_baseline"] = cb
            except Exception as e:  # report, never hide
                out["cpu_baseline"] = {"error": str(e)[:300]}
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
