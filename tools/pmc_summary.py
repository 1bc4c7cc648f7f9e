"""Summarise tools/pmc_bench.sh: the render kernels' VALU/SALU busy fractions
and HBM traffic under the bench command, per launch and per sample.  A render
is one pt_render_fast launch, or for lane-walk scenes a split launch
(pt_render_light over every chunk, then pt_render_fast over the chunks it
left): the counters of both kernels are summed, so "per launch" is per render.

VALUBusy follows rocprof's derived metric: SQ_ACTIVE_INST_VALU (quad-cycles
summed over waves) x 4 / SIMDs / GRBM_GUI_ACTIVE per XCD (GRBM is summed over
the 8 XCDs).  It counts one quad-cycle per VALU instruction, so it measures
VALU issue occupancy, not lane utilisation.  HBM bytes: FETCH_SIZE doubled
(gfx950 tallies 128-B requests at 64 B, MI355X_MICROARCH.md) + WRITE_SIZE,
both in KB.  usage: pmc_summary.py OUTDIR"""
import collections
import csv
import glob
import json
import sys

out = sys.argv[1]
SIMDS, XCDS = 1024, 8


RENDER_KERNELS = ("pt_render_fast", "pt_render_light")
seen = set()


def counters(name):
    agg = collections.defaultdict(float)
    for f in glob.glob("%s/%s/**/*counter_collection.csv" % (out, name), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].strip()
            if k in RENDER_KERNELS:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                seen.add(k)
    return agg


def bench_line(name):
    for line in open("%s/%s.log" % (out, name)):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit("no bench line in %s.log" % name)


busy, fetch, write = counters("busy"), counters("fetch"), counters("write")
stall, cache, tex = counters("stall"), counters("cache"), counters("tex")
b = bench_line("busy")
# the code object every pass ran (bench.py attaches this file only to a line that timed the same one)
keys = {bench_line(n).get("kernel_key") for n in ("busy", "fetch", "write", "stall", "cache", "tex")}
if len(keys) != 1 or None in keys:
    raise SystemExit("passes ran different or unknown code objects: %s" % sorted(map(str, keys)))
launches = b["steps"]  # one render launch per step at the bench config (one pass)
samples = b["value"] * 1e6 * b["ms_per_step"] * 1e-3 * b["steps"]
kernel_s = b["roofline"]["avg_launch_ms"] * 1e-3 if "roofline" in b else None
gui = busy["GRBM_GUI_ACTIVE"] / XCDS
res = {
    "kernel": " + ".join(k for k in reversed(RENDER_KERNELS) if k in seen), "kernel_key": b["kernel_key"], "workload": b["config"]["workload"],
    "bench_value": b["value"], "avg_launch_ms": b["roofline"]["avg_launch_ms"],
    "valu_busy": busy["SQ_ACTIVE_INST_VALU"] * 4 / SIMDS / gui,
    # > 1 here: SQ_ACTIVE_INST_VALU is summed over waves, and several waves'
    # VALU instructions are in flight on one SIMD at once, so also report the
    # issue rate itself (ceiling 0.5 per SIMD-cycle for wave64)
    "valu_insts_per_simd_cycle": busy["SQ_INSTS_VALU"] / SIMDS / gui,
    "salu_insts_per_simd_cycle": busy["SQ_INSTS_SALU"] / SIMDS / gui,
    "salu_busy": busy["SQ_ACTIVE_INST_SCA"] * 4 / SIMDS / gui,
    "valu_insts_per_sample": busy["SQ_INSTS_VALU"] / samples,
    "salu_insts_per_sample": busy["SQ_INSTS_SALU"] / samples,
    "wave_cycles_per_sample": 4 * busy["SQ_WAVE_CYCLES"] / samples,
    "fetch_bytes_per_launch": 2 * 1024 * fetch["FETCH_SIZE"] / launches,
    "write_bytes_per_launch": 1024 * write["WRITE_SIZE"] / launches,
}
if stall:
    wc = stall["SQ_WAVE_CYCLES"]
    # disjoint buckets of a wave's life (MI355X_MICROARCH.md, PMC slots)
    res["wave_cycle_split"] = {"waiting (s_waitcnt/barrier)": stall["SQ_WAIT_ANY"] / wc,
                               "issue-stalled": stall["SQ_WAIT_INST_ANY"] / wc,
                               "issuing": stall["SQ_ACTIVE_INST_ANY"] / wc}
    for k in ("SQ_INSTS_VMEM_RD", "SQ_INSTS_FLAT", "SQ_INSTS_LDS", "SQ_INSTS_SMEM"):
        res[k.lower()[9:] + "_insts_per_sample"] = stall[k] / samples
if cache:
    res["l2_hit_rate"] = cache["TCC_HIT_sum"] / max(1.0, cache["TCC_HIT_sum"] + cache["TCC_MISS_sum"])
if tex:
    tgui = tex["GRBM_GUI_ACTIVE"] / XCDS
    # one TA and one TD per CU (256): busy cycles over the kernel's active cycles
    res["ta_busy"] = tex["TA_TA_BUSY_sum"] / 256 / tgui
    res["td_busy"] = tex["TD_TD_BUSY_sum"] / 256 / tgui
    res["flat_read_wavefronts_per_sample"] = tex["TA_FLAT_READ_WAVEFRONTS_sum"] / samples
res["hbm_bytes_per_launch"] = res["fetch_bytes_per_launch"] + res["write_bytes_per_launch"]
res["hbm_bytes_per_sample"] = res["hbm_bytes_per_launch"] * launches / samples
if kernel_s:
    res["hbm_GBps"] = res["hbm_bytes_per_launch"] / kernel_s / 1e9
print(json.dumps(res, indent=1))
