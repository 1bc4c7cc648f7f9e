"""Per-phase wave-cycle split of the C3 render kernel (profiling build).
Runs tools/perf_probe.py with PT_DEVICE_DEFINES=PT_PHASE_TIMING and
PT_PHASE_DUMP=1 and prints each phase's share of the sample total.
usage: phase_probe.py [spp] [extra defines]
       phase_probe.py cfg CONFIG W H SPP [extra defines]   (tools/probe_cfg.py instead)
       phase_probe.py bench CONFIG [extra defines]         (bench.py --config CONFIG, one step)"""
import os
import subprocess
import sys

here = os.path.dirname(os.path.abspath(__file__))
if len(sys.argv) > 1 and sys.argv[1] == "bench":
    cmd = [sys.executable, os.path.join(os.path.dirname(here), "bench.py"), "--config", sys.argv[2], "--no-cpu"]
    extra = sys.argv[3:]
elif len(sys.argv) > 1 and sys.argv[1] == "cfg":
    cmd = [sys.executable, os.path.join(here, "probe_cfg.py")] + sys.argv[2:6]
    extra = sys.argv[6:]
else:
    cmd = [sys.executable, os.path.join(here, "perf_probe.py"), sys.argv[1] if len(sys.argv) > 1 else "16"]
    extra = sys.argv[2:]
defs = " ".join(["PT_PHASE_TIMING"] + extra)
env = dict(os.environ, PT_DEVICE_DEFINES=defs, PT_PHASE_DUMP="1")
r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
print(r.stdout.strip().splitlines()[-1] if r.stdout.strip() else "no stdout", r.stderr[-1500:] if r.returncode else "")
names = ["generation", "gen-attempts", "fastpass", "slowpass", "groupsum", "burst", "sample"]
for line in r.stderr.splitlines():
    if line.startswith("pt_phases"):
        v = [int(x) for x in line.split()[1:]]
        tot = v[6] or 1  # wave-walked samples (none when lanes finish every sample)
        for n, x in zip(names, v):
            print("%-12s %6.1f%%" % (n, 100.0 * x / tot))
        print("%-12s %6.1f%%" % ("spine", 100.0 * (v[6] - v[5]) / tot))
        print("%-12s %6.1f%%" % ("burst-other", 100.0 * (v[5] - v[0] - sum(v[2:5])) / tot))
        if len(v) >= 16 and v[15]:
            print("%-12s %6.1f%%  (of the whole chunk loop: lane-parallel camera queries, lane samples, writes)" %
                  ("sample/loop", 100.0 * tot / v[15]))
        if len(v) >= 20 and v[15]:
            print("%-12s %6.1f%%  lane front end (camera queries, lane walks) of the chunk loop" % ("lanes", 100.0 * v[18] / v[15]))
            print("%-12s %6.1f%%  wave-walked samples of the chunk loop" % ("wave-walks", 100.0 * v[6] / v[15]))
            print("%-12s %6.1f%%  result writes of the chunk loop" % ("writes", 100.0 * v[19] / v[15]))
        if len(v) >= 18 and v[17]:
            print("%-12s %6.1f%%  (%.0f cycles per query)" % ("spine-query", 100.0 * v[16] / tot, v[16] / v[17]))
            if len(v) >= 21:
                print("%-12s %6.1f%%  of the spine's queries ran the lazy merge" % ("spine-merge", 100.0 * v[20] / v[17]))
        if len(v) >= 15:
            import json as _j
            last = _j.loads(r.stdout.strip().splitlines()[-1])
            smp = last.get("samples") or last.get("samples_per_step")
            ev = ["bursts", "iterations", "stageA_passes", "fast_passes", "slow_passes", "group_sums",
                  "fast_lanes", "slow_lanes"]
            for n, x in zip(ev, v[7:15]):
                print("%-14s %10.3f per sample" % (n, x / smp))
