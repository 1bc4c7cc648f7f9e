"""Precompile config megakernels for A/B variants into the in-tree cache (no GPU).
usage: precompile_variants.py CONFIG[:wg[:lane_walk]] "defines|-" ...   (all pairs, in parallel)"""
import dataclasses
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "--one":
    sys.path.insert(0, os.path.join(ROOT, "path-trace_amd"))
    from pathtrace import scenes
    name, *rest = sys.argv[2].split(":")
    cfg = scenes.CONFIGS[name]
    if len(rest) > 0 and rest[0]:
        cfg = dataclasses.replace(cfg, wg_per_cu=int(rest[0]))
    if len(rest) > 1 and rest[1]:
        cfg = dataclasses.replace(cfg, lane_walk=int(rest[1]))
    cfg.device_scene().compile(cfg.depth)
    sys.exit(0)
cfgs = [a for a in sys.argv[1:] if a.split(":")[0].startswith("C")]
defs = [a for a in sys.argv[1:] if a not in cfgs] or ["-"]
procs = []
for c in cfgs:
    for d in defs:
        env = dict(os.environ)
        if d != "-":
            env["PT_DEVICE_DEFINES"] = d
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--one", c], env=env, cwd=ROOT))
sys.exit(max(p.wait() for p in procs))
