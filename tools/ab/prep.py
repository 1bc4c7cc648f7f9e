"""Precompile the C3 megakernel for A/B variants into the in-tree cache (no GPU).
usage: python tools/ab/prep.py [header|-] ...   (PT_DEVICE_DEFINES passes through)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
code = ("import sys; sys.path.insert(0, %r)\n"
        "import pathtrace as pt\nfrom pathtrace import scenes\n"
        "scenes.CONFIGS[\"C3\"].device_scene().compile(8)\n") % os.path.join(ROOT, "path-trace_amd")
procs = []
for h in sys.argv[1:] or ["-"]:
    env = dict(os.environ)
    if h != "-":
        env["PT_DEVICE_HEADER"] = h
    procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, cwd=ROOT))
sys.exit(max(p.wait() for p in procs))
