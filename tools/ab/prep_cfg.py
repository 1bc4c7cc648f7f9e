"""Precompile benchmark configs' scene modules for A/B device headers (no GPU).
usage: python tools/ab/prep_cfg.py CONFIG[,CONFIG...] header|- ..."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
code = ("import sys; sys.path.insert(0, %r)\nfrom pathtrace import scenes\n"
        "c = scenes.CONFIGS[sys.argv[1]]\nc.device_scene().compile(c.depth)\n") % os.path.join(ROOT, "path-trace_amd")
procs = []
for cfg in sys.argv[1].split(","):
    for h in sys.argv[2:] or ["-"]:
        env = dict(os.environ)
        if h != "-":
            env["PT_DEVICE_HEADER"] = h
        procs.append(subprocess.Popen([sys.executable, "-c", code, cfg], env=env, cwd=ROOT, stderr=subprocess.DEVNULL))
sys.exit(max(p.wait() for p in procs))
