"""Precompile, under PT_DEVICE_DEFINES variants, the modules that the core GPU
parity tests and the C3 probe load (the render goldens' zoo scenes and the C3
config), so a define can be checked for bits and timed on a box without JIT.
usage: precompile_defs.py "defines" ...   (no GPU)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 2 and sys.argv[1] == "--one":
    sys.path[:0] = [os.path.join(ROOT, "path-trace_amd"), os.path.join(ROOT, "tests")]
    import pathtrace as pt
    import zoo
    from pathtrace import scenes
    what = sys.argv[2]
    if what.startswith("C"):
        cfg = scenes.CONFIGS[what]
        cfg.device_scene().compile(cfg.depth)
    else:
        b, d = what.split(":")
        pt.DeviceScene(zoo.build(b)).compile(int(d))
    sys.exit(0)
sys.path[:0] = [os.path.join(ROOT, "path-trace_amd"), os.path.join(ROOT, "tests")]
import zoo  # noqa: E402
jobs = ["C3"] + ["%s:%d" % (b, d) for (_, b, _, _, _, d) in zoo.RENDER_CASES]
procs = []
for defs in sys.argv[1:]:
    for j in jobs:
        env = dict(os.environ, PT_DEVICE_DEFINES=defs)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--one", j], env=env, cwd=ROOT))
        if len(procs) >= 8:
            procs.pop(0).wait()
sys.exit(max([p.wait() for p in procs] + [0]))
