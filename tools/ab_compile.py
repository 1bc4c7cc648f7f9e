"""Pre-compile the C3 kernel for A/B device headers into the in-tree cache.
usage: python tools/ab_compile.py [header ...]   ("-" = built-in library)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "path-trace_amd"))
import pathtrace as pt  # noqa: E402
from pathtrace import scenes  # noqa: E402

for h in sys.argv[1:] or ["-"]:
    if h == "-":
        os.environ.pop("PT_DEVICE_HEADER", None)
    else:
        os.environ["PT_DEVICE_HEADER"] = h
    pt.DeviceScene(scenes.scene_p1()).compile(8)
    print("compiled", h)
