"""Static instruction mix between PT_MARK(n) markers of the C3 fast kernel.
usage: python tools/isa_sections.py [CONFIG]  (compiles with PT_DEVICE_DEFINES=PT_MARKERS)"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "path-trace_amd"))
os.environ["PT_DEVICE_DEFINES"] = (os.environ.get("PT_DEVICE_DEFINES", "") + " PT_MARKERS").strip()
import build_ext  # noqa: E402
build_ext.build()
import pathtrace as pt  # noqa: E402
from pathtrace import scenes  # noqa: E402

if len(sys.argv) > 1:  # a benchmark config (its occupancy and walk settings)
    cfg = scenes.CONFIGS[sys.argv[1]]
    ds = cfg.device_scene()
    ds.compile(cfg.depth)
else:
    ds = pt.DeviceScene(scenes.scene_p1())
    ds.compile(8)
cache = os.path.join(ROOT, "path-trace_amd", "_jit_cache")
f = max((os.path.join(cache, x) for x in os.listdir(cache) if x.endswith(".hsaco")), key=os.path.getmtime)
dis = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--mcpu=gfx950", f], capture_output=True,
                     text=True).stdout
sect = dis.split("<pt_render_fast>:")[1].split("<pt_render_strict>:")[0]
cur, counts = None, collections.defaultdict(collections.Counter)
for line in sect.splitlines():
    parts = line.split()
    if not parts or parts[0].endswith(">:"):
        continue
    m = re.match(r"s_nop (\d+)", line.strip())
    if parts[0] == "s_nop" and len(parts) > 1 and parts[1] in ("8", "9", "10", "11", "12", "13", "14", "15", "16", "17"):
        cur = int(parts[1])
        counts[cur]["__markers"] += 1
        continue
    if cur is not None:
        kind = "VALU" if parts[0].startswith("v_") else "SALU" if parts[0].startswith("s_") else "LDS" if parts[0].startswith("ds_") else "SCR" if parts[0].startswith("scratch_") else "MEM"
        counts[cur][kind] += 1
        counts[cur]["op:" + parts[0]] += 1
for k in sorted(counts):
    c = counts[k]
    print("after mark %d: VALU %d SALU %d LDS %d MEM %d SCRATCH %d (markers %d)" % (
        k, c["VALU"], c["SALU"], c["LDS"], c["MEM"], c["SCR"], c["__markers"]))
    top = sorted(((n, op[3:]) for op, n in c.items() if op.startswith("op:")), reverse=True)[:12]
    print("    " + ", ".join("%s %d" % (o, n) for n, o in top))
