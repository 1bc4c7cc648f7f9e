"""Compile a benchmark scene's megakernel and print its resource usage and
instruction mix (no GPU needed).  usage: python tools/inspect_kernel.py [C3|C1|...]"""
import collections
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "path-trace_amd"))
import build_ext  # noqa: E402

build_ext.build()
import pathtrace as pt  # noqa: E402
from pathtrace import scenes  # noqa: E402

cfg = scenes.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C3"]
ds = cfg.device_scene()
t = time.time()
key = ds.compile(cfg.depth)
print("compile %.1fs" % (time.time() - t))
cache = os.path.join(ROOT, "path-trace_amd", "_jit_cache")
hsaco = [os.path.join(cache, f) for f in os.listdir(cache) if f.endswith(".hsaco")]
hsaco.sort(key=os.path.getmtime)
f = os.path.join(cache, key + ".hsaco")
if not os.path.exists(f):
    f = hsaco[-1]
print("code object", os.path.basename(f))
notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", f], capture_output=True, text=True).stdout
for line in notes.splitlines():
    if any(k in line for k in (".name:", "vgpr_count", "sgpr_count", "spill", "private_segment_fixed_size",
                               "group_segment_fixed_size")):
        print(line.strip())
dis = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--mcpu=gfx950", f], capture_output=True,
                     text=True).stdout
sect = dis.split("<pt_render_fast>:")[1].split("<pt_render_strict>:")[0]
ops = collections.Counter()
for line in sect.splitlines():
    parts = line.split()
    if parts and not parts[0].endswith(">:"):
        ops[parts[0]] += 1
print("pt_render_fast instructions:", sum(ops.values()))
for op, n in ops.most_common(25):
    print("  %6d %s" % (n, op))
with open("/tmp/pt_render_fast.s", "w") as fo:
    fo.write(sect)
