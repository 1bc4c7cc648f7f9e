"""Precompile the C3 megakernel for compiler-option / define variants into the
in-tree JIT cache (no GPU) and print each variant's register use and spills.
usage: python tools/ab/opt_prep.py "opts1" "opts2" ...   ("-" = none)
An argument starting with "D:" is a PT_DEVICE_DEFINES variant instead.
PT_PREP_CFG=C2 (etc.) compiles that benchmark config's scene instead of C3."""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CACHE = os.path.join(ROOT, "path-trace_amd", "_jit_cache")
CFG = os.environ.get("PT_PREP_CFG", "")
code = ("import sys; sys.path.insert(0, %r)\n"
        "import pathtrace as pt\nfrom pathtrace import scenes\n" % os.path.join(ROOT, "path-trace_amd"))
code += ("c = scenes.CONFIGS[%r]; c.device_scene().compile(c.depth)\n" % CFG if CFG else
         "pt.DeviceScene(scenes.scene_p1()).compile(8)\n")


def notes(path):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", path], capture_output=True,
                         text=True).stdout
    r, name = {}, None
    for line in out.splitlines():
        line = line.strip()
        if line.startswith(".name:"):
            name = line.split()[-1]
        for k in ("sgpr_spill_count", "vgpr_spill_count", "vgpr_count", "private_segment_fixed_size"):
            if line.startswith("." + k + ":") and name == "pt_render_fast":
                r[k] = int(line.split()[-1])
    return r


jobs = []
for v in sys.argv[1:] or ["-"]:
    env = dict(os.environ)
    env.pop("PT_JIT_OPTIONS", None)
    env.pop("PT_DEVICE_DEFINES", None)
    if v.startswith("D:"):
        env["PT_DEVICE_DEFINES"] = v[2:]
    elif v != "-":
        env["PT_JIT_OPTIONS"] = v
    tmp = tempfile.mkdtemp(prefix="ptjc")
    env["PT_JIT_CACHE"] = tmp
    jobs.append((v, tmp, subprocess.Popen([sys.executable, "-c", code], env=env, cwd=ROOT,
                                          stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)))
rc = 0
for v, tmp, p in jobs:
    err = p.communicate()[1].decode()
    if p.returncode:
        print("%-60s FAILED %s" % (v, err.strip().splitlines()[-1:] if err else ""))
        rc = 1
        continue
    for f in os.listdir(tmp):
        if f.endswith(".hsaco"):
            print("%-60s %s" % (v, notes(os.path.join(tmp, f))))
            shutil.copy(os.path.join(tmp, f), os.path.join(CACHE, f))
    shutil.rmtree(tmp)
sys.exit(rc)
