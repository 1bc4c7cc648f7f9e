"""Static ISA statistics of the C3 fast kernel for device-library variants
(A/B triage on the CPU before a GPU run).
usage: python tools/ab/isa_stat.py [header|-] ...  (PT_DEVICE_DEFINES passes through)"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
code = ("import sys; sys.path.insert(0, %r)\n"
        "import pathtrace as pt\nfrom pathtrace import scenes\n"
        "print(scenes.CONFIGS[\"C3\"].device_scene().compile(8))\n") % os.path.join(ROOT, "path-trace_amd")
for h in sys.argv[1:] or ["-"]:
    env = dict(os.environ)
    if h != "-":
        env["PT_DEVICE_HEADER"] = h
    key = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True,
                         text=True).stdout.strip().splitlines()[-1]
    f = os.path.join(ROOT, "path-trace_amd", "_jit_cache", key + ".hsaco")
    notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", f], capture_output=True,
                           text=True).stdout
    meta = {}
    cur = None
    for line in notes.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            cur = m.group(1)
        m = re.match(r"\s+\.(sgpr_spill_count|vgpr_spill_count|vgpr_count|private_segment_fixed_size):\s+(\d+)", line)
        if m and cur == "pt_render_fast":
            meta[m.group(1)] = int(m.group(2))
    dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", f], capture_output=True, text=True).stdout
    fast = dis.split("<pt_render_fast>:")[1].split("<pt_render_strict>:")[0]
    lines = [l.split("//")[0].strip() for l in fast.splitlines()]
    ops = [l.split()[0] for l in lines if l and not l.endswith(":")]
    c = collections.Counter(ops)
    addc = [i for i, l in enumerate(lines) if l.startswith("v_addc_co_u32_e64")]
    lm = collections.Counter()
    if addc:
        a, b = addc[0] - 120, addc[len(addc) // 2 - 1] + 60  # the first lane-major round instance
        lm = collections.Counter(l.split()[0] for l in lines[a:b] if l)
    scr = sum(n for o, n in c.items() if o.startswith("scratch_"))
    lscr = sum(n for o, n in lm.items() if o.startswith("scratch_"))
    print("%-26s key %s  insts %d  readlane %d writelane %d scratch %d nop %d | %s | LM round: %d insts, "
          "readlane %d, scratch %d, VALU %d" % (
              h, key, len(ops), c["v_readlane_b32"], c["v_writelane_b32"], scr, c["s_nop"], meta,
              sum(lm.values()), lm["v_readlane_b32"], lscr, sum(n for o, n in lm.items() if o.startswith("v_"))))
