"""Run tools/perf_probe.py once per device-code variant (PT_DEVICE_DEFINES)
and print one line each.  usage: exp_variants.py spp "" "PT_LEAF_STUB=1" ..."""
import json
import os
import subprocess
import sys

here = os.path.dirname(os.path.abspath(__file__))
spp = sys.argv[1]
for v in sys.argv[2:]:
    env = dict(os.environ, PT_DEVICE_DEFINES=v)
    r = subprocess.run([sys.executable, os.path.join(here, "perf_probe.py"), spp], env=env, capture_output=True,
                       text=True, timeout=600)
    line = (r.stdout.strip().splitlines() or ["{}"])[-1]
    try:
        d = json.loads(line)
        print("%-30s %8.2f Msamples/s  kernel %8.1f ms" % (v or "baseline", d["Msamples_per_s"], d["kernel_ms"]),
              flush=True)
    except Exception:
        print(v, "FAILED", r.returncode, r.stderr[-2000:], flush=True)
