bash tools/gpu_check.sh gpurun_out/check5 || exit $?
bash tools/ab_probe.sh 16 2 tools/ab/base.h tools/ab/urel.h || exit $?
for h in tools/ab/base.h tools/ab/urel.h; do
  PT_DEVICE_HEADER=$h timeout -k 10 300 python tools/probe_cfg.py C2 320 180 1 > gpurun_out/c2_$(basename $h).json 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/c2_$(basename $h).json').read().splitlines()[-1]); print('$h C2 320x180x1: %.3f Msamples/s slow_frac %.3f' % (d['Msamples_per_s'], d['slow_frac']))"
done
