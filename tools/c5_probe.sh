#!/bin/bash
# C5 cost split: the bench-like hashed subset and the glass-ball disk, plain and with phase timing.
mkdir -p gpurun_out/r3k
timeout -k 10 200 python3 tools/cfg_probe.py C5 65536 256 > gpurun_out/r3k/mixed.json 2>&1 || exit $?
timeout -k 10 200 python3 tools/cfg_probe.py C5 4096 256 disk:2460:1080:400 > gpurun_out/r3k/disk.json 2>&1 || exit $?
PT_DEVICE_DEFINES=PT_PHASE_TIMING PT_PHASE_DUMP=1 timeout -k 10 200 python3 tools/cfg_probe.py C5 4096 256 disk:2460:1080:400 > gpurun_out/r3k/disk_phase.txt 2>&1 || exit $?
PT_DEVICE_DEFINES=PT_PHASE_TIMING PT_PHASE_DUMP=1 timeout -k 10 200 python3 tools/cfg_probe.py C5 65536 256 > gpurun_out/r3k/mixed_phase.txt 2>&1 || exit $?
