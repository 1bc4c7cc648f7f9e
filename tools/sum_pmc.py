"""Sum rocprofv3 counter CSVs per directory for kernels matching a name.
usage: sum_pmc.py KERNEL_SUBSTR DIR..."""
import collections
import csv
import glob
import json
import sys

sub = sys.argv[1]
for d in sys.argv[2:]:
    agg = collections.defaultdict(float)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    log = glob.glob(d + ".log")
    ms = None
    if log:
        for line in open(log[0]):
            if line.startswith("{"):
                j = json.loads(line)
                ms, samples = j["kernel_ms"], j["samples"]
    print(d, "kernel_ms", ms)
    if ms:
        for k in sorted(agg):
            print("   %-22s %14.4g  per-sample %10.1f" % (k, agg[k], agg[k] / samples))
