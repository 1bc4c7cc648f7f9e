"""Summarise a rocprofv3 PC-sampling CSV on the GPU box (the raw file is too
large to bring back): the header and three rows as written, then the samples
grouped by code-object offset (+ instruction text), with the wave-issue and
stall-reason columns when the sampling method records them.
usage: pc_summary.py DIR_OR_CSV [top]"""
import collections
import csv
import glob
import os
import sys

src = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 400
files = [src] if os.path.isfile(src) else sorted(glob.glob(os.path.join(src, "**", "*pc_sampling*.csv"),
                                                        recursive=True))
if not files:
    print("no pc sampling csv under", src)
    for f in glob.glob(os.path.join(src, "**", "*"), recursive=True):
        print("  ", f, os.path.getsize(f) if os.path.isfile(f) else "")
    sys.exit(1)
for path in files:
    print("== %s (%.1f MB)" % (path, os.path.getsize(path) / 1e6))
    with open(path, newline="") as fh:
        rd = csv.reader(fh)
        hdr = next(rd)
        print("columns:", hdr)
        col = {h: i for i, h in enumerate(hdr)}
        first = []
        groups = collections.Counter()
        stall = collections.defaultdict(collections.Counter)
        issued = collections.Counter()
        text = {}
        total = 0
        off_keys = [h for h in hdr if "offset" in h.lower() or h.lower() in ("pc", "pc_offset")]
        ins_key = next((h for h in hdr if h.lower() == "instruction"), None)
        stall_key = next((h for h in hdr if "stall" in h.lower() and "reason" in h.lower()), None)
        iss_key = next((h for h in hdr if "issued" in h.lower()), None)
        for row in rd:
            if len(first) < 3:
                first.append(row)
            total += 1
            key = tuple(row[col[k]] for k in off_keys) if off_keys else (row[col[ins_key]] if ins_key else "?",)
            groups[key] += 1
            if ins_key:
                text[key] = row[col[ins_key]]
            if stall_key:
                stall[key][row[col[stall_key]]] += 1
            if iss_key and row[col[iss_key]] not in ("0", "false", "False", ""):
                issued[key] += 1
        for r in first:
            print("row:", r)
        print("samples:", total, "distinct keys:", len(groups), "key columns:", off_keys or [ins_key])
        if stall_key:
            allr = collections.Counter()
            for c in stall.values():
                allr.update(c)
            print("stall reasons overall:", allr.most_common())
        for key, n in groups.most_common(top):
            extra = ""
            if stall_key:
                extra = " | " + ", ".join("%s %d" % kv for kv in stall[key].most_common(4))
            if iss_key:
                extra += " | issued %d" % issued[key]
            print("%7d %6.3f%% %s %s%s" % (n, 100.0 * n / max(1, total), "/".join(key), text.get(key, ""), extra))
