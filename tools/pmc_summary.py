"""Average per-dispatch PMC counters of one kernel from rocprofv3 csv passes.
    python tools/pmc_summary.py <dir> <kernel-substring>"""
import collections
import csv
import glob
import sys

d, kname = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
waves = None
for k in sorted(agg):
    v = sum(agg[k]) / len(agg[k])
    if k == "SQ_WAVES":
        waves = v
    print(f"{k:32s} {v:16.1f}  (n={len(agg[k])})" + (f"  per-wave {v / waves:12.1f}" if waves else ""))
