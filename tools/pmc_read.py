#!/usr/bin/env python3
"""Summarise tools/pmc_mb.sh output: counters of the LAST dispatch of each kernel (name filter)."""
import collections
import csv
import glob
import sys

tag, filt = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
tot = collections.defaultdict(dict)
for f in sorted(glob.glob(f"gpurun_out/pmc_{tag}/*/run_counter_collection.csv")):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for x in csv.DictReader(open(f)):
        if filt not in x["Kernel_Name"]:
            continue
        key = x["Kernel_Name"][:60]
        per[(key, int(x["Dispatch_Id"]))][x["Counter_Name"]] += float(x["Counter_Value"])
    last = {}
    for (k, d), v in per.items():
        if k not in last or d > last[k][0]:
            last[k] = (d, v)
    for k, (d, v) in last.items():
        tot[k].update(v)
for k, v in tot.items():
    print(k)
    for c in sorted(v):
        print(f"   {c:28s} {v[c]:16.0f}")
    if "SQ_WAVE_CYCLES" in v:
        wc = v["SQ_WAVE_CYCLES"]
        print("   split: active %.2f wait_any %.2f wait_inst %.2f" % (
            v.get("SQ_ACTIVE_INST_ANY", 0) / wc, v.get("SQ_WAIT_ANY", 0) / wc, v.get("SQ_WAIT_INST_ANY", 0) / wc))
