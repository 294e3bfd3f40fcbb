#!/usr/bin/env python3
"""Summarise a tools/profile.sh output dir: per-kernel average of every counter.
Usage: python tools/prof_summary.py gpurun_out/prof_<tag> [kernel-substring]"""
import collections, csv, glob, os, sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "k_rs147"
for f in sorted(glob.glob(os.path.join(d, "*", "run_kernel_stats.csv"))):
    for r in csv.DictReader(open(f)):
        print(f"trace  {r['Name'][:60]:60s} calls={r['Calls']} avg_ms={float(r['AverageNs'])/1e6:.4f}")
agg = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"pmc    {k:28s} n={len(v)} avg={sum(v)/len(v):.6g}")
