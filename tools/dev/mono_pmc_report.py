#!/usr/bin/env python3
"""Dev: per timed group of tools/dev/alloc_modes.py (2 warmup + 10 dispatches)
the average of every counter of every pass under gpurun_out/mmp/<line>/p*,
with the group's ms from the pass log.  python3 tools/dev/mono_pmc_report.py [line]"""
import collections
import csv
import glob
import os
import re
import sys

line = sys.argv[1] if len(sys.argv) > 1 else "m24to48"
base = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "gpurun_out", "mmp", line)
for d in sorted(glob.glob(os.path.join(base, "p*/"))):
    per = collections.OrderedDict()
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if "rs147" not in r["Kernel_Name"]:
            continue
        e = per.setdefault(int(r["Dispatch_Id"]), {})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ms = [float(m.group(1)) for m in re.finditer(r"\s([\d.]+) ms", open(d.rstrip("/") + ".log").read())]
    ids = sorted(per)
    cn = sorted(per[ids[0]])
    print(os.path.basename(d.rstrip("/")), "  ms  " + "  ".join(c.replace("TCC_", "").replace("_sum", "") for c in cn))
    for g in range(0, len(ids), 12):
        grp = ids[g + 2:g + 12]
        avg = [sum(per[i][c] for i in grp) / len(grp) for c in cn]
        print(f"  {ms[g // 12] if g // 12 < len(ms) else float('nan'):6.3f}  " + "  ".join(f"{v:.4g}" for v in avg))
