#!/usr/bin/env python3
"""Dev: per line of tools/dev/write_survey.sh, per kernel family and call
(3 calls per pass): WRITE_SIZE in GB and the L2's 64-B write requests x 64 B.
    python3 tools/dev/write_survey_report.py <tag>"""
import collections
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
base = os.path.join(ROOT, "gpurun_out", sys.argv[1])
for d in sorted(glob.glob(os.path.join(base, "*/"))):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
        for ch in "<(":
            if ch in k:
                k = k[:k.index(ch)]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
    out = []
    for k, c in tot.items():
        if "synth" in k or "fill" in k:
            continue
        out.append(f"{k}: WRITE_SIZE {c['WRITE_SIZE'] * 1024 / 3 / 1e9:.3f} GB, 64-B reqs x 64 "
                   f"{c['TCC_EA0_WRREQ_64B_sum'] * 64 / 3 / 1e9:.3f} GB (all reqs {c['TCC_EA0_WRREQ_sum'] / 3:.4g})")
    print(os.path.basename(d.rstrip("/")), "; ".join(out))
