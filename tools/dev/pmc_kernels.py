#!/usr/bin/env python3
"""Dev: per-kernel PMC summary of one or more rocprofv3 --pmc passes over the
same command (each pass a directory holding run_counter_collection.csv).

Per kernel family (the name up to its first '<' or '('), per CALL of the
command (--calls: the number of timed calls the command made): launches and
every counter summed over its launches.  HBM bytes follow MI355X_MICROARCH.md
"HBM": FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half
the bytes of a wide streaming read, so fetch_GB = 2 x FETCH_SIZE x 1024.
Setup kernels (synthetic PCM, fills, copies) are listed apart.

    python3 tools/dev/pmc_kernels.py --calls 3 --out profiles/X.json gpurun_out/T/p1 gpurun_out/T/p2 ...
"""
import argparse
import collections
import csv
import json
import os


def family(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    for ch in "<(":
        i = name.find(ch)
        if i > 0:
            name = name[:i]
    return name.replace("void ", "").replace("(anonymous namespace)::", "").strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--calls", type=float, default=1.0)
    ap.add_argument("--out", default="")
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(set)
    for d in a.dirs:
        for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
            f = family(r["Kernel_Name"])
            cnt[f][r["Counter_Name"]] += float(r["Counter_Value"])
            launches[f].add((d, r["Dispatch_Id"]))
    out = {}
    for f, c in cnt.items():
        n = {k: v / a.calls for k, v in c.items()}
        # every pass ran the same command: launches per call from one pass
        per_pass = collections.Counter(d for d, _ in launches[f])
        n["launches"] = max(per_pass.values()) / a.calls
        if "FETCH_SIZE" in n:
            n["fetch_GB"] = n["FETCH_SIZE"] * 1024 * 2 / 1e9   # gfx950: x2 (MI355X_MICROARCH.md)
        if "WRITE_SIZE" in n:
            n["write_GB"] = n["WRITE_SIZE"] * 1024 / 1e9
        out[f] = n
    tot = {"fetch_GB": sum(v.get("fetch_GB", 0) for v in out.values()),
           "write_GB": sum(v.get("write_GB", 0) for v in out.values())}
    res = {"source": a.source, "fetch_correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 wide-read half count)",
           "per_call": out, "per_call_total": tot}
    js = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
