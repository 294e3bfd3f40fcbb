#!/usr/bin/env python3
"""Turn one tools/gpu_check.sh output dir into the committed profile record.

    python tools/profile_traffic.py gpurun_out/<tag> profiles/<round>_<tag>

Writes <dst>_kernel_stats.csv (the rocprofv3 --kernel-trace --stats summary,
verbatim) and <dst>_traffic.json: HBM bytes per launch of the headline kernel
from the separate FETCH_SIZE and WRITE_SIZE passes, corrected as
/opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes:
  * both counters are in KiB (x 1024);
  * on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced
    streaming read (16 B/lane global_load and buffer_load ... lds alike), so
    it is doubled; WRITE_SIZE is exact for streaming stores.
bench.py reads the newest profiles/*traffic*.json taken on its own kernel
sources (kernel_src_sha256, written by tools/gpu_check.sh) for roofline.traffic.
"""
import csv
import json
import os
import shutil
import sys

KERNEL = "k_rs147_mix"
# bench.py's headline launch: 512 mixes x 8 tracks x 480000 frames x 2 ch fp32
# in, 512 x 441000 x 2 fp32 out
ALG_READ = 512 * 8 * 480000 * 2 * 4
ALG_WRITE = 512 * 441000 * 2 * 4


def per_launch(path, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter]
    if not vals:
        raise SystemExit(f"no {counter} rows for {KERNEL} in {path}")
    return sum(vals) / len(vals), len(vals)


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), dst + "_kernel_stats.csv")
    avg_ns = None
    for r in csv.DictReader(open(dst + "_kernel_stats.csv")):
        if KERNEL in r["Name"]:
            avg_ns = float(r["AverageNs"])
    fetch_kib, nf = per_launch(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write_kib, nw = per_launch(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    rd = 2.0 * fetch_kib * 1024.0
    wr = write_kib * 1024.0
    rec = {
        "kernel": KERNEL,
        "source": src,
        "launches": {"FETCH_SIZE": nf, "WRITE_SIZE": nw},
        "fetch_size_kib_raw": fetch_kib,
        "write_size_kib_raw": write_kib,
        "correction": "bytes = KiB x 1024; FETCH_SIZE x 2 (gfx950 wide streaming reads, MI355X_MICROARCH.md HBM)",
        "hbm_read_bytes_per_launch": rd,
        "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr,
        "alg_bytes_per_launch": ALG_READ + ALG_WRITE,
        "traffic_over_alg": (rd + wr) / (ALG_READ + ALG_WRITE),
        "rocprof_avg_ms": avg_ns / 1e6 if avg_ns else None,
        "rocprof_achieved_GBps": (ALG_READ + ALG_WRITE) / avg_ns if avg_ns else None,
    }
    # the kernel sources the pass ran (bench.py reports this record only for them)
    sha = os.path.join(src, "kernel_src.sha256")
    if os.path.exists(sha):
        rec["kernel_src_sha256"] = open(sha).read().strip()
    with open(dst + "_traffic.json", "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec, indent=1))
    trace_bench(src, dst)
    sq_counters(src, dst)


def trace_bench(src, dst):
    """The bench line printed by the profiled run itself (trace.log) next to
    the per-dispatch kernel durations of that same run: the timed launches are
    the last `steps` dispatches of the headline kernel."""
    line = None
    log = os.path.join(src, "trace.log")
    if os.path.exists(log):
        for ln in open(log):
            if ln.startswith("{"):
                line = json.loads(ln)
    tr = os.path.join(src, "trace", "run_kernel_trace.csv")
    if line is None or not os.path.exists(tr):
        return
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(tr))
            if KERNEL in r["Kernel_Name"]]
    timed = durs[-line["steps"]:]
    avg_ms = sum(timed) / len(timed) / 1e6
    alg = line["roofline"]["alg_bytes_per_launch"]
    rec = {"command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps 20 --warmup 5",
           "bench_line": line,
           "rocprof_timed_launches": len(timed),
           "rocprof_avg_launch_ms": avg_ms,
           "rocprof_frac": alg / (avg_ms * 1e-3) / 8.0e12,
           "event_avg_launch_ms": line["roofline"]["avg_launch_ms"],
           "event_frac": line["roofline"]["frac"],
           "rocprof_over_event": avg_ms / line["roofline"]["avg_launch_ms"]}
    with open(dst + "_trace_bench.json", "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps({k: v for k, v in rec.items() if k != "bench_line"}, indent=1))


def sq_counters(src, dst):
    """SQ instruction counts per launch of the headline kernel (pmc_sq pass)
    against the tap minimum: 512 mixes x 8 tracks x 441000 outputs x 44
    packed VALU per output pair's half (22 taps x (mul + add) per channel
    pair) / 64 lanes."""
    f = os.path.join(src, "pmc_sq", "run_counter_collection.csv")
    if not os.path.exists(f):
        return
    per = {}
    for r in csv.DictReader(open(f)):
        if KERNEL not in r["Kernel_Name"]:
            continue
        per.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
        per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    rec = {c: sum(v.values()) / len(v) for c, v in per.items()}
    tap_min = 512 * 8 * 441000 * 44 / 64
    rec["valu_tap_minimum"] = tap_min
    if "SQ_INSTS_VALU" in rec:
        rec["valu_over_tap_minimum"] = rec["SQ_INSTS_VALU"] / tap_min
    with open(dst + "_sq.json", "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
