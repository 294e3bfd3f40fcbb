#!/usr/bin/env python3
"""VALU accounting per config line: how far each
resampling line's kernel is from the separately-rounded tap minimum, and how
busy its VALU pipes are.

  python3 tools/valu_lines.py run <tag> [lines...]     # GPU box: one rocprofv3 --pmc pass per line
  python3 tools/valu_lines.py report <tag> [--out F]   # anywhere: per-line JSON from those passes

Per line, one `rocprofv3 --pmc` pass (SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU,
SQ_WAVE_CYCLES, SQ_WAVES, GRBM_GUI_ACTIVE, GRBM_COUNT) over
`tools/bench_configs.py <line> --steps 2 --warmup 1`, counters summed per
dispatch of the line's resampling kernel and averaged over its dispatches.

  tap_min    the wave-instructions the taps alone need: per output and track
             2 VALU per used tap for interleaved stereo (one v_pk_mul_f32 and
             one v_pk_add_f32 carry L and R), 1 for mono (two planes packed),
             over 64 lanes; used taps = the nonzero coefficients of the
             output's phase row, averaged over the L phases
  valu_x_min SQ_INSTS_VALU / tap_min (1.0 = only the taps)
  valu_busy  SQ_INSTS_VALU x 4 cycles / (SIMDs x kernel cycles), kernel
             cycles = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs): the
             fraction of the SIMDs' cycles a VALU instruction occupies if every
             wave64 instruction takes 4 (packed f32 ops take about two issue
             slots, DESIGN §5.4, so this understates a packed-heavy kernel)
  active     SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES: the share of each wave's
             life spent issuing VALU (both quad-cycle counts)
"""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COUNTERS = "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"

# line -> (in rate, out rate, channels, tracks, mixes, frames_in); the shapes of
# tools/bench_configs.py with its default --mixes 512
LINES = {
    "hl": (48000, 44100, 2, 8, 512, 480000),
    "up": (44100, 48000, 2, 8, 512, 441000),
    "s16rs": (48000, 44100, 2, 8, 512, 480000),
    "s16rs3": (48000, 44100, 2, 3, 512, 480000),
    "conv": (48000, 44100, 2, 8, 512, 480000),
    "conv2": (48000, 44100, 2, 2, 512, 480000),
    "planar2": (48000, 44100, 2, 2, 512, 480000),
    "c1s16": (44100, 48000, 1, 1, 8192, 441000),
    "c1odd": (44100, 48000, 1, 1, 8192, 441001),
    "mono1": (44100, 48000, 1, 1, 8192, 441000),
    "mono8": (48000, 44100, 1, 8, 1024, 480000),
    "r32to48": (32000, 48000, 2, 8, 512, 320000),
    "r16to48": (16000, 48000, 2, 8, 512, 160000),
    "r24to48": (24000, 48000, 2, 8, 512, 240000),
    "r22to48": (22050, 48000, 2, 8, 512, 220500),
    "r44to96": (44100, 96000, 2, 8, 512, 441000),
    "r96to44": (96000, 44100, 2, 8, 512, 960000),
    "s16r24to48": (24000, 48000, 2, 8, 512, 240000),
    "s16r16to48": (16000, 48000, 2, 8, 512, 160000),
    "s16r22to48": (22050, 48000, 2, 8, 512, 220500),
}
RESAMPLE_KERNELS = ("k_rs147_mix", "k_rs_d2_mix", "k_resample_mix_generic")


def run(tag, lines):
    out = os.path.join(ROOT, "gpurun_out", tag)
    os.makedirs(out, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    for ln in lines:
        cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", *COUNTERS.split(), "-d",
               os.path.join(out, ln), "-o", "run", "--output-format", "csv", "--", sys.executable,
               os.path.join(ROOT, "tools", "bench_configs.py"), ln, "--steps", "2", "--warmup", "1", "--no-check",
               "--no-box"]
        with open(os.path.join(out, ln + ".log"), "w") as fh:
            rc = subprocess.run(cmd, stdout=fh, stderr=subprocess.STDOUT, env=env, cwd=ROOT).returncode
        print(ln, "rc", rc, flush=True)
        if rc:
            sys.exit(rc)


def family(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    for ch in "<(":
        i = name.find(ch)
        if i > 0:
            name = name[:i]
    return name.strip()


def tap_min(line):
    sys.path.insert(0, os.path.join(ROOT, "xm-audio-utils_amd"))
    import numpy as np
    import xmaudio as xm
    fi, fo, C, ntr, B, N = LINES[line]
    d, H = xm.design(fi, fo)
    nnz = float(np.mean(np.count_nonzero(H, axis=1)))
    F = xm.out_frames(fi, fo, N)
    per_out = 2.0 if C == 2 else 1.0
    return F * ntr * B * per_out * nnz / 64.0, nnz


def find_csv(d):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                return os.path.join(root, f)
    return None


def report(tag, out_file=None, simds=1024):
    base = os.path.join(ROOT, "gpurun_out", tag)
    res = {"source": f"tools/valu_lines.py run {tag}: one rocprofv3 --pmc pass per line "
                     f"(bench_configs <line> --steps 2 --warmup 1)", "counters": COUNTERS, "lines": {}}
    for line in LINES:
        f = find_csv(os.path.join(base, line))
        if not f:
            continue
        per = {}
        for r in csv.DictReader(open(f)):
            fam = family(r["Kernel_Name"])
            if fam not in RESAMPLE_KERNELS:
                continue
            key = r["Dispatch_Id"]
            per.setdefault(key, {"kernel": fam})
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        if not per:
            continue
        n = len(per)
        avg = {c: sum(v.get(c, 0.0) for v in per.values()) / n for c in COUNTERS.split()}
        tm, nnz = tap_min(line)
        cyc = avg["GRBM_GUI_ACTIVE"] / 8.0
        res["lines"][line] = {
            "kernel": sorted({v["kernel"] for v in per.values()}), "dispatches": n,
            "valu_insts": avg["SQ_INSTS_VALU"], "tap_min": round(tm), "used_taps": round(nnz, 3),
            "valu_x_min": round(avg["SQ_INSTS_VALU"] / tm, 4),
            "valu_busy": round(avg["SQ_INSTS_VALU"] * 4.0 / (simds * cyc), 4) if cyc else None,
            "active": round(avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"], 4) if avg["SQ_WAVE_CYCLES"] else None,
            "kernel_cycles": round(cyc), "waves": avg["SQ_WAVES"],
        }
    js = json.dumps(res, indent=1)
    if out_file:
        with open(out_file, "w") as fh:
            fh.write(js + "\n")
    print(js)


if __name__ == "__main__":
    if len(sys.argv) >= 3 and sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3:] or list(LINES))
    elif len(sys.argv) >= 3 and sys.argv[1] == "report":
        report(sys.argv[2], sys.argv[4] if len(sys.argv) > 4 and sys.argv[3] == "--out" else None)
    else:
        print(__doc__)
        sys.exit(2)
