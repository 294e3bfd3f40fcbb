#!/usr/bin/env python3
"""Dev only: the fused kernel's in-kernel clock (MI355X_MICROARCH.md "DVFS
give-back" item 6) on the headline shape.

Run against the diagnostic build, which stamps s_memtime / s_memrealtime once
per wave around its whole run (csrc/xm_resample_fast.hip, XM_CLOCK_STAMPS):

    tools/dev/ab_part.sh lib_clk -DXM_CLOCK_STAMPS      (part 1, the headline kernels)
    XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/lib_clk/libxm_audio.so python tools/dev/clock_stamp.py

It runs >= --seconds of back-to-back launches (random synthetic PCM), clears
the stamps, runs --steps more and prints one JSON line: the aggregate clock
(sum of shader cycles / sum of 100-MHz ticks), the mean wave lifetime and
the wall time per launch of that build.  The stamped build's wall time is not
the product's (its stamps add waits); read the clock, not the length.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "xm-audio-utils_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import xmaudio as xm  # noqa: E402
from bench import RAMPS, SEED  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mixes", type=int, default=512)
    ap.add_argument("--frames", type=int, default=480000)
    ap.add_argument("--seconds", type=float, default=2.5)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--fill", choices=["synth", "zero"], default="synth")
    ap.add_argument("--label", default="")
    ap.add_argument("--span", type=int, default=0, help="also time N single launches: first start to last end")
    ap.add_argument("--waves", type=int, default=0,
                    help="per-wave records of N single launches: end-time quantiles, per-XCD and per-CU ends")
    args = ap.parse_args()
    fn = getattr(xm._lib, "xm_dev_clock", None)
    if fn is None:
        raise SystemExit("clock_stamp.py: the loaded library has no xm_dev_clock (build with -DXM_CLOCK_STAMPS)")
    fn.restype, fn.argtypes = C.c_int, [C.POINTER(C.c_ulonglong)]
    B, ntr, N = args.mixes, 8, args.frames
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device", device=0)
    m.set_tracks(RAMPS)
    F = m.out_frames(N)
    x = torch.empty((B, ntr, N, 2), dtype=torch.float32, device="cuda")
    y = torch.empty((B, F, 2), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    xm.synth(x.data_ptr(), "f32", SEED, 0, B * ntr, 2, N, 0, s.cuda_stream)
    if args.fill == "zero":
        x.zero_()
    m.set_stream(s.cuda_stream)
    torch.cuda.synchronize()

    def step():
        m.process_strided(x.data_ptr(), N * 2, ntr * N * 2, y.data_ptr(), F * 2, B, N)

    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.seconds:   # warm the clock: back-to-back launches
        for _ in range(20):
            step()
        torch.cuda.synchronize()
    buf = (C.c_ulonglong * 8)()
    fn(buf)   # clear (the first read also resets the min slots)
    fn(buf)
    if args.span:   # single launches: dispatch ramp and tail per launch
        ramp, tail, span = [], [], []
        for _ in range(args.span):
            step()
            torch.cuda.synchronize()
            fn(buf)
            ramp.append((buf[5] - buf[4]) / 100.0)       # us: last wave start - first wave start
            tail.append((buf[3] - buf[6]) / 100.0)       # us: last wave end - first wave end
            span.append((buf[3] - buf[4]) / 100.0)       # us: first start to last end
        print(json.dumps({"label": args.label, "mixes": B, "launches": args.span,
                          "span_us": sorted(span)[len(span) // 2], "dispatch_ramp_us": sorted(ramp)[len(ramp) // 2],
                          "end_spread_us": sorted(tail)[len(tail) // 2]}), flush=True)
    if args.waves:
        wave_records(args, fn, buf, step)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    fn(buf)
    cyc, ticks, waves = buf[0], buf[1], buf[2]
    print(json.dumps({"label": args.label, "lib": os.environ.get("XM_AUDIO_LIB", ""), "mixes": B, "frames": N,
                      "fill": args.fill, "steps": args.steps, "waves": waves,
                      "clock_ghz": round(cyc / ticks * 0.1, 4) if ticks else None,
                      "wave_us_mean": round(ticks / waves * 0.01, 2) if waves else None,
                      "wave_cycles_mean": round(cyc / waves) if waves else None,
                      "wall_ms_per_launch_stamped_build": round(wall * 1e3, 4)}), flush=True)


def wave_records(args, fn, buf, step):
    """Where and when each wave of single launches ran: is the end spread a
    property of places (XCDs, CUs: a static skew could absorb it) or of
    waves (random: only a dynamic tail could)?"""
    import numpy as np
    wv = getattr(xm._lib, "xm_dev_waves")
    wv.restype, wv.argtypes = C.c_int, [C.POINTER(C.c_ulonglong), C.c_int]
    n = xm.last_fast_split()
    recs = []
    for it in range(args.waves):
        step()
        torch.cuda.synchronize()
        fn(buf)
        nw = int(buf[2])
        out = (C.c_ulonglong * (4 * nw))()
        assert wv(out, nw) == 0
        a = np.frombuffer(out, dtype=np.uint64).reshape(nw, 4).astype(np.int64)
        t0 = a[:, 0].min()
        start, end = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0
        hw, xcc = a[:, 3] & 0xffffffff, (a[:, 3] >> 32) & 15
        cu = (hw >> 8) & 15
        se = (hw >> 13) & 7
        place = xcc * 256 + se * 16 + cu
        recs.append((start, end, xcc, place, a[:, 2]))
    q = lambda v: [round(float(x), 1) for x in np.quantile(v, [0, 0.1, 0.5, 0.9, 0.99, 1])]
    for it, (start, end, xcc, place, cyc) in enumerate(recs):
        life = end - start
        per_xcc = [round(float(end[xcc == x].mean()), 1) for x in range(8)]
        per_xcc_max = [round(float(end[xcc == x].max()), 1) for x in range(8)]
        clk = [round(float(cyc[xcc == x].sum() / (life[xcc == x].sum() * 1e3)), 3) for x in range(8)]
        places = np.unique(place)
        pe = np.array([end[place == p].mean() for p in places])
        print(json.dumps({"label": args.label, "launch": it, "waves": len(end), "split": n,
                          "end_q_0_10_50_90_99_100_us": q(end), "start_q_us": q(start), "life_q_us": q(life),
                          "end_mean_per_xcc_us": per_xcc, "end_max_per_xcc_us": per_xcc_max, "ghz_per_xcc": clk,
                          "cus": int(len(places)), "cu_mean_end_q_us": q(pe)}), flush=True)
    if len(recs) >= 2:   # is a place slow in every launch?
        pl = recs[0][3]
        places = np.unique(pl)
        m = np.array([[r[1][r[3] == p].mean() for p in places] for r in recs])
        c = np.corrcoef(m)
        xc = np.array([[r[1][r[2] == x].mean() for x in range(8)] for r in recs])
        print(json.dumps({"label": args.label, "cu_end_corr_between_launches": round(float(c[np.triu_indices(len(recs), 1)].mean()), 3),
                          "xcc_end_corr_between_launches": round(float(np.corrcoef(xc)[np.triu_indices(len(recs), 1)].mean()), 3)}),
              flush=True)


if __name__ == "__main__":
    main()
