#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Runs ONLY in the build container (needs scipy 1.15.3).  The reference
snapshot has no code and no fixtures (/root/reference/README.md:1), so the
expected outputs come from the third-party algorithm BASELINE.json:5 names,
executed here:
  scipy.signal.firwin + resample_poly   (resampler tables and outputs)
  scipy.signal.sosfilt                  (biquad cascade)
  scipy.signal.upfirdn                  (FIR)
The mix / gain outputs have no scipy counterpart: they come from the numpy
statement of the contract in include/xm_audio_common.h (oracle/np_oracle.py)
applied to scipy-resampled tracks.  Inputs come from the deterministic
splitmix64 generator (np_oracle.gen_*), whose first samples are stored too so
the C / HIP generators are pinned to the same bits.

Usage: python tools/gen_golden.py           (rewrites tests/golden/*.npz + MANIFEST.json)
       python tools/gen_golden.py --fused   (only resample_fused.npz and its entry)
"""
from __future__ import annotations

import hashlib
import json
import math
import os
import sys

import numpy as np
import scipy
from scipy import signal

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import np_oracle as O  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
SEED = O.SEED

RATE_PAIRS = [
    (48000, 44100), (44100, 48000), (16000, 48000), (48000, 16000),
    (22050, 44100), (44100, 22050), (32000, 48000), (48000, 32000),
    (44100, 16000), (16000, 44100), (8000, 48000), (48000, 8000),
    (11025, 44100), (44100, 11025), (96000, 44100), (44100, 96000),
    (48000, 96000), (96000, 48000), (24000, 16000), (44100, 32000),
]


def scipy_table(L: int, M: int):
    mx = max(L, M)
    h = signal.firwin(2 * 10 * mx + 1, 1.0 / mx, window=("kaiser", 5.0)).astype(np.float32)
    h *= np.float32(L)
    return O.table_from_prototype(h, L, M)


def bits_equal(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and np.array_equal(
        a.view(np.uint8), b.view(np.uint8))


FUSED_CASES = [
    # (name, fi, fo, N, C, clip, fmt) -- round 6: scipy outputs at
    # every ratio a fused kernel serves that had only tables before, with lengths
    # around the super-period edges (SPI input frames per super-period, below) and
    # odd N.  fmt "s16": s16 input, s16 output = clip(rint(resample_poly(f32(x)))).
    # 320/147 (SPI 147): 44.1k -> 96k, 22.05k -> 48k
    ("u2_44to96_st_146", 44100, 96000, 146, 2, 300, "f32"),
    ("u2_44to96_st_147", 44100, 96000, 147, 2, 301, "f32"),
    ("u2_44to96_st_148", 44100, 96000, 148, 2, 302, "f32"),
    ("u2_44to96_st_1471", 44100, 96000, 1471, 2, 303, "f32"),
    ("u2_22to48_st_295", 22050, 48000, 295, 2, 304, "f32"),
    ("u2_22to48_mono_147", 22050, 48000, 147, 1, 305, "f32"),
    ("u2_22to48_mono_1177", 22050, 48000, 1177, 1, 306, "f32"),
    # 2/1 (SPI 160): 24k -> 48k, 22.05k -> 44.1k
    ("x2_24to48_st_159", 24000, 48000, 159, 2, 310, "f32"),
    ("x2_24to48_st_160", 24000, 48000, 160, 2, 311, "f32"),
    ("x2_24to48_st_161", 24000, 48000, 161, 2, 312, "f32"),
    ("x2_24to48_st_1601", 24000, 48000, 1601, 2, 313, "f32"),
    ("x2_22to44_mono_160", 22050, 44100, 160, 1, 314, "f32"),
    ("x2_22to44_mono_1283", 22050, 44100, 1283, 1, 315, "f32"),
    # 3/1 (SPI 160): 16k -> 48k
    ("x3_16to48_st_161", 16000, 48000, 161, 2, 320, "f32"),
    ("x3_16to48_st_960", 16000, 48000, 960, 2, 321, "f32"),
    ("x3_16to48_mono_159", 16000, 48000, 159, 1, 322, "f32"),
    ("x3_16to48_mono_1121", 16000, 48000, 1121, 1, 323, "f32"),
    # 1/2 (SPI 160): 96k -> 48k
    ("d2_96to48_st_160", 96000, 48000, 160, 2, 330, "f32"),
    ("d2_96to48_st_161", 96000, 48000, 161, 2, 331, "f32"),
    ("d2_96to48_st_2883", 96000, 48000, 2883, 2, 332, "f32"),
    ("d2_96to48_mono_319", 96000, 48000, 319, 1, 333, "f32"),
    ("d2_96to48_mono_3201", 96000, 48000, 3201, 1, 334, "f32"),
    # 2/3 (SPI 159): 48k -> 32k
    ("t23_48to32_st_158", 48000, 32000, 158, 2, 340, "f32"),
    ("t23_48to32_st_159", 48000, 32000, 159, 2, 341, "f32"),
    ("t23_48to32_st_160", 48000, 32000, 160, 2, 342, "f32"),
    ("t23_48to32_st_2545", 48000, 32000, 2545, 2, 343, "f32"),
    ("t23_48to32_mono_1591", 48000, 32000, 1591, 1, 344, "f32"),
    # 3/2 (SPI 160): 32k -> 48k stereo
    ("t32_32to48_st_160", 32000, 48000, 160, 2, 350, "f32"),
    ("t32_32to48_st_1763", 32000, 48000, 1763, 2, 351, "f32"),
    # 147/320 (SPI 320): 96k -> 44.1k, mono and stereo
    ("d2x_96to44_mono_319", 96000, 44100, 319, 1, 360, "f32"),
    ("d2x_96to44_mono_320", 96000, 44100, 320, 1, 361, "f32"),
    ("d2x_96to44_mono_3201", 96000, 44100, 3201, 1, 362, "f32"),
    ("d2x_96to44_st_321", 96000, 44100, 321, 2, 363, "f32"),
    ("d2x_96to44_st_2561", 96000, 44100, 2561, 2, 364, "f32"),
    # 160/147 and 147/160 mono s16 at odd N (config 1's form, BASELINE.json:7)
    ("s16_44to48_mono_147", 44100, 48000, 147, 1, 370, "s16"),
    ("s16_44to48_mono_1471", 44100, 48000, 1471, 1, 371, "s16"),
    ("s16_44to48_mono_4411", 44100, 48000, 4411, 1, 372, "s16"),
    ("s16_44to48_mono_14701", 44100, 48000, 14701, 1, 373, "s16"),
    ("s16_48to44_mono_161", 48000, 44100, 161, 1, 374, "s16"),
    ("s16_48to44_mono_3201", 48000, 44100, 3201, 1, 375, "s16"),
    ("s16_44to48_st_1471", 44100, 48000, 1471, 2, 376, "s16"),
    # stereo s16 at 2/1, 3/1 and 320/147 (round 6: fused IO kernels)
    ("s16_24to48_st_1601", 24000, 48000, 1601, 2, 377, "s16"),
    ("s16_16to48_st_963", 16000, 48000, 963, 2, 378, "s16"),
    ("s16_22to48_st_1471", 22050, 48000, 1471, 2, 379, "s16"),
    ("s16_44to96_st_295", 44100, 96000, 295, 2, 380, "s16"),
]


def fused_vectors():
    """resample_fused.npz: scipy resample_poly outputs at the fused kernels' ratios."""
    out = {}
    for name, fi, fo, N, C, clip, fmt in FUSED_CASES:
        L, M = O.reduce_ratio(fi, fo)
        H, T, rm, _, _ = scipy_table(L, M)
        if fmt == "f32":
            x = O.gen_f32(SEED, clip, C, N)
            y = signal.resample_poly(x, L, M, axis=0).astype(np.float32, copy=False)
            assert y.dtype == np.float32
            assert bits_equal(O.resample_f32(x, H, L, M, rm), y), name
        else:
            x = O.gen_s16(SEED, clip, C, N)
            yf = signal.resample_poly(x.astype(np.float32), L, M, axis=0)
            assert yf.dtype == np.float32
            y = np.clip(np.rint(yf), -32768, 32767).astype(np.int16)
            assert bits_equal(O.resample_s16(x, H, L, M, rm), y), name
        out[f"{name}__y"] = y
        out[f"{name}__meta"] = np.array([fi, fo, N, C, clip, 16 if fmt == "s16" else 32], np.int64)
    return out


def write_manifest_entry(manifest, f):
    with open(os.path.join(OUT, f), "rb") as fh:
        data = fh.read()
    manifest["files"][f] = {"sha256": hashlib.sha256(data).hexdigest(), "bytes": len(data)}


def main_fused():
    """--fused: (re)write only resample_fused.npz and its MANIFEST entry."""
    np.savez_compressed(os.path.join(OUT, "resample_fused.npz"), **fused_vectors())
    path = os.path.join(OUT, "MANIFEST.json")
    with open(path) as fh:
        manifest = json.load(fh)
    write_manifest_entry(manifest, "resample_fused.npz")
    with open(path, "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)
    print(json.dumps(manifest["files"]["resample_fused.npz"]))


def main():
    os.makedirs(OUT, exist_ok=True)
    manifest = {"generator": "tools/gen_golden.py", "scipy": scipy.__version__,
                "numpy": np.__version__, "files": {}}

    # ---------------- resampler tables -------------------------------------
    tables = {}
    for fi, fo in RATE_PAIRS:
        L, M = O.reduce_ratio(fi, fo)
        key = f"{L}_{M}"
        if f"H_{key}" in tables:
            continue
        H, T, rm, half, pre = scipy_table(L, M)
        tables[f"H_{key}"] = H
        tables[f"meta_{key}"] = np.array([L, M, T, rm, half, pre], np.int64)
    np.savez_compressed(os.path.join(OUT, "tables.npz"), **tables)

    # ---------------- generator pin ----------------------------------------
    gen = {
        "f32_clip0_st": O.gen_f32(SEED, 0, 2, 512),
        "f32_clip77_mono": O.gen_f32(SEED, 77, 1, 512),
        "s16_clip5_st": O.gen_s16(SEED, 5, 2, 512),
        "f32_clip4095_st_tail": O.gen_f32(SEED, 4095, 2, 480000)[-256:],
    }
    np.savez_compressed(os.path.join(OUT, "generator.npz"), **gen)

    # ---------------- resample_poly vectors --------------------------------
    rs = {}
    cases = []
    # (name, L, M, frames, channels, clip)  generator inputs
    for name, fi, fo, N, C, clip in [
        ("h48to44_st_9600", 48000, 44100, 9600, 2, 1),
        ("h48to44_mono_4800", 48000, 44100, 4800, 1, 2),
        ("h44to48_st_8820", 44100, 48000, 8820, 2, 3),
        ("h44to48_mono_1000", 44100, 48000, 1000, 1, 4),
        ("r16to48_st_1600", 16000, 48000, 1600, 2, 5),
        ("r48to16_st_4800", 48000, 16000, 4800, 2, 6),
        ("r32to48_mono_3200", 32000, 48000, 3200, 1, 7),
        ("r44to16_st_4410", 44100, 16000, 4410, 2, 8),
        ("r96to44_st_4800", 96000, 44100, 4800, 2, 9),
        # ragged / tiny lengths around the halo and the super-period
        ("h48to44_st_1", 48000, 44100, 1, 2, 10),
        ("h48to44_st_7", 48000, 44100, 7, 2, 11),
        ("h48to44_st_22", 48000, 44100, 22, 2, 12),
        ("h48to44_st_23", 48000, 44100, 23, 2, 13),
        ("h48to44_st_159", 48000, 44100, 159, 2, 14),
        ("h48to44_st_160", 48000, 44100, 160, 2, 15),
        ("h48to44_st_161", 48000, 44100, 161, 2, 16),
        ("h48to44_st_3333", 48000, 44100, 3333, 2, 17),
        ("h44to48_st_147", 44100, 48000, 147, 2, 18),
        ("h44to48_st_149", 44100, 48000, 149, 2, 19),
    ]:
        x = O.gen_f32(SEED, clip, C, N)
        L, M = O.reduce_ratio(fi, fo)
        y = signal.resample_poly(x, L, M, axis=0).astype(np.float32, copy=False)
        assert y.dtype == np.float32
        H, T, rm, _, _ = scipy_table(L, M)
        assert bits_equal(O.resample_f32(x, H, L, M, rm), y), name
        rs[f"{name}__y"] = y
        rs[f"{name}__meta"] = np.array([fi, fo, N, C, clip], np.int64)
        cases.append(name)
    # explicit-input edge cases: silence, full scale, denormals, impulse
    N = 800
    special = {
        "silence": np.zeros((N, 2), np.float32),
        "fullscale": np.where(np.arange(N * 2).reshape(N, 2) % 3 == 0, 1.0, -1.0).astype(np.float32),
        "denormal": (O.gen_f32(SEED, 20, 2, N) * np.float32(2.0 ** -130)).astype(np.float32),
        "impulse": np.zeros((N, 2), np.float32),
    }
    special["impulse"][400, 0] = 1.0
    special["impulse"][401, 1] = -1.0
    for nm, x in special.items():
        y = signal.resample_poly(x, 147, 160, axis=0).astype(np.float32, copy=False)
        rs[f"special_{nm}__x"] = x
        rs[f"special_{nm}__y"] = y
    np.savez_compressed(os.path.join(OUT, "resample.npz"), **rs)

    # ---------------- config 1: mono 44.1k -> 48k s16, 10 s -----------------
    x16 = O.gen_s16(SEED, 0, 1, 441000)
    yf = signal.resample_poly(x16.astype(np.float32), 160, 147, axis=0)
    assert yf.dtype == np.float32
    y16 = np.clip(np.rint(yf), -32768, 32767).astype(np.int16)
    cfg1 = {"y_head": y16[:4096], "y_tail": y16[-4096:],
            "meta": np.array([44100, 48000, 441000, 1, 0], np.int64)}
    np.savez_compressed(os.path.join(OUT, "config1.npz"), **cfg1)
    manifest["config1_sha256"] = hashlib.sha256(y16.tobytes()).hexdigest()
    # small s16 resample with saturation (loud input)
    xs = (O.gen_s16(SEED, 30, 2, 3000).astype(np.int32) // 2 * 2).astype(np.int16)
    xs[100:140] = 32767
    xs[600:660] = -32768
    ys = np.clip(np.rint(signal.resample_poly(xs.astype(np.float32), 147, 160, axis=0)),
                 -32768, 32767).astype(np.int16)
    np.savez_compressed(os.path.join(OUT, "resample_s16.npz"), x=xs, y=ys)

    # ---------------- effects -----------------------------------------------
    bands = [(1, 48000.0, 100.0, 4.0, 1.0), (0, 48000.0, 400.0, -3.0, 1.2),
             (0, 48000.0, 2000.0, 5.0, 0.9), (0, 48000.0, 6000.0, -4.0, 1.5),
             (2, 48000.0, 11000.0, 3.0, 1.0)]
    sos = np.stack([O.rbj_section(*b) for b in bands])
    xe = O.gen_f32(SEED, 40, 2, 6000)
    ybq = np.ascontiguousarray(signal.sosfilt(sos, xe, axis=0))
    assert ybq.dtype == np.float32 and bits_equal(O.biquad_f32(xe, sos), ybq)
    h63 = (O.gen_f32(SEED, 41, 1, 63)[:, 0] * np.float32(0.05)).astype(np.float32)
    yfir = np.ascontiguousarray(signal.upfirdn(h63, xe, axis=0)[: xe.shape[0]])
    assert yfir.dtype == np.float32 and bits_equal(O.fir_f32(xe, h63), yfir)
    h7 = np.array([0.1, -0.2, 0.35, 0.5, 0.35, -0.2, 0.1], np.float32)
    yfir7 = signal.upfirdn(h7, xe[:1000, 0])[:1000]
    np.savez_compressed(os.path.join(OUT, "effects.npz"), bands=np.array(bands), sos=sos,
                        x=xe, y_biquad=ybq, h63=h63, y_fir63=yfir, h7=h7, y_fir7_mono=yfir7)

    # ---------------- mixes ---------------------------------------------------
    mix = {}
    ramps_f = [
        dict(gain0=1.0, gain1=1.0, ramp_start=0, ramp_len=0, mode=0),
        dict(gain0=0.0, gain1=1.0, ramp_start=100, ramp_len=2000, mode=0),
        dict(gain0=0.8, gain1=0.25, ramp_start=0, ramp_len=4410, mode=0),
        dict(gain0=0.5, gain1=0.5, ramp_start=0, ramp_len=0, mode=0),
        dict(gain0=0.0, gain1=0.0, ramp_start=1000, ramp_len=3000, mode=1),  # xfade out
        dict(gain0=0.0, gain1=1.0, ramp_start=1000, ramp_len=3000, mode=0),  # xfade in
        dict(gain0=1.5, gain1=0.1, ramp_start=3000, ramp_len=7, mode=0),
        dict(gain0=0.3, gain1=0.9, ramp_start=2500, ramp_len=0, mode=0),       # step
    ]
    N = 4800
    xs_f = [O.gen_f32(SEED, 100 + t, 2, N) for t in range(8)]
    tracks44 = [signal.resample_poly(x, 147, 160, axis=0) for x in xs_f]
    ymix = O.mix_f32(tracks44, ramps_f)
    assert bits_equal(O.resample_mix_f32(xs_f, ramps_f, *scipy_table(147, 160)[:1], 147, 160,
                                         scipy_table(147, 160)[2]), ymix)
    mix["f32_resample8__y"] = ymix
    mix["f32_resample8__ramps"] = np.array(json.dumps(ramps_f))
    ramps_q = [
        dict(gain0_q15=32768, gain1_q15=32768, ramp_start=0, ramp_len=0, mode=0),
        dict(gain0_q15=0, gain1_q15=32768, ramp_start=50, ramp_len=1999, mode=0),
        dict(gain0_q15=65535, gain1_q15=1, ramp_start=0, ramp_len=4800, mode=0),
        dict(gain0_q15=16384, gain1_q15=16384, ramp_start=0, ramp_len=0, mode=0),
        dict(gain0_q15=0, gain1_q15=0, ramp_start=1200, ramp_len=3001, mode=1),
        dict(gain0_q15=0, gain1_q15=32768, ramp_start=1200, ramp_len=3001, mode=0),
        dict(gain0_q15=40000, gain1_q15=3, ramp_start=4000, ramp_len=13, mode=0),
        dict(gain0_q15=7, gain1_q15=60000, ramp_start=2400, ramp_len=0, mode=0),
    ]
    s_tr = [O.gen_s16(SEED, 200 + t, 2, N) for t in range(8)]
    s_tr[0][10:20] = 32767   # force saturation in the sum
    s_tr[1][10:20] = 32767
    s_tr[2][30:40] = -32768
    ys16 = O.mix_s16(s_tr, ramps_q)
    mix["s16_mix8__y"] = ys16
    mix["s16_mix8__ramps"] = np.array(json.dumps(ramps_q))
    # s16 with resampling (per-track s16 resample, then Q15 mix)
    ys16r = O.mix_s16([np.clip(np.rint(signal.resample_poly(s.astype(np.float32), 147, 160,
                                                            axis=0)), -32768, 32767
                               ).astype(np.int16) for s in s_tr[:4]], ramps_q[:4])
    mix["s16_resample4__y"] = ys16r
    np.savez_compressed(os.path.join(OUT, "mix.npz"), **mix)
    np.savez_compressed(os.path.join(OUT, "resample_fused.npz"), **fused_vectors())

    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            write_manifest_entry(manifest, f)
    with open(os.path.join(OUT, "MANIFEST.json"), "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    if "--fused" in sys.argv[1:]:
        main_fused()
    else:
        main()
