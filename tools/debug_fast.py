#!/usr/bin/env python3
"""Debug helper: run the fused kernel on one mix and map mismatches vs the C oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "xm-audio-utils_amd"), os.path.join(ROOT, "oracle")]
import numpy as np
import xmaudio as xm
import c_oracle as CO
import np_oracle as O
N = int(sys.argv[1]) if len(sys.argv) > 1 else 48000
solo = int(sys.argv[2]) if len(sys.argv) > 2 else -1
ramps = ([dict(gain0=1.0 if t == solo else 0.0) for t in range(8)] if solo >= 0
         else [dict(gain0=0.5 + 0.05 * t) for t in range(8)])
x = np.stack([O.gen_f32(O.SEED, 10 + t, 2, N) for t in range(8)])[None]
m = xm.Mixer(48000, 44100, 2, "f32")
m.set_tracks(ramps)
y = m.process(x)[0]
ref = CO.resample_mix_f32(list(x[0]), ramps, 147, 160)
bad = np.nonzero(np.any(y.view(np.uint32) != ref.view(np.uint32), axis=1))[0]
print("solo", solo, "N", N, "frames_out", y.shape[0], "bad frames", len(bad))
if len(bad):
    sp = bad // 147
    print("bad SPs (first 20):", np.unique(sp)[:20], "count", len(np.unique(sp)))
    print("bad k within SP histogram (first 20):", np.bincount(bad % 147)[:20])
    i = bad[0]
    print("first bad", i, y[i], ref[i], " max abs err", np.max(np.abs(y - ref)))
