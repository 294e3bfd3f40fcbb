#!/usr/bin/env python3
"""Dev only: the block kernel (csrc/xm_resample_blk.hip) against the C oracle
on small cases, printing where outputs first differ."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "xm-audio-utils_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import xmaudio as xm  # noqa: E402
import c_oracle as CO  # noqa: E402
import np_oracle as O  # noqa: E402

SEED = O.SEED


def show(name, y, ref):
    y = np.asarray(y)
    ref = np.asarray(ref)
    if y.shape != ref.shape:
        print(name, "SHAPE", y.shape, ref.shape, flush=True)
        return
    bad = np.argwhere(y.view(np.uint32 if y.dtype == np.float32 else np.uint16) !=
                      ref.view(np.uint32 if ref.dtype == np.float32 else np.uint16))
    print(f"{name}: {len(bad)} of {y.size} differ", flush=True)
    for idx in bad[:6]:
        i = tuple(idx)
        print("   ", i, y[i], ref[i], flush=True)


def main():
    for fi, fo, C, N in [(32000, 48000, 2, 3201), (32000, 48000, 1, 3201), (44100, 48000, 1, 4410),
                         (48000, 16000, 2, 4801), (44100, 48000, 2, 4410)]:
        from math import gcd
        g = gcd(fi, fo)
        L, M = fo // g, fi // g
        x = O.gen_f32(SEED, 7, C, N)
        m = xm.Mixer(fi, fo, C, "f32")
        y = m.process(x[None, None])[0]
        t = m.timing()
        show(f"f32 {fi}->{fo} C{C} N{N} (launches {t.n_launches} fast {t.fast_launches})", y,
             CO.resample_f32(x, L, M))
    xs = O.gen_s16(SEED, 0, 1, 44100)
    m = xm.Mixer(44100, 48000, 1, "s16")
    show("s16 mono 44.1->48", m.process(xs[None, None])[0], CO.resample_s16(xs, 160, 147))
    # streamed 48k -> 44.1k stereo: window jobs
    x = np.stack([O.gen_f32(SEED, 11 + t, 2, 9000) for t in range(2)])[None]
    ramps = [dict(gain0=0.8), dict(gain0=0.5)]
    m = xm.Mixer(48000, 44100, 2, "f32")
    m.set_tracks(ramps)
    whole = m.process(x)
    m.stream_begin(1)
    parts = [m.stream_push(x[:, :, a:b]) for a, b in ((0, 1), (1, 38), (38, 1038), (1038, 5134), (5134, 9000))]
    parts.append(m.stream_flush())
    show("stream 48->44.1", np.concatenate(parts, axis=1), whole)
    show("whole 48->44.1 vs oracle", whole, CO.resample_mix_f32(list(x[0]), ramps, 147, 160)[None])


if __name__ == "__main__":
    main()
