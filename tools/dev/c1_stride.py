#!/usr/bin/env python3
"""Dev: config 1's form (8192 mono s16 clips, 44.1k -> 48k, unity Q15), or
config 2's (--c2: 4096 stereo f32 clips, 48k -> 44.1k), with the output rows
at strides F + d frames: what does a row base off the 64-B grid cost?  GPU box:

    python3 tools/dev/c1_stride.py [--c2] [d ...]      # default d: 0 2 16 32 (c2: 0 1 4 8)
    python3 tools/dev/c1_stride.py --rows FI FO N B [d ...]   # B stereo f32 1-track rows FI -> FO
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "xm-audio-utils_amd"))
import xmaudio as xm  # noqa: E402


def main():
    argv = sys.argv[1:]
    rows = argv[:1] == ["--rows"]
    if rows:
        fi, fo, N, B = (int(v) for v in argv[1:5])
        argv = argv[5:]
    c2 = "--c2" in argv or rows
    ds = [int(v) for v in argv if v != "--c2"] or ([0, 1, 4, 8] if c2 else [0, 2, 16, 32])
    if rows:
        C, fmt, esz = 2, "f32", 4
        m = xm.Mixer(fi, fo, 2, "f32", mem="device")
        m.set_tracks([dict(gain0=1.0)])
    elif c2:
        B, N, C, fmt, esz = 4096, 480000, 2, "f32", 4
        m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    else:
        B, N, C, fmt, esz = 8192, 441000, 1, "s16", 2
        m = xm.Mixer(44100, 48000, 1, "s16", mem="device")
        m.set_tracks([dict(gain0_q15=32768)])
    F = m.out_frames(N)
    s = torch.cuda.current_stream()
    m.set_stream(s.cuda_stream)
    dt = torch.float32 if c2 else torch.int16
    x = torch.empty((B, N * C), dtype=dt, device="cuda")
    xm.synth(x.data_ptr(), fmt, 1234, 0, B, C, N, 0, s.cuda_stream)
    y = torch.empty(B * (F + max(ds)) * C + 64, dtype=dt, device="cuda")
    for rep in range(2):
        for d in ds:
            st = F + d
            step = lambda: m.process_strided(x.data_ptr(), N * C, N * C, y.data_ptr(), st * C, B, N)  # noqa: E731
            for _ in range(2):
                step()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(s)
            for _ in range(10):
                step()
            e1.record(s)
            torch.cuda.synchronize()
            t = m.timing()
            print(f"stride F+{d:<3d} ({st * C * esz % 64:2d} B off the 64-B grid per row)  {e0.elapsed_time(e1) / 10:.3f} ms  "
                  f"fused {t.fast_launches}/{t.n_launches}", flush=True)


if __name__ == "__main__":
    main()
