#!/usr/bin/env python3
"""Dev: config 1's form (8192 mono s16 clips, 44.1k -> 48k, unity Q15) with
the output rows at strides F + d frames: does a row base off the 64-B grid
(d = 2: 4 B per row, as an odd N gives) cost what c1odd pays?  GPU box:

    python3 tools/dev/c1_stride.py [d ...]      # default 0 2 16 32
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "xm-audio-utils_amd"))
import xmaudio as xm  # noqa: E402


def main():
    ds = [int(v) for v in sys.argv[1:]] or [0, 2, 16, 32]
    B, N = 8192, 441000
    m = xm.Mixer(44100, 48000, 1, "s16", mem="device")
    m.set_tracks([dict(gain0_q15=32768)])
    F = m.out_frames(N)
    s = torch.cuda.current_stream()
    m.set_stream(s.cuda_stream)
    x = torch.empty((B, N), dtype=torch.int16, device="cuda")
    xm.synth(x.data_ptr(), "s16", 1234, 0, B, 1, N, 0, s.cuda_stream)
    y = torch.empty(B * (F + max(ds)) + 64, dtype=torch.int16, device="cuda")
    for rep in range(2):
        for d in ds:
            st = F + d
            step = lambda: m.process_strided(x.data_ptr(), N, N, y.data_ptr(), st, B, N)  # noqa: E731
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
            print(f"stride F+{d:<3d} ({st * 2 % 64:2d} B off the 64-B grid per row)  {e0.elapsed_time(e1) / 10:.3f} ms  "
                  f"fused {t.fast_launches}/{t.n_launches}", flush=True)


if __name__ == "__main__":
    main()
