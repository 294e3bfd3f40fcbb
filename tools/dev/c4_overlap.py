#!/usr/bin/env python3
"""Dev only: does the config-4 biquad stage slow down when the resample kernel
runs beside it on another stream?  The biquad chain waves are latency-bound
and occupy few SIMDs (1024 stereo clips x 5 sections: 160 chain waves), so a
time-block pipeline could hide the resample and the mix under it.

Prints the biquad stage alone, the resample (1024 1-track 48k->44.1k mixes)
alone, and both launched together on two streams (events on each stream)."""
import sys
import time

sys.path[:0] = ["xm-audio-utils_amd", "oracle"]
import torch  # noqa: E402
import xmaudio as xm  # noqa: E402

B, N, NI = 1024, 441000, 480000
x = torch.empty((B, N, 2), dtype=torch.float32, device="cuda")
xi = torch.empty((B, NI, 2), dtype=torch.float32, device="cuda")
yr = torch.empty((B, N, 2), dtype=torch.float32, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
xm.synth(x.data_ptr(), "f32", 0x584D4155, 0, B, 2, N, 0, torch.cuda.current_stream().cuda_stream)
xm.synth(xi.data_ptr(), "f32", 0x584D4155, 7, B, 2, NI, 0, torch.cuda.current_stream().cuda_stream)
e = xm.Effects(44100, 2, mem="device")
for f0, g in ((60, 3.0), (250, -2.0), (1000, 4.0), (4000, -3.0), (12000, 2.0)):
    e.add_eq_band(0, float(f0), g, 1.0)
e.set_stream(s1.cuda_stream)
m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
m.set_tracks([dict(gain0=1.0)])
m.set_stream(s2.cuda_stream)
ptrs = [x[i].data_ptr() for i in range(B)]
torch.cuda.synchronize()


def bq():
    e.process_ptrs(ptrs, ptrs, N)


def rs(k=1):
    for _ in range(k):
        m.process_strided(xi.data_ptr(), NI * 2, NI * 2, yr.data_ptr(), N * 2, B, NI)


def timed(fn, st):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    fn()
    b.record(st)
    return a, b


for it in range(3):
    a, b = timed(bq, s1)
    torch.cuda.synchronize()
    t_bq = a.elapsed_time(b)
    a, b = timed(rs, s2)
    torch.cuda.synchronize()
    t_rs = a.elapsed_time(b)
    t0 = time.perf_counter()
    a1, b1 = timed(bq, s1)
    a2, b2 = timed(lambda: rs(3), s2)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    print(f"run {it}: biquad alone {t_bq:.2f} ms, resample alone {t_rs:.2f} ms; together: biquad {a1.elapsed_time(b1):.2f} ms, "
          f"3 resamples {a2.elapsed_time(b2):.2f} ms, wall {wall:.2f} ms", flush=True)
