"""Dev: is the odd-N slowdown of the fused kernel the 8-B track misalignment?
Times the headline shape with (a) even N, aligned tracks, (b) even N, track
stride + 2 floats (every other track 8 B off), (c) odd N, contiguous."""
import sys
import time
sys.path[:0] = ["xm-audio-utils_amd", "."]
import torch
import xmaudio as xm
from bench import RAMPS, SEED

B = 512
for name, N, pad in (("even aligned", 480000, 0), ("even stride+8B", 480000, 2), ("odd contiguous", 480001, 0),
                     ("odd stride+8B", 480001, 2)):
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    m.set_tracks(RAMPS)
    F = m.out_frames(N)
    ts = N * 2 + pad
    x = torch.empty((B, 8 * ts), dtype=torch.float32, device="cuda")
    y = torch.empty((B, F, 2), dtype=torch.float32, device="cuda")
    x.normal_()
    s = torch.cuda.current_stream()
    m.set_stream(s.cuda_stream)
    for _ in range(2):
        m.process_strided(x.data_ptr(), ts, 8 * ts, y.data_ptr(), F * 2, B, N)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        m.process_strided(x.data_ptr(), ts, 8 * ts, y.data_ptr(), F * 2, B, N)
    torch.cuda.synchronize()
    print(f"{name:18s} {(time.perf_counter() - t0) / 10 * 1e3:.3f} ms  fast={m.timing().fast_launches}", flush=True)
    del x, y
