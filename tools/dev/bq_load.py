"""Dev: config-4 biquad stage alone (1024 stereo clips x 441000 frames, 5-band
EQ, device memory, in place), for timing and PMC passes on k_biquad_pipe."""
import sys
import time
sys.path[:0] = ["xm-audio-utils_amd", "oracle"]
import torch
import xmaudio as xm

B, N = 1024, 441000
x = torch.empty((B, N, 2), dtype=torch.float32, device="cuda")
xm.synth(x.data_ptr(), "f32", 0x584D4155, 0, B, 2, N, 0, torch.cuda.current_stream().cuda_stream)
e = xm.Effects(44100, 2, mem="device")
for f0, g in ((60, 3.0), (250, -2.0), (1000, 4.0), (4000, -3.0), (12000, 2.0)):
    e.add_eq_band(0, float(f0), g, 1.0)
ptrs = [x[i].data_ptr() for i in range(B)]
torch.cuda.synchronize()
for it in range(2):
    t0 = time.perf_counter()
    e.process_ptrs(ptrs, ptrs, N)
    torch.cuda.synchronize()
    print(f"biquad pass {it}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
