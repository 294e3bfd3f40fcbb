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
# dev builds with -DXM_BQ_PROF: per-wave cycle split of the last pass (k_biquad_pc:
# [workgroup][chain, producer, load, store][work, barrier wait])
import ctypes
import numpy as np
fn = getattr(xm._lib, "xm_dev_bq_prof", None)
if fn is not None:
    buf = np.zeros(4096, np.uint64)
    fn(buf.ctypes.data_as(ctypes.c_void_p))
    w = buf.reshape(512, 4, 2).astype(np.float64)
    w = w[w[:, 0, 0] > 0]                      # the launch's workgroups
    steps = (N + 63) // 64 + 2 * 5 + 1
    for k, name in enumerate(("chain", "producer", "load", "store")):
        print("%-8s wave, cycles per 64-frame step: work %.0f  barrier/wait %.0f" % ((name,) + tuple(w[:, k].mean(0) / steps)),
              flush=True)
fh = getattr(xm._lib, "xm_dev_bq_hw", None)
if fh is not None:
    hw = np.zeros(2048, np.uint32)
    fh(hw.ctypes.data_as(ctypes.c_void_p))
    hw = hw.reshape(512, 4)[: len(w)]
    simd = (hw >> 4) & 3
    same = sum(len(set(r)) < 4 for r in simd)
    print("SIMD of (chain, producer, load, store), first workgroups:", [tuple(int(v) for v in r) for r in simd[:6]],
          "; workgroups with a shared SIMD:", same, "of", len(simd), flush=True)
