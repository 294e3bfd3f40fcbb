#!/usr/bin/env python3
"""Cycle attribution for the fast kernel (dev, GPU box): runs the headline
workload once on the lib_ablate/ build with XM_FAST_ABLATE=16 and prints the
share of wave time spent waiting for LDS-DMA segments (copy_seg's vmcnt)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["XM_AUDIO_LIB"] = os.path.join(ROOT, "xm-audio-utils_amd", "lib_ablate", "libxm_audio.so")
os.environ.setdefault("XM_FAST_ABLATE", "16")   # 16 | other ablation bits
sys.path.insert(0, os.path.join(ROOT, "xm-audio-utils_amd"))
import torch  # noqa: E402
import xmaudio as xm  # noqa: E402

sys.path.insert(0, ROOT)
from bench import RAMPS, SEED  # noqa: E402

B, NT, N = int(os.environ.get("MIXES", "512")), 8, 480000
m = xm.Mixer(48000, 44100, 2, "f32", mem="device", device=0)
m.set_tracks(RAMPS)
F = m.out_frames(N)
x = torch.empty((B, NT, N, 2), dtype=torch.float32, device="cuda")
y = torch.empty((B, F, 2), dtype=torch.float32, device="cuda")
xm.synth(x.data_ptr(), "f32", SEED, 0, B * NT, 2, N, 0, 0)
lib = xm._lib
f = lib.xm_dev_fast_prof
f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 8)()
for it in range(2):
    f(buf)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    m.process_strided(x.data_ptr(), N * 2, NT * N * 2, y.data_ptr(), F * 2, B, N)
    ev1.record()
    torch.cuda.synchronize()
    f(buf)
    tot, wait, waves, issue, copy, ssum = list(buf)[:6]
    ms = ev0.elapsed_time(ev1)
    print(f"abl {os.environ['XM_FAST_ABLATE']} run {it}: {ms:.3f} ms  clock {tot / waves / (ms * 1e3):.0f} MHz(1 gen)  waves {waves}  cycles/wave {tot / waves:.0f}  "
          f"dma-wait {100 * wait / tot:.1f}%  dma-issue {100 * issue / tot:.1f}%  "
          f"copy {100 * copy / tot:.1f}%  sum-store {100 * ssum / tot:.1f}%", flush=True)
