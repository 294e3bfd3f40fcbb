"""Dev: minimal stream push on the GPU with HIP error logging."""
import os, sys
sys.path[:0] = ["xm-audio-utils_amd", "oracle"]
import numpy as np
import xmaudio as xm
m = xm.Mixer(48000, 44100, 2, "f32")
m.stream_begin(1)
for n in (0, 1, 5, 137):
    x = np.ones((1, 1, n, 2), np.float32)
    try:
        y = m.stream_push(x)
        print("push", n, "->", y.shape, flush=True)
    except Exception as e:
        print("push", n, "FAILED", e, flush=True)
        break
