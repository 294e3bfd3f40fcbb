"""Dev: one planar 8-track mix through the fused kernel, output saved for CPU analysis."""
import sys
sys.path[:0] = ["xm-audio-utils_amd", "oracle", "."]
import numpy as np
import xmaudio as xm
import np_oracle as O
from bench import RAMPS
N = 4800
x = np.stack([np.stack([O.gen_f32(O.SEED, 6600 + t, 2, N) for t in range(8)])])
m = xm.Mixer(48000, 44100, 2, "f32", planar=True)
m.set_tracks(RAMPS)
y = m.process(np.ascontiguousarray(np.swapaxes(x, -1, -2)))
print("fast", m.timing().fast_launches)
np.savez("gpurun_out/pl_dbg.npz", x=x, y=y)
