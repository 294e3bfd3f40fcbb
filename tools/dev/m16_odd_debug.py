"""Dev: where mono s16 odd-N outputs differ from the oracle (clip, output
index, plane half, SP position)."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "xm-audio-utils_amd"))
import c_oracle as CO  # noqa: E402
import np_oracle as O  # noqa: E402
import xmaudio as xm  # noqa: E402

for (fi, fo, L, M, SPO) in ((48000, 44100, 147, 160, 147), (44100, 48000, 160, 147, 160)):
    for N in (48001, 4801, 961):
        for nt in (1, 3):
            B = 11 if nt == 1 else 3
            x = np.stack([np.stack([O.gen_s16(O.SEED, 30000 + 100 * nt + 16 * b + t, 1, N) for t in range(nt)]) for b in range(B)])
            q = [dict(gain0_q15=32768)] * nt
            m = xm.Mixer(fi, fo, 1, "s16")
            m.set_tracks(q)
            y = m.process(x)
            R, tpm = xm.last_fast_split()
            ref = np.stack([CO.resample_mix_s16(list(x[b]), q, L, M) for b in range(B)])
            bad = np.argwhere(y[..., 0] != ref[..., 0])
            print(f"{fi}->{fo} N={N} nt={nt} R={R} tpm={tpm} F={y.shape[1]} bad={len(bad)}", flush=True)
            for b, n in bad[:12]:
                print("   clip", b, "out", n, "sp", n // SPO, "k", n % SPO, "got", y[b, n, 0], "want", ref[b, n, 0])
