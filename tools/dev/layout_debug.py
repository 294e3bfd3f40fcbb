"""Dev: the 16-row (S = 4) layout through pointer tables vs strides; prints
where the outputs differ from the oracle (first bad frame, fraction)."""
import sys
sys.path[:0] = ["xm-audio-utils_amd", "oracle", "tests"]
import numpy as np
import torch
import xmaudio as xm
import c_oracle as CO
import np_oracle as O
from test_gpu_fast_layouts import _ramps, _x

for nt in (12, 9, 16, 8):
    N, B = 9601, 9
    x = _x(B, nt, N, 8000 + 100 * nt)
    ramps = _ramps(nt, N)
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    m.set_tracks(ramps)
    F = m.out_frames(N)
    ts, ms = N * 2 + 6, (N * 2 + 6) * nt + 10
    buf = np.zeros(B * ms + 16, np.float32)
    for b in range(B):
        for t in range(nt):
            buf[b * ms + t * ts: b * ms + t * ts + 2 * N] = x[b, t].reshape(-1)
    xd = torch.from_numpy(buf).cuda()
    perm = [(5 * t + 3) % nt for t in range(nt)]
    ref, _ = CO.batch_resample_mix_f32(x[:, perm], ramps, 147, 160, threads=8)
    for mode in ("in_table_out_strided", "in_table_out_table", "in_identity_table"):
        p = perm if mode != "in_identity_table" else list(range(nt))
        ins = [xd[b * ms + p[t] * ts:].data_ptr() for b in range(B) for t in range(nt)]
        y = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
        outs = [y[b].data_ptr() for b in range(B)] if mode != "in_table_out_table" else \
            [y[(3 * b) % B].data_ptr() for b in range(B)]
        m.process_ptrs(ins, outs, B, N)
        torch.cuda.synchronize()
        got = y.cpu().numpy()
        want = ref if mode != "in_identity_table" else CO.batch_resample_mix_f32(x, ramps, 147, 160, threads=8)[0]
        for b in range(B):
            o = (3 * b) % B if mode == "in_table_out_table" else b
            bad = np.nonzero((got[o].view(np.uint32) != want[b].view(np.uint32)).any(axis=1))[0]
            if len(bad):
                print(f"nt={nt} {mode} mix {b}: {len(bad)} bad frames of {F}, first {bad[0]}, last {bad[-1]}, "
                      f"fast={m.timing().fast_launches}", flush=True)
                break
        else:
            print(f"nt={nt} {mode}: all equal, fast={m.timing().fast_launches}", flush=True)
