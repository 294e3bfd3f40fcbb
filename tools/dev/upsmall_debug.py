#!/usr/bin/env python3
"""Dev only: the 2/1 and 3/1 fused mixes at runs of several super-periods per
lane, where the production bench lines disagree with the oracle.  Outputs are
pre-filled with a sentinel; prints which (SP, output) positions differ and
whether they were written at all."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "xm-audio-utils_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import xmaudio as xm  # noqa: E402
import c_oracle as CO  # noqa: E402
import np_oracle as O  # noqa: E402

SEED = O.SEED
SENT = np.uint32(0x7FC0DEAD)
for fi, fo, L, M, SPO in ((24000, 48000, 2, 1, 320), (16000, 48000, 3, 1, 480)):
    for B, nt, N in ((64, 2, 48000), (16, 8, 96000)):
        x = np.stack([np.stack([O.gen_f32(SEED, 100 * b + t, 2, N) for t in range(nt)]) for b in range(B)])
        ramps = [dict(gain0=0.9 - 0.1 * t) for t in range(nt)]
        m = xm.Mixer(fi, fo, 2, "f32", mem="device")
        m.set_tracks(ramps)
        F = m.out_frames(N)
        xd = torch.from_numpy(x).cuda()
        yd = torch.full((B, F, 2), 0, dtype=torch.int32, device="cuda")
        yd.fill_(int(SENT.view(np.int32)))
        m.process_strided(xd.data_ptr(), N * 2, nt * N * 2, yd.data_ptr(), F * 2, B, N)
        torch.cuda.synchronize()
        t = m.timing()
        y = yd.cpu().numpy().view(np.float32)
        ref, _ = CO.batch_resample_mix_f32(x, ramps, L, M, threads=16)
        badm = (y.view(np.uint32) != ref.view(np.uint32)).any(axis=2)
        unw = (y.view(np.uint32) == SENT).any(axis=2)
        nb = int(badm.sum())
        print(f"{fi}->{fo} B{B} nt{nt} N{N}: fast {t.fast_launches}, {nb} of {badm.size} frames differ, "
              f"{int(unw.sum())} unwritten", flush=True)
        if nb:
            bm, bf = np.nonzero(badm)
            for mix in np.unique(bm)[:2]:
                fr = bf[bm == mix]
                sps = fr // SPO
                print(f"   mix {mix}: SPs with errors {np.unique(sps)[:40]}", flush=True)
                for s in np.unique(sps)[:4]:
                    ks = fr[sps == s] % SPO
                    w = unw[mix, fr[sps == s]]
                    print(f"     SP {s}: k {ks.min()}..{ks.max()} ({len(ks)}), unwritten {int(w.sum())}", flush=True)
