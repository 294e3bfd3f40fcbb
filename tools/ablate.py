#!/usr/bin/env python3
"""Time the headline kernel under XM_FAST_ABLATE variants, interleaved in one
process (methodology: cdna_hip_programming.md §5.4 rule 24).  Profiling only."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xm-audio-utils_amd"))
import torch
import xmaudio as xm
sys.path.insert(0, ROOT)
from bench import RAMPS, SEED
B, ntr, N = int(os.environ.get("MIXES", 512)), 8, 480000
m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
m.set_tracks(RAMPS)
F = m.out_frames(N)
x = torch.empty((B, ntr, N, 2), dtype=torch.float32, device="cuda")
y = torch.empty((B, F, 2), dtype=torch.float32, device="cuda")
xm.synth(x.data_ptr(), "f32", SEED, 0, B * ntr, 2, N)
s = torch.cuda.current_stream(); m.set_stream(s.cuda_stream)
variants = [int(v) for v in (sys.argv[1:] or ["0", "1", "2", "4", "7"])]
res = {v: [] for v in variants}
for rnd in range(5):
    for v in variants:
        os.environ["XM_FAST_ABLATE"] = str(v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        m.process_strided(x.data_ptr(), N * 2, ntr * N * 2, y.data_ptr(), F * 2, B, N)
        e0.record(s)
        for _ in range(3):
            m.process_strided(x.data_ptr(), N * 2, ntr * N * 2, y.data_ptr(), F * 2, B, N)
        e1.record(s); torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / 3)
print(json.dumps({v: [round(min(t), 3), round(sorted(t)[len(t)//2], 3)] for v, t in res.items()}))
