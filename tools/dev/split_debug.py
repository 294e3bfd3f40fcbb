"""Dev: config 2's split mode at production size; which clips are unwritten
(NaN) or differ from the oracle (sampled)."""
import sys
sys.path[:0] = ["xm-audio-utils_amd", "oracle"]
import numpy as np
import torch
import xmaudio as xm
import c_oracle as CO

for B, N in ((4096, 480000), (512, 480000), (4096, 48000), (1024, 480000)):
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    m.set_tracks([dict(gain0=1.0)])
    F = m.out_frames(N)
    x = torch.empty((B, N, 2), dtype=torch.float32, device="cuda")
    xm.synth(x.data_ptr(), "f32", 0x584D4155, 0, B, 2, N)
    y = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    m.process_strided(x.data_ptr(), N * 2, N * 2, y.data_ptr(), F * 2, B, N)
    torch.cuda.synchronize()
    t = m.timing()
    nanclip = y.isnan().any(dim=2).any(dim=1).nonzero().flatten().cpu().numpy()
    frames_nan = y[nanclip[:1]].isnan().any(dim=2).nonzero()[:, 1].cpu().numpy() if len(nanclip) else []
    bad = []
    for b in sorted({0, 7, 8, B // 2, B - 8, B - 1}):
        if not np.array_equal(y[b].cpu().numpy().view(np.uint32), CO.resample_f32(x[b].cpu().numpy(), 147, 160).view(np.uint32)):
            bad.append(b)
    print(f"B={B} N={N} fast={t.fast_launches}/{t.n_launches} nan clips={len(nanclip)} first={nanclip[:5]} "
          f"last={nanclip[-3:]} nan frames of first: {len(frames_nan)} [{frames_nan[:3]}..{frames_nan[-3:] if len(frames_nan) else ''}] "
          f"mismatch (sampled)={bad}", flush=True)
    del x, y
    torch.cuda.empty_cache()
