"""Config 5 (BASELINE.json:11): 64-track mixdowns whose tracks live on
different devices.  On one GPU the devices are separate mixer handles, each
holding 8 of the 64 tracks, exactly as 8 ranks would: each forms the int32
Q15 partial of its tracks, the partials are summed (by finish_s16 over 8
parts, or by xmaudio.dist's exchange at world 1) and saturated.  Every mix
must equal the oracle's one-pass 64-track mix bit for bit, saturation
included (DESIGN.md §2 "Config 5 partials")."""
import numpy as np
import pytest

from conftest import bits_equal

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED
NT, PARTS = 64, 8
_R = [(32768, 32768, 0, 0, 0), (0, 32768, 100, 20000, 0), (65535, 100, 0, 9600, 0), (16384, 16384, 0, 0, 0),
      (0, 0, 5000, 900, 1), (0, 32768, 5000, 900, 0), (40000, 3, 7000, 13, 0), (7, 60000, 4800, 0, 0)]
RAMPS64 = [dict(gain0_q15=q + 97 * i if q else 0, gain1_q15=q2, ramp_start=s + 31 * i, ramp_len=ln, mode=md)
           for i in range(PARTS) for q, q2, s, ln, md in _R]
for r in RAMPS64:
    r["gain0_q15"] = min(r["gain0_q15"], 65535)


def _tracks(B, N):
    x = np.stack([np.stack([O.gen_s16(SEED, 9000 + NT * b + t, 2, N) for t in range(NT)]) for b in range(B)])
    x[:, :6, 200:700] = 32767        # the 64-track sum saturates high ...
    x[:, 58:, 1500:1900] = -32768    # ... and low
    return x


def _oracle(x):
    return CO.batch_mix_s16(x, RAMPS64, threads=4)[0]


def test_64_tracks_8_parts_finish(xm, gpu):
    """64 s16 tracks over 8 handles -> 8 int32 partials -> finish_s16(n_parts=8)."""
    import torch
    B, N = 4, 48000
    x = _tracks(B, N)
    want = _oracle(x)
    assert np.sum(np.abs(want.astype(np.int32)) >= 32767) > 1000   # saturation is exercised
    xd = torch.from_numpy(x).cuda()
    parts = torch.empty((PARTS, B, N * 2), dtype=torch.int32, device="cuda")
    m = None
    for p in range(PARTS):
        m = xm.Mixer(48000, 48000, 2, "s16", mem="device")
        m.set_tracks(RAMPS64[8 * p: 8 * p + 8])
        xh = xd[:, 8 * p: 8 * p + 8].contiguous()
        m.process_partial_strided(xh.data_ptr(), N * 2, 8 * N * 2, parts[p].data_ptr(), N * 2, B, N)
    torch.cuda.synchronize()
    for p in (0, PARTS - 1):          # the partials themselves vs the numpy oracle
        got = parts[p, 1].cpu().numpy()
        assert bits_equal(got, O.mix_s16_partial(list(x[1, 8 * p: 8 * p + 8]), RAMPS64[8 * p: 8 * p + 8]).reshape(-1))
    y = torch.empty((B, N, 2), dtype=torch.int16, device="cuda")
    m.finish_s16(parts.data_ptr(), PARTS, B * N * 2, N * 2, y.data_ptr(), N * 2, B, N)
    assert bits_equal(y.cpu().numpy(), want)
    # one handle holding all 64 tracks gives the same bits
    full = xm.Mixer(48000, 48000, 2, "s16")
    full.set_tracks(RAMPS64)
    assert bits_equal(full.process(x), want)


def test_mix_spanning_world1(xm, gpu):
    """xmaudio.dist.mix_spanning_s16 at world size 1 (partial -> exchange ->
    finish through the same function the multi-rank job runs)."""
    import torch
    from xmaudio import dist as xdist
    B, N = 3, 24000
    x = _tracks(B, N)
    m = xm.Mixer(48000, 48000, 2, "s16", mem="device")
    m.set_tracks(RAMPS64)
    y = xdist.mix_spanning_s16(xdist.Rank(0, 1, 0), m, torch.from_numpy(x).cuda())
    assert bits_equal(y.cpu().numpy(), _oracle(x))


def test_64_tracks_8_parts_resampled(xm, gpu):
    """The same split through the resampling (generic) kernel, 48k -> 44.1k:
    8 partial handles + finish equal one 64-track handle bit for bit."""
    import torch
    B, N = 2, 9600 + 33
    x = _tracks(B, N)
    full = xm.Mixer(48000, 44100, 2, "s16")
    full.set_tracks(RAMPS64)
    want = full.process(x)
    F = full.out_frames(N)
    for b in range(B):                # the one-handle resample+mix vs the C oracle
        assert bits_equal(want[b], CO.resample_mix_s16(list(x[b]), RAMPS64, 147, 160))
    xd = torch.from_numpy(x).cuda()
    parts = torch.empty((PARTS, B, F * 2), dtype=torch.int32, device="cuda")
    for p in range(PARTS):
        m = xm.Mixer(48000, 44100, 2, "s16", mem="device")
        m.set_tracks(RAMPS64[8 * p: 8 * p + 8])
        xh = xd[:, 8 * p: 8 * p + 8].contiguous()
        m.process_partial_strided(xh.data_ptr(), N * 2, 8 * N * 2, parts[p].data_ptr(), F * 2, B, N)
    y = torch.empty((B, F, 2), dtype=torch.int16, device="cuda")
    m.finish_s16(parts.data_ptr(), PARTS, B * F * 2, F * 2, y.data_ptr(), F * 2, B, F)
    assert bits_equal(y.cpu().numpy(), want)
