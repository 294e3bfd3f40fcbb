"""The fused kernel at L/M = 147/320 (round 5, VERDICT r4 item 5 / SURVEY.md
§8(f)2): 96k -> 44.1k and 48k -> 22.05k, stereo f32 mixes of 2-8 tracks
(csrc/xm_resample_d2.hip), and since round 5 stereo 1-track rows (eight
clips per wave).

A super-period is 320 input frames -> 147 outputs over a 12-segment window;
each output runs 43 or 44 used taps in two phases (taps 0..21, then 22.. one
round later), with literal coefficients.  Every case must run as one fused
launch (fast_launches == 1) and equal the C oracle bit for bit: track counts
(phantom rows), odd and tiny frame counts, lengths around super-period edges,
lanes walking several super-periods (XM_FAST_SPLIT_R), padded device strides
and scattered pointer tables, and the bench grid."""
import numpy as np
import pytest

from conftest import bits_equal

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED
RATES = [(96000, 44100), (48000, 22050)]
IDS = ["96_44", "48_22"]
L, M, SPI = 147, 320, 320


def _F(N):
    return (N * L + M - 1) // M


def _ramps(nt, F):
    base = [dict(gain0=0.9), dict(gain0=0.0, gain1=0.8, ramp_start=41, ramp_len=max(1, F // 3)),
            dict(mode=1, ramp_start=F // 4, ramp_len=max(1, F // 5)), dict(gain0=0.3, gain1=0.6, ramp_start=F // 2),
            dict(gain0=1.25, gain1=0.5, ramp_start=0, ramp_len=max(1, F)),
            dict(gain0=0.5, gain1=0.0, ramp_start=max(0, F - 900), ramp_len=800)]
    return [base[t % 6] for t in range(nt)]


def _x(B, nt, N, base):
    return np.stack([np.stack([O.gen_f32(SEED, base + 16 * b + t, 2, N) for t in range(nt)]) for b in range(B)])


def _fast(m, want=1):
    t = m.timing()
    assert t.n_launches == 1 and t.fast_launches == want, (t.n_launches, t.fast_launches)


@pytest.mark.parametrize("rates", RATES, ids=IDS)
@pytest.mark.parametrize("nt", [2, 5, 8])
def test_d2_track_counts_and_lengths(xm, gpu, rates, nt):
    fi, fo = rates
    for N in (20 * SPI + 37, 20 * SPI + 38, SPI - 1, SPI + 1, 2 * SPI, 7):
        B = 3
        x = _x(B, nt, N, 50000 + N + nt)
        ramps = _ramps(nt, _F(N))
        m = xm.Mixer(fi, fo, 2, "f32")
        m.set_tracks(ramps)
        assert m.out_frames(N) == _F(N)
        y = m.process(x)
        _fast(m)
        ref, _ = CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)
        assert bits_equal(y, ref), N


@pytest.mark.parametrize("rates", RATES, ids=IDS)
@pytest.mark.parametrize("N", [5 * SPI + 11, 20 * SPI + 38, SPI - 1, 7])
def test_d2_one_track_rows(xm, gpu, rates, N):
    """1-track mixes (round 5): eight clips per wave, each row stored to its own
    output; a ninth clip in a partly filled wave, ramped and unity gain."""
    fi, fo = rates
    B = 9
    x = _x(B, 1, N, 51000 + N)
    for ramps in ([dict(gain0=0.75)], _ramps(2, _F(N))[1:2], [dict(gain0=1.0)]):
        m = xm.Mixer(fi, fo, 2, "f32")
        m.set_tracks(ramps)
        y = m.process(x)
        _fast(m)
        assert bits_equal(y, CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)[0]), N
    c = xm.Mixer(fi, fo, 2, "f32", convert_out=True)   # s16 output
    c.set_tracks([dict(gain0=0.75)])
    ys = c.process(x)
    _fast(c)
    ref, _ = CO.batch_resample_mix_f32(x, [dict(gain0=0.75)], L, M, threads=4)
    assert bits_equal(ys, O.sat16(np.rint(ref.astype(np.float32) * np.float32(32768.0))).astype(np.int16))


@pytest.mark.parametrize("odd", [0, 1])
def test_d2_one_track_rows_multi_sp_and_tables(xm, gpu, monkeypatch, odd):
    """1-track rows walking 3 super-periods, clips ending inside a run; a
    device batch at padded strides; a scattered input pointer table."""
    import torch
    monkeypatch.setenv("XM_FAST_SPLIT_R", "3")
    N, B = SPI * (8 * 3 * 5 // 2 + 3) + 36 + odd, 11
    x = _x(B, 1, N, 51500 + odd)
    ramps = _ramps(2, _F(N))[1:2]
    m = xm.Mixer(96000, 44100, 2, "f32")
    m.set_tracks(ramps)
    y = m.process(x)
    _fast(m)
    assert xm.last_fast_split()[0] == 3
    ref, _ = CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)
    assert bits_equal(y, ref)
    monkeypatch.delenv("XM_FAST_SPLIT_R")
    d = xm.Mixer(96000, 44100, 2, "f32", mem="device")
    d.set_tracks(ramps)
    F = d.out_frames(N)
    pad = 12
    xd = torch.zeros((B, N + pad, 2), dtype=torch.float32, device="cuda")
    xd[:, :N] = torch.from_numpy(x[:, 0]).cuda()
    yd = torch.full((B, F + 4, 2), float("nan"), dtype=torch.float32, device="cuda")
    d.process_strided(xd.data_ptr(), (N + pad) * 2, (N + pad) * 2, yd.data_ptr(), (F + 4) * 2, B, N)
    torch.cuda.synchronize()
    _fast(d)
    assert bits_equal(yd[:, :F].cpu().numpy(), ref)
    # a scattered input table (evenly spaced outputs: the host passes them
    # as a stride), on the fused kernel
    perm = [(b * 5 + 2) % B for b in range(B)]
    y2 = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    d.process_ptrs([xd[b].data_ptr() for b in perm], [y2[b].data_ptr() for b in range(B)], B, N)
    torch.cuda.synchronize()
    _fast(d)
    assert bits_equal(y2.cpu().numpy(), ref[perm])


@pytest.mark.parametrize("R", [2, 3, 5])
@pytest.mark.parametrize("nt", [3, 8])
def test_d2_multi_sp(xm, gpu, monkeypatch, R, nt):
    """Lanes walking R super-periods (the carry, the next SP's segment-2 DMA
    during this one, the previous SP's last round stored in the next); clips
    ending inside a run."""
    monkeypatch.setenv("XM_FAST_SPLIT_R", str(R))
    for odd in (0, 1):
        N = SPI * (8 * R * 5 // 2 + 3) + 36 + odd
        B = 3
        x = _x(B, nt, N, 52000 + N)
        ramps = _ramps(nt, _F(N))
        m = xm.Mixer(96000, 44100, 2, "f32")
        m.set_tracks(ramps)
        y = m.process(x)
        _fast(m)
        assert xm.last_fast_split()[0] == R
        assert bits_equal(y, CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)[0]), N


def test_d2_device_strides_tables_s16_out(xm, gpu):
    """Padded device strides, a scattered pointer table, s16 output."""
    import torch
    B, nt, N = 5, 6, 9 * SPI + 3
    x = _x(B, nt, N, 53000)
    ramps = _ramps(nt, _F(N))
    ref, _ = CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)
    m = xm.Mixer(96000, 44100, 2, "f32", mem="device")
    m.set_tracks(ramps)
    F = m.out_frames(N)
    pad = 24
    xd = torch.zeros((B, nt, N + pad, 2), dtype=torch.float32, device="cuda")
    xd[:, :, :N] = torch.from_numpy(x).cuda()
    y = torch.full((B, F + 8, 2), float("nan"), dtype=torch.float32, device="cuda")
    m.process_strided(xd.data_ptr(), (N + pad) * 2, nt * (N + pad) * 2, y.data_ptr(), (F + 8) * 2, B, N)
    torch.cuda.synchronize()
    _fast(m)
    assert bits_equal(y[:, :F].cpu().numpy(), ref)
    perm = [(b * 7 + 3) % B for b in range(B)]
    ins = [xd[b, t].data_ptr() for b in perm for t in range(nt)]
    outs = [y[i].data_ptr() for i in range(B)]
    y.fill_(float("nan"))
    m.process_ptrs(ins, outs, B, N)
    torch.cuda.synchronize()
    _fast(m)
    assert bits_equal(y[:, :F].cpu().numpy(), ref[perm])
    c = xm.Mixer(96000, 44100, 2, "f32", convert_out=True)   # s16 output (round 5: the fused kernel's epilogue)
    c.set_tracks(ramps)
    ys = c.process(x)
    _fast(c)
    assert bits_equal(ys, O.sat16(np.rint(ref.astype(np.float32) * np.float32(32768.0))).astype(np.int16))


def test_d2_production_grid_96_44(xm, gpu):
    """The r96to44 bench line's shape (512 mixes x 8 tracks x 10 s at 96 kHz
    -> 44.1 kHz): first and last mix bit-checked, every output written (two
    calls over differently filled outputs agree), the split pick_split
    chooses (R >= 2)."""
    import torch
    B, nt, N = 512, 8, 960000
    ramps = _ramps(nt, _F(N))
    m = xm.Mixer(96000, 44100, 2, "f32", mem="device")
    m.set_tracks(ramps)
    F = m.out_frames(N)
    x = torch.empty((B * nt, N, 2), dtype=torch.float32, device="cuda")
    xm.synth(x.data_ptr(), "f32", SEED, 0, B * nt, 2, N)
    ys = []
    for fill in (float("nan"), 7.0):
        y = torch.full((B, F, 2), fill, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        m.process_strided(x.data_ptr(), N * 2, N * 2 * nt, y.data_ptr(), F * 2, B, N)
        torch.cuda.synchronize()
        _fast(m)
        ys.append(y)
    assert xm.last_fast_split()[0] >= 2
    for b in (0, B - 1):
        xb = x[b * nt:(b + 1) * nt].cpu().numpy()[None]
        ref, _ = CO.batch_resample_mix_f32(xb, ramps, L, M, threads=8)
        assert bits_equal(ys[0][b].cpu().numpy(), ref[0]), b
    assert bool(torch.equal(ys[0].view(torch.int32), ys[1].view(torch.int32))), "unwritten outputs"
    del x, ys
    torch.cuda.empty_cache()
