"""The fused kernel at L/M = 320/147 (round 5, VERDICT r4 item 5 / SURVEY.md
§8(f)2): 44.1k -> 96k and 22.05k -> 48k, stereo f32 mixes of 2-8 tracks.

A super-period is 147 input frames -> 320 outputs (40 exchange rounds); each
output runs its own used-tap run (kOffU2 / kPtU2, tools/gen_coefs.c
emit_offsets), like 44.1k -> 48k.  Round 5 added stereo 1-track rows and
mono f32 tracks (1-track rows with grouped, transposed stores; mixes of 2-8).  Every case must run as one fused launch
(fast_launches == 1) and equal the C oracle bit for bit: track counts (phantom
rows), odd and tiny frame counts, lengths around super-period edges, lanes
walking several super-periods (XM_FAST_SPLIT_R), padded device strides and
scattered pointer tables, the s16 store epilogue, and the bench grid."""
import numpy as np
import pytest

from conftest import bits_equal

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED
RATES = [(44100, 96000), (22050, 48000)]
IDS = ["44_96", "22_48"]
L, M, SPI = 320, 147, 147


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
def test_u2_track_counts_and_lengths(xm, gpu, rates, nt):
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


@pytest.mark.parametrize("R", [2, 3, 5])
@pytest.mark.parametrize("nt", [3, 8])
def test_u2_multi_sp(xm, gpu, monkeypatch, R, nt):
    """Lanes walking R super-periods (the carry, the next SP's segment-2 DMA
    during this one, the previous SP's last round stored in the next); clips
    ending inside a run."""
    monkeypatch.setenv("XM_FAST_SPLIT_R", str(R))
    for odd in (0, 1):
        N = SPI * (8 * R * 5 // 2 + 3) + 36 + odd
        B = 3
        x = _x(B, nt, N, 52000 + N)
        ramps = _ramps(nt, _F(N))
        m = xm.Mixer(44100, 96000, 2, "f32")
        m.set_tracks(ramps)
        y = m.process(x)
        _fast(m)
        assert xm.last_fast_split()[0] == R
        assert bits_equal(y, CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)[0]), N


def test_u2_device_strides_tables_s16_out(xm, gpu):
    """Padded device strides, a scattered pointer table, s16 output."""
    import torch
    B, nt, N = 5, 6, 9 * SPI + 3
    x = _x(B, nt, N, 53000)
    ramps = _ramps(nt, _F(N))
    ref, _ = CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)
    m = xm.Mixer(44100, 96000, 2, "f32", mem="device")
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
    c = xm.Mixer(44100, 96000, 2, "f32", convert_out=True)
    c.set_tracks(ramps)
    ys = c.process(x)
    _fast(c)
    assert bits_equal(ys, O.sat16(np.rint(ref.astype(np.float32) * np.float32(32768.0))).astype(np.int16))


def test_u2_production_grid_44_96(xm, gpu):
    """The r44to96 bench line's shape (512 mixes x 8 tracks x 10 s at 44.1 kHz
    -> 96 kHz): first and last mix bit-checked, every output written (two
    calls over differently filled outputs agree), the split pick_split
    chooses (R >= 2)."""
    import torch
    B, nt, N = 512, 8, 441000
    ramps = _ramps(nt, _F(N))
    m = xm.Mixer(44100, 96000, 2, "f32", mem="device")
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


# ---- round 5: 320/147 mono f32 tracks and stereo 1-track rows ------------------

@pytest.mark.parametrize("rates", RATES, ids=IDS)
@pytest.mark.parametrize("nt", [1, 3, 8])
def test_u2_mono(xm, gpu, rates, nt):
    """Mono f32 tracks at 320/147: 1-track rows (eight clips per wave, the
    grouped transposed stores DSF) and mixes of 2-8 tracks; odd and short
    lengths, every output against the C oracle."""
    fi, fo = rates
    for N in (20 * SPI + 37, SPI * 16 + 1, SPI + 1, 7):
        B = 11 if nt == 1 else 3
        x = np.stack([np.stack([O.gen_f32(SEED, 54000 + N + 16 * b + t, 1, N) for t in range(nt)]) for b in range(B)])
        ramps = _ramps(nt, _F(N))
        m = xm.Mixer(fi, fo, 1, "f32")
        m.set_tracks(ramps)
        y = m.process(x)
        _fast(m)
        assert bits_equal(y, CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)[0]), N


@pytest.mark.parametrize("R", [4, 6])
@pytest.mark.parametrize("nt", [1, 8])
def test_u2_mono_multi_sp(xm, gpu, monkeypatch, R, nt):
    """Mono runs of 2 and 3 SPs per plane; clips ending inside a run."""
    monkeypatch.setenv("XM_FAST_SPLIT_R", str(R))
    N = SPI * (8 * R * 5 // 2 + 3) + 36
    B = 11 if nt == 1 else 3
    x = np.stack([np.stack([O.gen_f32(SEED, 55000 + N + 16 * b + t, 1, N) for t in range(nt)]) for b in range(B)])
    ramps = _ramps(nt, _F(N))
    m = xm.Mixer(44100, 96000, 1, "f32")
    m.set_tracks(ramps)
    y = m.process(x)
    _fast(m)
    assert xm.last_fast_split()[0] == R
    assert bits_equal(y, CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)[0]), N


@pytest.mark.parametrize("rates", RATES, ids=IDS)
def test_u2_stereo_one_track_rows(xm, gpu, rates):
    """Stereo 1-track mixes at 320/147 (eight clips per wave: a timeline's
    per-track resampling, resample-only batches), ramped and unity gain,
    f32 and s16 output, a ninth clip in a partly filled wave."""
    fi, fo = rates
    N, B = 20 * SPI + 37, 9
    x = _x(B, 1, N, 56000)
    for ramps in ([dict(gain0=0.75)], _ramps(2, _F(N))[1:2], [dict(gain0=1.0)]):
        m = xm.Mixer(fi, fo, 2, "f32")
        m.set_tracks(ramps)
        y = m.process(x)
        _fast(m)
        ref, _ = CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)
        assert bits_equal(y, ref)
    c = xm.Mixer(fi, fo, 2, "f32", convert_out=True)
    c.set_tracks([dict(gain0=0.75)])
    ys = c.process(x)
    _fast(c)
    ref, _ = CO.batch_resample_mix_f32(x, [dict(gain0=0.75)], L, M, threads=4)
    assert bits_equal(ys, O.sat16(np.rint(ref.astype(np.float32) * np.float32(32768.0))).astype(np.int16))


def test_u2_stereo_one_track_multi_sp(xm, gpu, monkeypatch):
    monkeypatch.setenv("XM_FAST_SPLIT_R", "3")
    N, B = SPI * (8 * 3 * 5 // 2 + 3) + 37, 11
    x = _x(B, 1, N, 57000)
    ramps = _ramps(2, _F(N))[1:2]
    m = xm.Mixer(44100, 96000, 2, "f32")
    m.set_tracks(ramps)
    y = m.process(x)
    _fast(m)
    assert xm.last_fast_split()[0] == 3
    assert bits_equal(y, CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)[0])


def test_u2_mono_s16_stays_generic(xm, gpu):
    """Mono s16 tracks at 320/147 have no fused instantiation: the generic
    kernel, with the same bits as the oracle."""
    N, B = 9 * SPI + 3, 3
    x = np.stack([np.stack([O.gen_s16(SEED, 58000 + 16 * b, 1, N)]) for b in range(B)])
    q = [dict(gain0_q15=29491)]
    m = xm.Mixer(44100, 96000, 1, "s16")
    m.set_tracks(q)
    y = m.process(x)
    _fast(m, 0)
    for b in range(B):
        assert bits_equal(y[b], CO.resample_mix_s16(list(x[b]), q, L, M)), b
