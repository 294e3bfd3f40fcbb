"""Multi-super-period lanes for every fused instantiation added in round 4
(VERDICT r4 item 1).

Small batches make pick_split choose R = 1 (one super-period per lane), so
they never cross from one SP to the next inside a lane: the register carry,
the previous SP's last round stored in the next one, and the next SP's
segment-2 DMA issued during this one (the round-4 bug at 2/1 and 3/1, found
only at the production shape).  Here XM_FAST_SPLIT_R forces R >= 2 (mono:
>= 2 SPs per plane, R >= 4) on small batches whose clips end inside a lane's
run, every output of every mix is compared with the C oracle bit for bit, and
each case asserts it ran as one fused launch with the R it asked for
(xm_audio_mixer_last_fast_split).  One production-grid case (512 mixes x 8
stereo s16 tracks x 10 s at 3/2) runs with the split pick_split chooses.
"""
import numpy as np
import pytest

from conftest import bits_equal

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED

# (in rate, out rate, L, M, input frames per super-period)
SMALL = [(32000, 48000, 3, 2, 160), (48000, 32000, 2, 3, 159), (96000, 48000, 1, 2, 160)]
SMALL_IDS = ["3_2", "2_3", "1_2"]
UP = [(24000, 48000, 2, 1, 160), (16000, 48000, 3, 1, 160)]
TABLE = [(48000, 44100, 147, 160, 160), (44100, 48000, 160, 147, 147)]


def _F(N, L, M):
    return (N * L + M - 1) // M


def _q15(nt, F):
    return [dict(gain0_q15=29491 - 1000 * t, gain1_q15=3000 * t, ramp_start=173 * t, ramp_len=max(1, F // 3))
            for t in range(nt)]


def _ramps(nt, F):
    base = [dict(gain0=0.9), dict(gain0=0.0, gain1=0.8, ramp_start=41, ramp_len=max(1, F // 3)),
            dict(mode=1, ramp_start=F // 4, ramp_len=max(1, F // 5)), dict(gain0=0.3, gain1=0.6, ramp_start=F // 2),
            dict(gain0=1.25, gain1=0.5, ramp_start=0, ramp_len=max(1, F)),
            dict(gain0=0.5, gain1=0.0, ramp_start=max(0, F - 900), ramp_len=800)]
    return [base[t % 6] for t in range(nt)]


def _frames(SPI, R, lanes_per_run=8, odd=1):
    """~2.5 runs of 8 lanes x R SPs per clip: three tasks per mix, the last
    one partial, the clip end inside a lane's run (odd: an odd frame count)."""
    return SPI * (lanes_per_run * R * 5 // 2 + 3) + 36 + odd


@pytest.fixture
def split(monkeypatch):
    def _set(R):
        monkeypatch.setenv("XM_FAST_SPLIT_R", str(R))
    return _set


def _ran(xm, m, R):
    t = m.timing()
    assert t.n_launches == 1 and t.fast_launches == 1, (t.n_launches, t.fast_launches)
    got = xm.last_fast_split()
    assert got is not None and got[0] == R, (got, R)
    return got


@pytest.mark.parametrize("ratio", SMALL, ids=SMALL_IDS)
@pytest.mark.parametrize("nt", [4, 8])
@pytest.mark.parametrize("R", [2, 3])
def test_stereo_s16_multi_sp(xm, gpu, split, ratio, nt, R):
    """Stereo s16 tracks at 3/2, 2/3, 1/2: the s16 Q15 mix and s16 tracks into
    the f32 mix (IN_CONVERT), lanes walking R SPs."""
    fi, fo, L, M, SPI = ratio
    split(R)
    for odd in (0, 1):
        N = _frames(SPI, R, odd=odd)
        B = 3
        xs = np.stack([np.stack([O.gen_s16(SEED, 40000 + N + 16 * b + t, 2, N) for t in range(nt)]) for b in range(B)])
        xs[:, :2, 1000:1400] = 32767    # saturating terms cross a round
        F = _F(N, L, M)
        q = _q15(nt, F)
        m = xm.Mixer(fi, fo, 2, "s16")
        m.set_tracks(q)
        y = m.process(xs)
        _, tpm = _ran(xm, m, R)
        assert tpm >= 2
        for b in range(B):
            assert bits_equal(y[b], CO.resample_mix_s16(list(xs[b]), q, L, M)), (N, b)
        ramps = _ramps(nt, F)
        c = xm.Mixer(fi, fo, 2, "f32", convert_in=True)
        c.set_tracks(ramps)
        yc = c.process(xs)
        _ran(xm, c, R)
        xf = xs.astype(np.float32) * np.float32(2.0 ** -15)
        assert bits_equal(yc, CO.batch_resample_mix_f32(xf, ramps, L, M, threads=4)[0]), N


@pytest.mark.parametrize("ratio", SMALL, ids=SMALL_IDS)
@pytest.mark.parametrize("nt", [1, 3, 8])
@pytest.mark.parametrize("R", [4, 6])
def test_mono_f32_multi_sp(xm, gpu, split, ratio, nt, R):
    """Mono f32 tracks at the small ratios with 2 or 3 SPs per plane (the two
    halves of a run ride as the planar pair), odd and even N."""
    fi, fo, L, M, SPI = ratio
    if (L, M, nt) == (3, 2, 1):
        pytest.skip("3/2 one-track mono rows run on the generic kernel (xmg_fast_kern_mono_r32)")
    split(R)
    for odd in (0, 1):
        N = _frames(SPI, R, odd=odd)
        B = 11 if nt == 1 else 3
        x = np.stack([np.stack([O.gen_f32(SEED, 41000 + N + 16 * b + t, 1, N) for t in range(nt)]) for b in range(B)])
        ramps = _ramps(nt, _F(N, L, M))
        m = xm.Mixer(fi, fo, 1, "f32")
        m.set_tracks(ramps)
        y = m.process(x)
        _ran(xm, m, R)
        assert bits_equal(y, CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)[0]), N


@pytest.mark.parametrize("ratio", SMALL + TABLE, ids=SMALL_IDS + ["48_44", "44_48"])
@pytest.mark.parametrize("nt", [1, 5])
def test_mono_s16_q15_multi_sp(xm, gpu, split, ratio, nt):
    """Mono s16 tracks into the Q15 mix (M16) with 2 SP pairs per plane, at
    the small and the table ratios (dword-aligned N: the fused kernel)."""
    fi, fo, L, M, SPI = ratio
    if (L, M, nt) == (3, 2, 1):
        pytest.skip("3/2 one-track mono rows run on the generic kernel")
    R = 8
    split(R)
    N = _frames(SPI, R, odd=0) + 1   # even
    N += N & 1
    B = 11 if nt == 1 else 3
    x = np.stack([np.stack([O.gen_s16(SEED, 42000 + N + 16 * b + t, 1, N) for t in range(nt)]) for b in range(B)])
    q = _q15(nt, _F(N, L, M))
    m = xm.Mixer(fi, fo, 1, "s16")
    m.set_tracks(q)
    y = m.process(x)
    _ran(xm, m, R)
    for b in range(B):
        assert bits_equal(y[b], CO.resample_mix_s16(list(x[b]), q, L, M)), b


@pytest.mark.parametrize("ratio", UP, ids=["2_1", "3_1"])
@pytest.mark.parametrize("nt", [2, 8])
@pytest.mark.parametrize("R", [2, 3])
def test_up_small_multi_sp(xm, gpu, split, ratio, nt, R):
    """2/1 and 3/1 stereo f32 mixes (320 and 480 outputs per SP) with lanes
    walking R SPs, odd and even N."""
    fi, fo, L, M, SPI = ratio
    split(R)
    for odd in (0, 1):
        N = _frames(SPI, R, odd=odd)
        B = 3
        x = np.stack([np.stack([O.gen_f32(SEED, 43000 + N + 16 * b + t, 2, N) for t in range(nt)]) for b in range(B)])
        ramps = _ramps(nt, _F(N, L, M))
        m = xm.Mixer(fi, fo, 2, "f32")
        m.set_tracks(ramps)
        y = m.process(x)
        _ran(xm, m, R)
        assert bits_equal(y, CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)[0]), N


@pytest.mark.parametrize("ratio", SMALL + TABLE, ids=SMALL_IDS + ["48_44", "44_48"])
@pytest.mark.parametrize("nt", [1, 2, 8])
def test_stereo_f32_multi_sp(xm, gpu, split, ratio, nt):
    """Stereo f32 rows of 1, 2 and 8 tracks with lanes walking 3 SPs."""
    fi, fo, L, M, SPI = ratio
    R = 3
    split(R)
    N = _frames(SPI, R)
    B = 9 if nt < 8 else 3
    x = np.stack([np.stack([O.gen_f32(SEED, 44000 + N + 16 * b + t, 2, N) for t in range(nt)]) for b in range(B)])
    ramps = _ramps(nt, _F(N, L, M))
    m = xm.Mixer(fi, fo, 2, "f32")
    m.set_tracks(ramps)
    y = m.process(x)
    _ran(xm, m, R)
    assert bits_equal(y, CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)[0])


def test_stereo_s16_production_grid_32_48(xm, gpu):
    """Stereo s16 Q15 mix at 3/2 on the bench grid (512 mixes x 8 tracks x
    10 s at 32 kHz), the split pick_split chooses (R >= 2): first and last
    mix bit-checked, nothing left unwritten."""
    import torch
    B, nt, N = 512, 8, 320000
    L, M = 3, 2
    F = _F(N, L, M)
    q = _q15(nt, F)
    m = xm.Mixer(32000, 48000, 2, "s16", mem="device")
    m.set_tracks(q)
    assert m.out_frames(N) == F
    x = torch.empty((B * nt, N, 2), dtype=torch.int16, device="cuda")
    y = torch.full((B, F, 2), -32768, dtype=torch.int16, device="cuda")
    xm.synth(x.data_ptr(), "s16", SEED, 0, B * nt, 2, N)
    torch.cuda.synchronize()
    m.process_strided(x.data_ptr(), N * 2, N * 2 * nt, y.data_ptr(), F * 2, B, N)
    torch.cuda.synchronize()
    t = m.timing()
    assert t.n_launches == 1 and t.fast_launches == 1
    R, tpm = xm.last_fast_split()
    assert R >= 2, (R, tpm)
    for b in (0, B - 1):
        xb = x[b * nt:(b + 1) * nt].cpu().numpy()
        assert bits_equal(y[b].cpu().numpy(), CO.resample_mix_s16(list(xb), q, L, M)), b
    # nothing unwritten: a second call over an output filled with another
    # value must give the same bits everywhere (saturated mixes make any one
    # sentinel a legal output)
    y2 = torch.full((B, F, 2), 32767, dtype=torch.int16, device="cuda")
    m.process_strided(x.data_ptr(), N * 2, N * 2 * nt, y2.data_ptr(), F * 2, B, N)
    torch.cuda.synchronize()
    assert bool(torch.equal(y, y2)), "unwritten output frames"
    del x, y, y2
    torch.cuda.empty_cache()
