"""Stereo s16 tracks on the fused kernel at 2/1, 3/1 and 320/147 (round 6,
VERDICT r5 item 7): 24k, 16k, 22.05k -> 48k and 44.1k ->
96k with s16 tracks (voice tracks are s16) into the s16 Q15 mix (3-8
tracks) or into the f32 mix (XM_MIXER_IN_CONVERT, 2-8 tracks), the 8-row IO
instantiations the small ratios 3/2, 2/3, 1/2 already had.  Every case must
be one fused launch and equal the C oracle bit for bit: track counts
(phantom rows), odd and even N, lengths around super-period edges, lanes
walking several super-periods (XM_FAST_SPLIT_R), Q15 ramps and saturation,
the bench-sized grid.  Against scipy directly: tests/test_gpu_golden_fused.py
(resample_fused.npz holds s16 clips at each of these ratios)."""
import numpy as np
import pytest

from conftest import bits_equal

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED
# (in rate, out rate, L, M, SPI: input frames per super-period)
RATIOS = [(24000, 48000, 2, 1, 160), (16000, 48000, 3, 1, 160), (22050, 48000, 320, 147, 147),
          (44100, 96000, 320, 147, 147)]
IDS = ["2_1", "3_1", "22_48", "44_96"]


def _F(N, L, M):
    return (N * L + M - 1) // M


def _q15(nt, F):
    base = [dict(gain0_q15=29491), dict(gain0_q15=0, gain1_q15=32768, ramp_start=31, ramp_len=max(1, F // 3)),
            dict(mode=1, ramp_start=F // 4, ramp_len=max(1, F // 5)), dict(gain0_q15=65535, gain1_q15=3, ramp_start=F // 2),
            dict(gain0_q15=40000, gain1_q15=9000, ramp_start=0, ramp_len=max(1, F)),
            dict(gain0_q15=16384), dict(gain0_q15=0, gain1_q15=26214, ramp_start=max(0, F - 700), ramp_len=600),
            dict(gain0_q15=7, gain1_q15=60000, ramp_start=F // 3, ramp_len=0)]
    return [base[t % 8] for t in range(nt)]


def _ramps(nt, F):
    base = [dict(gain0=0.9), dict(gain0=0.0, gain1=0.8, ramp_start=41, ramp_len=max(1, F // 3)),
            dict(mode=1, ramp_start=F // 4, ramp_len=max(1, F // 5)), dict(gain0=0.3, gain1=0.6, ramp_start=F // 2),
            dict(gain0=1.25, gain1=0.5, ramp_start=0, ramp_len=max(1, F)),
            dict(gain0=0.5, gain1=0.0, ramp_start=max(0, F - 900), ramp_len=800)]
    return [base[t % 6] for t in range(nt)]


def _xs(B, nt, N, base, loud=False):
    x = np.stack([np.stack([O.gen_s16(SEED, base + 16 * b + t, 2, N) for t in range(nt)]) for b in range(B)])
    if loud:   # full-scale runs: the resampled tracks and the Q15 sum saturate
        x[:, :2, N // 3:N // 3 + 200] = 32767
        x[:, -1:, N // 2:N // 2 + 150] = -32768
    return x


def _fast(m):
    t = m.timing()
    assert t.n_launches == 1 and t.fast_launches == 1, (t.n_launches, t.fast_launches)


@pytest.mark.parametrize("ratio", RATIOS, ids=IDS)
@pytest.mark.parametrize("nt", [3, 5, 8])
def test_s16_ups_q15_mix(xm, gpu, ratio, nt):
    fi, fo, L, M, SPI = ratio
    for N in (20 * SPI + 37, 20 * SPI + 38, SPI - 1, SPI + 1, 2 * SPI, 7):
        B = 3
        x = _xs(B, nt, N, 60000 + N + nt, loud=N > SPI)
        q = _q15(nt, _F(N, L, M))
        m = xm.Mixer(fi, fo, 2, "s16")
        m.set_tracks(q)
        y = m.process(x)
        _fast(m)
        for b in range(B):
            assert bits_equal(y[b], CO.resample_mix_s16(list(x[b]), q, L, M)), (N, b)


@pytest.mark.parametrize("ratio", RATIOS, ids=IDS)
@pytest.mark.parametrize("nt", [2, 4, 8])
def test_s16_ups_into_f32_mix(xm, gpu, ratio, nt):
    """s16 tracks into the f32 mix: x * 2^-15 exactly, then the f32 path."""
    fi, fo, L, M, SPI = ratio
    for N in (20 * SPI + 37, 20 * SPI + 38, SPI + 1, 3):
        B = 2
        x = _xs(B, nt, N, 61000 + N + nt)
        ramps = _ramps(nt, _F(N, L, M))
        m = xm.Mixer(fi, fo, 2, "f32", convert_in=True)
        m.set_tracks(ramps)
        y = m.process(x)
        _fast(m)
        xf = x.astype(np.float32) * np.float32(2.0 ** -15)
        assert bits_equal(y, CO.batch_resample_mix_f32(xf, ramps, L, M, threads=4)[0]), N


@pytest.mark.parametrize("ratio", RATIOS, ids=IDS)
def test_s16_ups_multi_sp(xm, gpu, ratio, monkeypatch):
    """Every lane walking 2 and 5 super-periods."""
    fi, fo, L, M, SPI = ratio
    N, nt, B = 60 * SPI + 11, 6, 2
    x = _xs(B, nt, N, 62000, loud=True)
    q = _q15(nt, _F(N, L, M))
    for R in (2, 5):
        monkeypatch.setenv("XM_FAST_SPLIT_R", str(R))
        m = xm.Mixer(fi, fo, 2, "s16")
        m.set_tracks(q)
        y = m.process(x)
        _fast(m)
        assert xm.last_fast_split()[0] == R
        for b in range(B):
            assert bits_equal(y[b], CO.resample_mix_s16(list(x[b]), q, L, M)), (R, b)


@pytest.mark.parametrize("ratio", RATIOS, ids=IDS)
def test_s16_ups_device_strides_and_tables(xm, gpu, ratio):
    """Padded strides in device memory and a scattered pointer table."""
    import torch
    fi, fo, L, M, SPI = ratio
    nt, N, B = 5, 9 * SPI + 3, 4
    x = _xs(B, nt, N, 63000)
    q = _q15(nt, _F(N, L, M))
    ref = np.stack([CO.resample_mix_s16(list(x[b]), q, L, M) for b in range(B)])
    m = xm.Mixer(fi, fo, 2, "s16", mem="device")
    m.set_tracks(q)
    F = m.out_frames(N)
    ts, ms = N + 5, (N + 5) * nt + 3          # frames
    buf = np.zeros((B * ms + 8, 2), np.int16)
    for b in range(B):
        for t in range(nt):
            buf[b * ms + t * ts: b * ms + t * ts + N] = x[b, t]
    xd = torch.from_numpy(buf).cuda()
    yd = torch.full((B, F + 2, 2), -9, dtype=torch.int16, device="cuda")
    m.process_strided(xd.data_ptr(), ts * 2, ms * 2, yd.data_ptr(), (F + 2) * 2, B, N)
    torch.cuda.synchronize()
    _fast(m)
    assert bits_equal(yd.cpu().numpy()[:, :F], ref)
    assert (yd.cpu().numpy()[:, F:] == -9).all(), "no store past the mix"
    # the same tracks through a pointer table in reverse track order
    perm = list(range(nt))[::-1]
    ins = [xd[b * ms + perm[t] * ts:].data_ptr() for b in range(B) for t in range(nt)]
    yt = torch.zeros((B, F, 2), dtype=torch.int16, device="cuda")
    m.process_ptrs(ins, [yt[b].data_ptr() for b in range(B)], B, N)
    torch.cuda.synchronize()
    _fast(m)
    for b in range(B):
        assert bits_equal(yt[b].cpu().numpy(), CO.resample_mix_s16([x[b, p] for p in perm], q, L, M)), b


@pytest.mark.parametrize("ratio", RATIOS[:3], ids=IDS[:3])
def test_s16_ups_production_grid(xm, gpu, ratio):
    """512 mixes x 8 s16 tracks x 10 s at the input rate (the bench shape):
    first and last mix against the oracle."""
    import torch
    fi, fo, L, M, SPI = ratio
    B, nt, N = 512, 8, 10 * fi
    m = xm.Mixer(fi, fo, 2, "s16", mem="device")
    F = m.out_frames(N)
    q = _q15(nt, F)
    m.set_tracks(q)
    x = torch.empty((B, nt, N, 2), dtype=torch.int16, device="cuda")
    xm.synth(x.data_ptr(), "s16", SEED, 0, B * nt, 2, N, 0)
    y = torch.empty((B, F, 2), dtype=torch.int16, device="cuda")
    m.process_strided(x.data_ptr(), N * 2, nt * N * 2, y.data_ptr(), F * 2, B, N)
    torch.cuda.synchronize()
    _fast(m)
    for b in (0, B - 1):
        xb = x[b].cpu().numpy()
        assert bits_equal(y[b].cpu().numpy(), CO.resample_mix_s16(list(xb), q, L, M)), b
    del x, y
    torch.cuda.empty_cache()
