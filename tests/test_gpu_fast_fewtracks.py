"""Stereo s16 and planar mixes of fewer than 4 tracks on the fused kernel
(round 5; VERDICT r4 "missing" item 4).

The stereo s16 and planar instantiations have 8-track rows only; a mix of
fewer tracks leaves phantom rows (out-of-range loads, zero gains, terms of
+-0 or 0).  The launcher sends the Q15 mix from 3 tracks and the planar and
s16-into-f32 mixes from 2 to the fused kernel, where they measured faster
than the generic kernel (profiles/r5_q_io_tracks.txt); fewer stay generic.
Every case asserts which kernel ran and equals the C oracle bit for bit:
full-scale samples (every saturation stage), odd and short lengths, the
table and small ratios, lanes walking several super-periods."""
import numpy as np
import pytest

from conftest import bits_equal

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED

Q15 = [dict(gain0_q15=29491), dict(gain0_q15=0, gain1_q15=26214, ramp_start=0, ramp_len=4800),
       dict(mode=1, ramp_start=2000, ramp_len=3000)]
RAMPS = [dict(gain0=0.9), dict(gain0=0.0, gain1=0.8, ramp_start=41, ramp_len=3000),
         dict(mode=1, ramp_start=1200, ramp_len=2500)]
# (in rate, out rate, L, M)
RATES = [(48000, 44100, 147, 160), (44100, 48000, 160, 147), (32000, 48000, 3, 2), (96000, 48000, 1, 2)]
IDS = ["48_44", "44_48", "32_48", "96_48"]


def _fast(m, want):
    t = m.timing()
    assert t.n_launches == 1 and t.fast_launches == want, (t.n_launches, t.fast_launches, want)


def _planar(a):
    return np.ascontiguousarray(np.swapaxes(a, -1, -2))


@pytest.mark.parametrize("rates", RATES, ids=IDS)
@pytest.mark.parametrize("nt", [1, 2, 3])
@pytest.mark.parametrize("N", [48000, 48001, 160 * 7 + 5])
def test_few_tracks_q15_mix(xm, gpu, rates, nt, N):
    fi, fo, L, M = rates
    B = 3
    x = np.stack([np.stack([O.gen_s16(SEED, 8100 + N % 97 + 8 * b + t, 2, N) for t in range(nt)]) for b in range(B)])
    x[:, :, 300:340] = 32767
    x[:, nt - 1:, 700:720] = -32768
    m = xm.Mixer(fi, fo, 2, "s16")
    m.set_tracks(Q15[:nt])
    y = m.process(x)
    _fast(m, 1 if nt >= 3 else 0)
    for b in range(B):
        assert bits_equal(y[b], CO.resample_mix_s16(list(x[b]), Q15[:nt], L, M)), b


@pytest.mark.parametrize("rates", RATES, ids=IDS)
@pytest.mark.parametrize("nt", [1, 2, 3])
def test_few_tracks_s16_into_f32_mix(xm, gpu, rates, nt):
    fi, fo, L, M = rates
    B, N = 3, 48003
    x = np.stack([np.stack([O.gen_s16(SEED, 8200 + 8 * b + t, 2, N) for t in range(nt)]) for b in range(B)])
    x[:, :, 300:340] = 32767
    m = xm.Mixer(fi, fo, 2, "f32", convert_in=True)
    m.set_tracks(RAMPS[:nt])
    y = m.process(x)
    _fast(m, 1 if nt >= 2 else 0)
    xf = x.astype(np.float32) * np.float32(2.0 ** -15)
    assert bits_equal(y, CO.batch_resample_mix_f32(xf, RAMPS[:nt], L, M, threads=4)[0])


@pytest.mark.parametrize("nt", [1, 2, 3])
@pytest.mark.parametrize("N", [48000, 48001])
def test_few_tracks_planar(xm, gpu, nt, N):
    B = 3
    x = np.stack([np.stack([O.gen_f32(SEED, 8300 + 8 * b + t, 2, N) for t in range(nt)]) for b in range(B)])
    m = xm.Mixer(48000, 44100, 2, "f32", planar=True)
    m.set_tracks(RAMPS[:nt])
    y = m.process(_planar(x))
    _fast(m, 1 if nt >= 2 else 0)
    ref, _ = CO.batch_resample_mix_f32(x, RAMPS[:nt], 147, 160, threads=4)
    assert bits_equal(y, _planar(ref))


@pytest.mark.parametrize("nt", [2, 3])
def test_few_tracks_multi_sp(xm, gpu, monkeypatch, nt):
    """Lanes walking 3 super-periods with phantom rows (the carry, the next
    SP's DMA), Q15 (3 tracks) and s16-into-f32 (2 and 3 tracks)."""
    monkeypatch.setenv("XM_FAST_SPLIT_R", "3")
    N = 160 * (8 * 3 * 5 // 2 + 3) + 37
    B = 3
    x = np.stack([np.stack([O.gen_s16(SEED, 8400 + 8 * b + t, 2, N) for t in range(nt)]) for b in range(B)])
    x[:, :, 1000:1400] = 32767
    c = xm.Mixer(48000, 44100, 2, "f32", convert_in=True)
    c.set_tracks(RAMPS[:nt])
    yc = c.process(x)
    _fast(c, 1)
    assert xm.last_fast_split()[0] == 3
    xf = x.astype(np.float32) * np.float32(2.0 ** -15)
    assert bits_equal(yc, CO.batch_resample_mix_f32(xf, RAMPS[:nt], 147, 160, threads=4)[0])
    if nt == 3:
        m = xm.Mixer(48000, 44100, 2, "s16")
        m.set_tracks(Q15)
        y = m.process(x)
        _fast(m, 1)
        for b in range(B):
            assert bits_equal(y[b], CO.resample_mix_s16(list(x[b]), Q15, 147, 160)), b
