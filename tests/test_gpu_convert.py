"""GPU parity of the output-format epilogues (XM_MIXER_OUT_CONVERT, SURVEY.md
§8(f) item 4): an F32 mixer writing s16 = sat16(rint(y * 32768)) and an S16
mixer writing f32 = y * 2^-15, against the oracle's mix converted in numpy
(np.rint is ties-to-even, as the kernels' v_rndne_f32)."""
import numpy as np
import pytest

from conftest import bits_equal

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED

RAMPS = [dict(gain0=0.9), dict(gain0=0.0, gain1=1.2, ramp_start=100, ramp_len=3000),
         dict(gain0=1.5, gain1=0.2, ramp_start=2000, ramp_len=441), dict(mode=1, ramp_start=3000, ramp_len=800)]


def _to_s16(y):
    return np.clip(np.rint(y.astype(np.float32) * np.float32(32768.0)), -32768, 32767).astype(np.int16)


@pytest.mark.parametrize("rates", [(48000, 44100), (48000, 48000)])
def test_f32_mix_to_s16_out(xm, gpu, rates):
    fi, fo = rates
    N = 9600 + 7
    x = np.stack([np.stack([O.gen_f32(SEED, 5000 + 4 * b + t, 2, N) for t in range(4)]) for b in range(2)])
    x[:, :, 100:140] = 0.99   # drive the sum past full scale: saturation
    m = xm.Mixer(fi, fo, 2, "f32", convert_out=True)
    m.set_tracks(RAMPS)
    y = m.process(x)
    assert y.dtype == np.int16
    for b in range(2):
        ref = (CO.resample_mix_f32(list(x[b]), RAMPS, 147, 160) if fi != fo else CO.mix_f32(list(x[b]), RAMPS))
        assert bits_equal(y[b], _to_s16(ref)), b
    # the streamed form converts the same way
    m.stream_begin(2)
    ys = np.concatenate([m.stream_push(x[:, :, :5000]), m.stream_push(x[:, :, 5000:]), m.stream_flush()], axis=1)
    assert bits_equal(ys, y)


@pytest.mark.parametrize("rates", [(44100, 48000), (48000, 48000)])
def test_s16_mix_to_f32_out(xm, gpu, rates):
    fi, fo = rates
    N = 8820 + 5
    ramps = [dict(r, gain0_q15=int(round(r.get("gain0", 1.0) * 32768)),
                  gain1_q15=int(round(r.get("gain1", r.get("gain0", 1.0)) * 32768))) for r in RAMPS]
    x = np.stack([np.stack([O.gen_s16(SEED, 5100 + 4 * b + t, 1, N) for t in range(4)]) for b in range(2)])
    m = xm.Mixer(fi, fo, 1, "s16", convert_out=True)
    m.set_tracks(ramps)
    y = m.process(x)
    assert y.dtype == np.float32
    for b in range(2):
        ref = (CO.resample_mix_s16(list(x[b]), ramps, 160, 147) if fi != fo else CO.mix_s16(list(x[b]), ramps))
        assert bits_equal(y[b], ref.astype(np.float32) * np.float32(2.0 ** -15)), b


def test_convert_with_track_effects_and_timeline(xm, gpu):
    x = np.stack([O.gen_f32(SEED, 5200 + t, 2, 4800) for t in range(2)])[None]
    ramps = [dict(gain0=0.7), dict(gain0=0.6)]
    e = xm.Effects(44100, 2)
    e.add_eq_band(0, 1000.0, 6.0, 1.0)
    m = xm.Mixer(48000, 44100, 2, "f32", convert_out=True)
    m.set_tracks(ramps)
    m.set_track_effects(e)
    y = m.process(x)[0]
    sos = e.biquad(0)[None]
    r = [CO.biquad_f32(CO.resample_f32(t, 147, 160), sos) for t in x[0]]
    assert bits_equal(y, _to_s16(CO.mix_f32(r, ramps)))
    m.set_track_effects(None)
    t = m.process_timeline([x[:, 0], x[:, 1]], [0, 100], 4500)[0]
    pl = np.zeros((2, 4500, 2), np.float32)
    r0, r1 = CO.resample_f32(x[0, 0], 147, 160), CO.resample_f32(x[0, 1], 147, 160)
    pl[0, :len(r0)] = r0[:4500]
    pl[1, 100:100 + len(r1)] = r1[:4400]
    assert bits_equal(t, _to_s16(CO.mix_f32(list(pl), ramps)))


# ---- input side (XM_MIXER_IN_CONVERT) and planar layouts (XM_MIXER_PLANAR) ----
def _q15(ramps):
    return [dict(r, gain0_q15=int(round(r.get("gain0", 1.0) * 32768)),
                 gain1_q15=int(round(r.get("gain1", r.get("gain0", 1.0)) * 32768))) for r in ramps]


def _planar(a):
    """[..., frames, channels] -> [..., channels, frames]"""
    return np.ascontiguousarray(np.swapaxes(a, -1, -2))


@pytest.mark.parametrize("rates", [(48000, 44100), (48000, 48000)])
@pytest.mark.parametrize("planar", [False, True])
@pytest.mark.parametrize("convert_out", [False, True])
def test_s16_tracks_into_f32_mix(xm, gpu, rates, planar, convert_out):
    """F32 mixer reading s16 tracks: each sample x * 2^-15 (exact) at load,
    then the f32 path; planar tracks and mixes read and written in place."""
    fi, fo = rates
    N, B = 9600 + 7, 3
    x = np.stack([np.stack([O.gen_s16(SEED, 5300 + 4 * b + t, 2, N) for t in range(4)]) for b in range(B)])
    m = xm.Mixer(fi, fo, 2, "f32", convert_in=True, planar=planar, convert_out=convert_out)
    m.set_tracks(RAMPS)
    y = m.process(_planar(x) if planar else x)
    assert y.dtype == (np.int16 if convert_out else np.float32)
    # 4-track 48k->44.1k interleaved mixes run on the fused kernel's 8-row
    # s16 layout (phantom rows); planar s16 tracks, and 48k->48k, do not
    assert m.timing().fast_launches == (1 if fi != fo and not planar else 0)
    xf = x.astype(np.float32) * np.float32(2.0 ** -15)
    for b in range(B):
        ref = CO.resample_mix_f32(list(xf[b]), RAMPS, 147, 160) if fi != fo else CO.mix_f32(list(xf[b]), RAMPS)
        if convert_out:
            ref = _to_s16(ref)
        assert bits_equal(_planar(y[b]) if planar else y[b], ref), b


@pytest.mark.parametrize("rates", [(44100, 48000), (48000, 48000)])
@pytest.mark.parametrize("planar", [False, True])
def test_f32_tracks_into_s16_mix(xm, gpu, rates, planar):
    """S16 mixer reading f32 tracks: sat16(rint(x * 32768)) at load (full
    scale and beyond saturate), then the Q15 path."""
    fi, fo = rates
    N, B = 8820 + 5, 2
    x = np.stack([np.stack([O.gen_f32(SEED, 5400 + 4 * b + t, 2, N) for t in range(4)]) for b in range(B)])
    x[:, 1, 50:80] = 1.5
    x[:, 2, 90:95] = -1.25
    ramps = _q15(RAMPS)
    m = xm.Mixer(fi, fo, 2, "s16", convert_in=True, planar=planar)
    m.set_tracks(ramps)
    y = m.process(_planar(x) if planar else x)
    assert y.dtype == np.int16
    xq = _to_s16(x)
    for b in range(B):
        ref = CO.resample_mix_s16(list(xq[b]), ramps, 160, 147) if fi != fo else CO.mix_s16(list(xq[b]), ramps)
        assert bits_equal(_planar(y[b]) if planar else y[b], ref), b


def test_planar_f32_headline_shape_and_effects(xm, gpu):
    """Planar stereo through the 48k->44.1k generic path with per-track
    effects (the resample stage reads the planar tracks, the final mix writes
    the planar mixes), and mono planar == interleaved (fast path kept)."""
    N, B = 4800 + 3, 2
    x = np.stack([np.stack([O.gen_f32(SEED, 5500 + 4 * b + t, 2, N) for t in range(4)]) for b in range(B)])
    e = xm.Effects(44100, 2)
    e.add_eq_band(0, 1000.0, 6.0, 1.0)
    e.add_eq_band(0, 3000.0, -4.0, 0.7)
    m = xm.Mixer(48000, 44100, 2, "f32", planar=True)
    m.set_tracks(RAMPS)
    m.set_track_effects(e)
    y = m.process(_planar(x))
    sos = np.stack([e.biquad(0), e.biquad(1)])
    for b in range(B):
        ref = CO.mix_f32([CO.biquad_f32(CO.resample_f32(t, 147, 160), sos) for t in x[b]], RAMPS)
        assert bits_equal(_planar(y[b]), ref), b
    # mono: planar is interleaved; the handle keeps every path
    xm1 = np.stack([np.stack([O.gen_f32(SEED, 5600 + t, 1, N) for t in range(4)])])
    m1 = xm.Mixer(48000, 48000, 1, "f32", planar=True)
    m1.set_tracks(RAMPS)
    assert bits_equal(m1.process(_planar(xm1))[0], _planar(CO.mix_f32(list(xm1[0]), RAMPS)))


def test_in_convert_device_strided(xm, gpu):
    """Device memory: strides count elements of the input format (s16 here,
    for an f32 mixer), mixes in a padded strided layout."""
    import torch
    N, B, ntr = 4410 + 1, 3, 4
    x = np.stack([np.stack([O.gen_s16(SEED, 5700 + 4 * b + t, 2, N) for t in range(ntr)]) for b in range(B)])
    ts, ms = N * 2 + 6, (N * 2 + 6) * ntr + 10
    buf = np.zeros(B * ms, np.int16)
    for b in range(B):
        for t in range(ntr):
            buf[b * ms + t * ts: b * ms + t * ts + 2 * N] = x[b, t].reshape(-1)
    m = xm.Mixer(44100, 48000, 2, "f32", mem="device", convert_in=True)
    m.set_tracks(RAMPS)
    F = m.out_frames(N)
    xd = torch.from_numpy(buf).cuda()
    yd = torch.zeros((B, F * 2 + 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    m.process_strided(xd.data_ptr(), ts, ms, yd.data_ptr(), F * 2 + 4, B, N)
    torch.cuda.synchronize()
    y = yd.cpu().numpy()[:, :2 * F].reshape(B, F, 2)
    xf = x.astype(np.float32) * np.float32(2.0 ** -15)
    for b in range(B):
        assert bits_equal(y[b], CO.resample_mix_f32(list(xf[b]), RAMPS, 160, 147)), b


def test_in_convert_planar_unsupported_calls(xm, gpu):
    """Streaming, timeline and config-5 calls refuse the layout / input flags."""
    m = xm.Mixer(48000, 44100, 2, "f32", convert_in=True)
    m.set_tracks(RAMPS)
    with pytest.raises(xm.XmError):
        m.stream_begin(1)
    p = xm.Mixer(48000, 48000, 2, "f32", planar=True)
    p.set_tracks(RAMPS[:2])
    with pytest.raises(xm.XmError):
        p.process_timeline([np.zeros((1, 10, 2), np.float32)] * 2, [0, 5], 20)
