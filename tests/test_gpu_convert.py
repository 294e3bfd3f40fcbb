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
