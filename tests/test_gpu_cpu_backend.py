"""GPU box: the two backends of the library agree bit for bit at production
clip lengths.  Each case runs the same C API call once on a GPU handle (the
gfx950 kernels: the fused kernel where its shape applies) and once on a CPU
handle (n_devices = 0, src/cpu/), and compares every output sample; the
first mix is also checked against the C oracle, which pins both to scipy.
"""
import numpy as np
import pytest

from conftest import bits_equal

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED

RAMPS = [dict(gain0=0.9), dict(gain0=0.0, gain1=0.8, ramp_start=0, ramp_len=44100),
         dict(gain0=0.7, gain1=0.2, ramp_start=220500, ramp_len=88200), dict(gain0=0.5),
         dict(mode=1, ramp_start=132300, ramp_len=88200), dict(gain0=0.0, gain1=1.0, ramp_start=132300, ramp_len=88200),
         dict(gain0=1.0, gain1=0.0, ramp_start=396900, ramp_len=44100), dict(gain0=0.3, gain1=0.6, ramp_start=300000)]


def _both(xm, args, kw, x, ramps=None, fx=None):
    ys = []
    for dev in (0, "cpu"):
        m = xm.Mixer(*args, device=dev, **kw)
        if ramps:
            m.set_tracks(ramps)
        if fx is not None:
            e = xm.Effects(args[1], args[2], device=dev)
            for s in fx:
                e.add_biquad(s)
            m.set_track_effects(e)
        ys.append(m.process(x))
    return ys


def test_headline_10s_gpu_equals_cpu(xm, gpu):
    """48k->44.1k + 8 ramped tracks, 10 s stereo: fused kernel vs CPU backend."""
    x = np.stack([np.stack([O.gen_f32(SEED, 64 * b + t, 2, 480000) for t in range(8)]) for b in range(3)])
    g, c = _both(xm, (48000, 44100, 2, "f32"), {}, x, RAMPS)
    assert bits_equal(g, c)
    ref, _ = CO.batch_resample_mix_f32(x[:1], RAMPS, 147, 160, threads=8)
    assert bits_equal(c[:1], ref)


def test_config1_clips_gpu_equals_cpu(xm, gpu):
    """Config 1's form (mono s16 44.1k->48k, 10 s) over a batch of clips."""
    x = np.stack([O.gen_s16(SEED, b, 1, 441000) for b in range(16)])[:, None]
    g, c = _both(xm, (44100, 48000, 1, "s16"), {}, x)
    assert bits_equal(g, c)
    assert bits_equal(c[0], CO.resample_s16(x[0, 0], 160, 147))


def test_config3_s16_mix_gpu_equals_cpu(xm, gpu):
    q = [dict(gain0_q15=a, gain1_q15=b, ramp_start=s, ramp_len=n, mode=md)
         for a, b, s, n, md in [(32768, 32768, 0, 0, 0), (0, 32768, 100, 48000, 0), (65535, 100, 0, 960000, 0),
                                (16384, 16384, 0, 0, 0), (0, 0, 300000, 96000, 1), (0, 32768, 300000, 96000, 0),
                                (40000, 3, 70000, 13, 0), (7, 60000, 480000, 0, 0)]]
    x = np.stack([np.stack([O.gen_s16(SEED, 500 + 8 * b + t, 2, 480000) for t in range(8)]) for b in range(4)])
    g, c = _both(xm, (48000, 48000, 2, "s16"), {}, x, q)
    assert bits_equal(g, c)
    assert bits_equal(c[:1], CO.batch_mix_s16(x[:1], q, threads=8)[0])


def test_config4_chain_gpu_equals_cpu(xm, gpu):
    """Config 4's chain: resample -> 5-band EQ -> gain -> ordered mix, 2 s."""
    from conftest import golden
    sos = golden("effects.npz")["sos"]
    x = np.stack([np.stack([O.gen_f32(SEED, 700 + 8 * b + t, 2, 96000) for t in range(8)]) for b in range(2)])
    g, c = _both(xm, (48000, 44100, 2, "f32"), {}, x, RAMPS, fx=sos)
    assert bits_equal(g, c)
    r = [CO.biquad_f32(CO.resample_f32(t, 147, 160), sos) for t in x[0]]
    assert bits_equal(c[0], CO.mix_f32(r, RAMPS))


@pytest.mark.parametrize("rates", [(44100, 48000), (32000, 48000), (48000, 16000)])
def test_other_ratios_gpu_equals_cpu(xm, gpu, rates):
    x = np.stack([np.stack([O.gen_f32(SEED, 900 + 4 * b + t, 2, 100000 + 7) for t in range(4)]) for b in range(3)])
    g, c = _both(xm, (*rates, 2, "f32"), {}, x, RAMPS[:4])
    assert bits_equal(g, c)
