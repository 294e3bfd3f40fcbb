"""The fused 48k->44.1k kernel's s16 store epilogue (XM_MIXER_OUT_CONVERT on an
f32 mixer): the 8-track mix, the resample-only split
mode and streamed releases write s16 = sat16(rint(y * 32768)) straight from
the kernel, bit-equal to the oracle's f32 result converted in numpy
(np.rint is ties-to-even, as v_rndne_f32), and the fused kernel is the one
that ran (XmMixerTiming.fast_launches)."""
import numpy as np
import pytest

from conftest import bits_equal

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED


def _to_s16(y):
    return np.clip(np.rint(y.astype(np.float32) * np.float32(32768.0)), -32768, 32767).astype(np.int16)


@pytest.mark.parametrize("N", [48000, 48001, 160 * 40 + 33])
def test_fast_mix_convert_out(xm, gpu, N):
    from bench import RAMPS
    B = 3
    x = np.stack([np.stack([O.gen_f32(SEED, 6000 + 8 * b + t, 2, N) for t in range(8)]) for b in range(B)])
    x[:, :, 1000:1400] = 0.97          # the 8-track sum passes full scale: both saturation edges
    x[:, 4:, 2000:2300] = -0.99
    m = xm.Mixer(48000, 44100, 2, "f32", convert_out=True)
    m.set_tracks(RAMPS)
    y = m.process(x)
    t = m.timing()
    assert y.dtype == np.int16
    assert t.fast_launches == 1, (t.n_launches, t.fast_launches)
    ref, _ = CO.batch_resample_mix_f32(x, RAMPS, 147, 160, threads=2)
    want = _to_s16(ref)
    assert (want == 32767).any() and (want == -32768).any()
    assert bits_equal(y, want)


def test_fast_split_convert_out(xm, gpu):
    """Resample-only batches (split mode) with s16 output: 8 clips on the
    fused kernel, the 9th on the generic kernel, every clip checked."""
    import torch
    N, B = 9601, 9
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device", convert_out=True)
    m.set_tracks([dict(gain0=1.0)])
    F = m.out_frames(N)
    x = torch.empty((B, N, 2), dtype=torch.float32, device="cuda")
    xm.synth(x.data_ptr(), "f32", SEED, 91, B, 2, N)
    x[:, 500:700] *= 3.0               # saturating clips
    y = torch.full((B, F, 2), 0x5a5a, dtype=torch.int16, device="cuda")
    m.process_strided(x.data_ptr(), N * 2, N * 2, y.data_ptr(), F * 2, B, N)
    t = m.timing()
    assert t.fast_launches == 1, (t.n_launches, t.fast_launches)
    xs = x.cpu().numpy()
    got = y.cpu().numpy()
    for b in range(B):
        assert bits_equal(got[b], _to_s16(CO.resample_f32(xs[b], 147, 160))), b


def test_fast_stream_convert_out(xm, gpu):
    """Streamed releases take the fused kernel for their super-period-aligned
    bulk with s16 output too; the concatenated releases equal the whole call."""
    from bench import RAMPS
    B, N = 2, 30001
    x = np.stack([np.stack([O.gen_f32(SEED, 6100 + 8 * b + t, 2, N) for t in range(8)]) for b in range(B)])
    m = xm.Mixer(48000, 44100, 2, "f32", convert_out=True)
    m.set_tracks(RAMPS)
    whole = m.process(x)
    m.stream_begin(B)
    parts, fast = [], 0
    for a, e in [(0, 7000), (7000, 7001), (7001, 19000), (19000, N)]:
        parts.append(m.stream_push(x[:, :, a:e]))
        fast += m.timing().fast_launches
    parts.append(m.stream_flush())
    ys = np.concatenate(parts, axis=1)
    assert fast >= 2, fast
    assert bits_equal(ys, whole)
    ref, _ = CO.batch_resample_mix_f32(x, RAMPS, 147, 160, threads=2)
    assert bits_equal(whole, _to_s16(ref))
