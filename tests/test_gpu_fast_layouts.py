"""The fused 48k->44.1k kernel beyond the 8-track shape:
row layouts of 1, 2, 4 and 8 tracks per mix with 8 / 4 / 2 / 1 mixes per
wave, and 9-16 tracks as 16 rows of 4 stream slots.  Track counts between
the layouts run with phantom rows (zero input, left out of the sum); a
batch that does not fill the last wave, and the padding waves of the last
8-wave workgroup, store nothing.  Every case must run on the fused kernel
(XmMixerTiming.fast_launches == 1) and equal the oracle bit for bit."""
import numpy as np
import pytest

from conftest import bits_equal

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED


def _ramps(nt, N):
    out = []
    F = (N * 147 + 159) // 160
    for t in range(nt):
        k = t % 6
        if k == 0:
            out.append(dict(gain0=0.9 - 0.05 * t))
        elif k == 1:
            out.append(dict(gain0=0.0, gain1=0.8, ramp_start=37 * t, ramp_len=F // 3))
        elif k == 2:
            out.append(dict(mode=1, ramp_start=F // 4, ramp_len=F // 5))
        elif k == 3:
            out.append(dict(gain0=0.3, gain1=0.6, ramp_start=F // 2))              # step
        elif k == 4:
            out.append(dict(gain0=1.25, gain1=0.5, ramp_start=0, ramp_len=F))
        else:
            out.append(dict(gain0=0.5, gain1=0.0, ramp_start=F - 900, ramp_len=800))
    return out


def _x(B, nt, N, base):
    return np.stack([np.stack([O.gen_f32(SEED, base + 16 * b + t, 2, N) for t in range(nt)]) for b in range(B)])


@pytest.mark.parametrize("nt", [1, 2, 3, 4, 5, 6, 7, 9, 12, 16])
@pytest.mark.parametrize("N", [48000, 48001])
def test_fast_track_counts(xm, gpu, nt, N):
    B = 5 if nt <= 8 else 3          # 5 mixes: the last wave of 2- and 4-mix rows is partly empty
    x = _x(B, nt, N, 7000 + 100 * nt)
    ramps = _ramps(nt, N)
    m = xm.Mixer(48000, 44100, 2, "f32")
    m.set_tracks(ramps)
    y = m.process(x)
    t = m.timing()
    assert t.n_launches == 1 and t.fast_launches == 1, (t.n_launches, t.fast_launches)
    ref, _ = CO.batch_resample_mix_f32(x, ramps, 147, 160, threads=4)
    assert bits_equal(y, ref)


@pytest.mark.parametrize("nt", [1, 2, 4, 12])
def test_fast_layouts_device_strides_tables_s16_out(xm, gpu, nt):
    """Device memory with padded strides, a scattered pointer table, and the
    s16 store epilogue, for each row layout."""
    import torch
    N, B = 9601, 9
    x = _x(B, nt, N, 8000 + 100 * nt)
    ramps = _ramps(nt, N)
    ref, _ = CO.batch_resample_mix_f32(x, ramps, 147, 160, threads=4)
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    m.set_tracks(ramps)
    F = m.out_frames(N)
    ts, ms = N * 2 + 6, (N * 2 + 6) * nt + 10
    buf = np.zeros(B * ms + 16, np.float32)
    for b in range(B):
        for t in range(nt):
            buf[b * ms + t * ts: b * ms + t * ts + 2 * N] = x[b, t].reshape(-1)
    xd = torch.from_numpy(buf).cuda()
    yd = torch.full((B, F * 2 + 4), float("nan"), dtype=torch.float32, device="cuda")
    m.process_strided(xd.data_ptr(), ts, ms, yd.data_ptr(), F * 2 + 4, B, N)
    torch.cuda.synchronize()
    assert m.timing().fast_launches == 1
    assert bits_equal(yd.cpu().numpy()[:, :2 * F].reshape(B, F, 2), ref)
    # pointer table: tracks of every mix in a scattered order
    perm = [(5 * t + 3) % nt for t in range(nt)]
    ins = [xd[b * ms + perm[t] * ts:].data_ptr() for b in range(B) for t in range(nt)]
    y2 = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    if nt <= 8 and 8 // max(1, 1 << (nt - 1).bit_length()) > 1:
        outs = [y2[b].data_ptr() for b in range(B)]   # several mixes per wave: a strided output table
    else:
        outs = [y2[(5 * b + 2) % B].data_ptr() for b in range(B)]   # a permutation of the rows
    m.process_ptrs(ins, outs, B, N)
    torch.cuda.synchronize()
    assert m.timing().fast_launches == 1
    ref2, _ = CO.batch_resample_mix_f32(x[:, perm], ramps, 147, 160, threads=4)   # gains follow the slot
    got = y2.cpu().numpy()
    for b in range(B):
        o = b if outs[1] - outs[0] == F * 8 else (5 * b + 2) % B
        assert bits_equal(got[o], ref2[b]), b
    # s16 output
    c = xm.Mixer(48000, 44100, 2, "f32", convert_out=True)
    c.set_tracks(ramps)
    y3 = c.process(x)
    assert c.timing().fast_launches == 1
    want = np.clip(np.rint(ref.astype(np.float32) * np.float32(32768)), -32768, 32767).astype(np.int16)
    assert bits_equal(y3, want)


def test_fast_split_with_gain(xm, gpu):
    """One track per mix with a gain ramp (not only unity resampling) on the
    1-track rows, 11 mixes (the last wave holds 3 of its 8)."""
    N, B = 48001, 11
    x = _x(B, 1, N, 9000)
    ramps = [dict(gain0=0.2, gain1=1.1, ramp_start=100, ramp_len=20000)]
    m = xm.Mixer(48000, 44100, 2, "f32")
    m.set_tracks(ramps)
    y = m.process(x)
    assert m.timing().fast_launches == 1
    assert bits_equal(y, CO.batch_resample_mix_f32(x, ramps, 147, 160, threads=4)[0])


@pytest.mark.parametrize("nt", [4, 5, 6])
def test_fast_phantom_rows_s16_and_planar(xm, gpu, nt):
    """4-7 tracks on the 8-row s16 and planar kernels (phantom rows)."""
    N, B = 9600 + 33, 3
    F = (N * 147 + 159) // 160
    xs = np.stack([np.stack([O.gen_s16(SEED, 9100 + 16 * b + t, 2, N) for t in range(nt)]) for b in range(B)])
    q15 = [dict(gain0_q15=29491 - 1000 * t, gain1_q15=3000 * t, ramp_start=200 * t, ramp_len=5000) for t in range(nt)]
    m = xm.Mixer(48000, 44100, 2, "s16")
    m.set_tracks(q15)
    y = m.process(xs)
    assert m.timing().fast_launches == 1
    for b in range(B):
        assert bits_equal(y[b], CO.resample_mix_s16(list(xs[b]), q15, 147, 160)), b
    ramps = _ramps(nt, N)
    c = xm.Mixer(48000, 44100, 2, "f32", convert_in=True)
    c.set_tracks(ramps)
    yc = c.process(xs)
    assert c.timing().fast_launches == 1
    xf = xs.astype(np.float32) * np.float32(2.0 ** -15)
    assert bits_equal(yc, CO.batch_resample_mix_f32(xf, ramps, 147, 160, threads=4)[0])
    xp = _x(B, nt, N, 9200)
    p = xm.Mixer(48000, 44100, 2, "f32", planar=True)
    p.set_tracks(ramps)
    yp = p.process(np.ascontiguousarray(np.swapaxes(xp, -1, -2)))
    assert p.timing().fast_launches == 1
    ref = CO.batch_resample_mix_f32(xp, ramps, 147, 160, threads=4)[0]
    assert bits_equal(yp, np.ascontiguousarray(np.swapaxes(ref, -1, -2)))
    assert F == ref.shape[1]
