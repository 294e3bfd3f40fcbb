"""The fused kernel at 44.1 kHz -> 48 kHz (L/M = 160/147, SURVEY.md §8(a) a1
second table, a2, config 1's direction): a super-period is
147 input frames -> 160 outputs, each output runs its 20 used taps (tap 0 or
tap 20 of its phase is an exact zero; one output per SP runs 21).  Every case
must run on the fused kernel (XmMixerTiming.fast_launches == 1) and equal the
C oracle bit for bit: every row layout and track count, odd and tiny frame
counts, strided device memory, pointer tables, the s16 store epilogue, s16
tracks (into the f32 mix and the Q15 mix), planar tracks, and the 1-track
(resample-only) rows at the production shape of the `up` bench line."""
import numpy as np
import pytest

from conftest import bits_equal, golden

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED


def _F(N):
    return (N * 160 + 146) // 147


def _ramps(nt, N):
    F = _F(N)
    out = []
    for t in range(nt):
        k = t % 6
        if k == 0:
            out.append(dict(gain0=0.9 - 0.05 * t))
        elif k == 1:
            out.append(dict(gain0=0.0, gain1=0.8, ramp_start=41 * t, ramp_len=F // 3))
        elif k == 2:
            out.append(dict(mode=1, ramp_start=F // 4, ramp_len=F // 5))
        elif k == 3:
            out.append(dict(gain0=0.3, gain1=0.6, ramp_start=F // 2))              # step
        elif k == 4:
            out.append(dict(gain0=1.25, gain1=0.5, ramp_start=0, ramp_len=F))
        else:
            out.append(dict(gain0=0.5, gain1=0.0, ramp_start=max(0, F - 900), ramp_len=800))
    return out


def _x(B, nt, N, base):
    return np.stack([np.stack([O.gen_f32(SEED, base + 16 * b + t, 2, N) for t in range(nt)]) for b in range(B)])


def _fast(m):
    t = m.timing()
    assert t.n_launches == 1 and t.fast_launches == m.fused, (t.n_launches, t.fast_launches)   # fused: GPU handles


@pytest.mark.parametrize("nt", [1, 2, 3, 4, 6, 8, 9, 16])
@pytest.mark.parametrize("N", [44100, 44101])
def test_up_track_counts(xm, gpu, nt, N):
    B = 5 if nt <= 8 else 3
    x = _x(B, nt, N, 11000 + 100 * nt)
    ramps = _ramps(nt, N)
    m = xm.Mixer(44100, 48000, 2, "f32")
    m.set_tracks(ramps)
    y = m.process(x)
    _fast(m)
    ref, _ = CO.batch_resample_mix_f32(x, ramps, 160, 147, threads=4)
    assert bits_equal(y, ref)


@pytest.mark.parametrize("N", [1, 2, 7, 146, 147, 148, 179, 180, 293, 294, 295, 147 * 40 + 1, 147 * 40 + 13])
def test_up_short_and_edge_lengths(xm, gpu, N):
    """Clips shorter than one super-period or one DMA segment, and lengths
    around an SP edge (the edge SPs redirect chunks past N)."""
    B, nt = 3, 8
    x = _x(B, nt, N, 12000 + N)
    ramps = _ramps(nt, N)
    m = xm.Mixer(44100, 48000, 2, "f32")
    m.set_tracks(ramps)
    y = m.process(x)
    _fast(m)
    ref, _ = CO.batch_resample_mix_f32(x, ramps, 160, 147, threads=4)
    assert bits_equal(y, ref)


@pytest.mark.parametrize("kind", ["silence", "fullscale", "denormal", "impulse"])
def test_up_special_inputs(xm, gpu, kind):
    """The 48k->44.1k golden special inputs resampled the other way (C oracle;
    a zero coefficient meets denormal, full-scale and silent samples)."""
    x = golden("resample.npz")[f"special_{kind}__x"]
    m = xm.Mixer(44100, 48000, 2, "f32")
    m.set_tracks([dict(gain0=1.0)])
    y = m.process(np.stack([x, x[::-1]])[:, None])
    _fast(m)
    for b, xb in enumerate((x, x[::-1])):
        assert bits_equal(y[b], CO.resample_f32(np.ascontiguousarray(xb), 160, 147)), b


def test_up_device_strides_tables_s16_out(xm, gpu):
    """Padded strides in device memory, a scattered pointer table, and the s16
    store epilogue."""
    import torch
    nt, N, B = 8, 8821, 9
    x = _x(B, nt, N, 13000)
    ramps = _ramps(nt, N)
    ref, _ = CO.batch_resample_mix_f32(x, ramps, 160, 147, threads=4)
    m = xm.Mixer(44100, 48000, 2, "f32", mem="device")
    m.set_tracks(ramps)
    F = m.out_frames(N)
    assert F == _F(N)
    ts, ms = N * 2 + 6, (N * 2 + 6) * nt + 10
    buf = np.zeros(B * ms + 16, np.float32)
    for b in range(B):
        for t in range(nt):
            buf[b * ms + t * ts: b * ms + t * ts + 2 * N] = x[b, t].reshape(-1)
    xd = torch.from_numpy(buf).cuda()
    yd = torch.full((B, F * 2 + 4), float("nan"), dtype=torch.float32, device="cuda")
    m.process_strided(xd.data_ptr(), ts, ms, yd.data_ptr(), F * 2 + 4, B, N)
    torch.cuda.synchronize()
    _fast(m)
    assert bits_equal(yd.cpu().numpy()[:, :2 * F].reshape(B, F, 2), ref)
    perm = [(5 * t + 3) % nt for t in range(nt)]
    ins = [xd[b * ms + perm[t] * ts:].data_ptr() for b in range(B) for t in range(nt)]
    y2 = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    outs = [y2[(5 * b + 2) % B].data_ptr() for b in range(B)]
    m.process_ptrs(ins, outs, B, N)
    torch.cuda.synchronize()
    _fast(m)
    ref2, _ = CO.batch_resample_mix_f32(x[:, perm], ramps, 160, 147, threads=4)
    got = y2.cpu().numpy()
    for b in range(B):
        assert bits_equal(got[(5 * b + 2) % B], ref2[b]), b
    c = xm.Mixer(44100, 48000, 2, "f32", convert_out=True)
    c.set_tracks(ramps)
    y3 = c.process(x)
    _fast(c)
    want = np.clip(np.rint(ref.astype(np.float32) * np.float32(32768)), -32768, 32767).astype(np.int16)
    assert bits_equal(y3, want)


@pytest.mark.parametrize("nt", [4, 8])
def test_up_s16_and_planar(xm, gpu, nt):
    """s16 tracks into the Q15 mix and into the f32 mix, planar f32 tracks and
    mixes (the 8-row kernels; 4 tracks leave phantom rows)."""
    N, B = 8820 + 33, 3
    xs = np.stack([np.stack([O.gen_s16(SEED, 14000 + 16 * b + t, 2, N) for t in range(nt)]) for b in range(B)])
    q15 = [dict(gain0_q15=29491 - 1000 * t, gain1_q15=3000 * t, ramp_start=200 * t, ramp_len=5000) for t in range(nt)]
    m = xm.Mixer(44100, 48000, 2, "s16")
    m.set_tracks(q15)
    y = m.process(xs)
    _fast(m)
    for b in range(B):
        assert bits_equal(y[b], CO.resample_mix_s16(list(xs[b]), q15, 160, 147)), b
    ramps = _ramps(nt, N)
    c = xm.Mixer(44100, 48000, 2, "f32", convert_in=True)
    c.set_tracks(ramps)
    yc = c.process(xs)
    _fast(c)
    xf = xs.astype(np.float32) * np.float32(2.0 ** -15)
    assert bits_equal(yc, CO.batch_resample_mix_f32(xf, ramps, 160, 147, threads=4)[0])
    xp = _x(B, nt, N, 15000)
    p = xm.Mixer(44100, 48000, 2, "f32", planar=True)
    p.set_tracks(ramps)
    yp = p.process(np.ascontiguousarray(np.swapaxes(xp, -1, -2)))
    _fast(p)
    ref = CO.batch_resample_mix_f32(xp, ramps, 160, 147, threads=4)[0]
    assert bits_equal(yp, np.ascontiguousarray(np.swapaxes(ref, -1, -2)))


def test_up_resample_only_production_grid(xm, gpu):
    """1-track unity mixes (resample only) at 4096 x 441000 frames: 64-B
    output segments are whole per store at this ratio (160 outputs per SP);
    the first and last clips bit-checked, nothing left unwritten."""
    import torch
    B, N = 4096, 441000
    m = xm.Mixer(44100, 48000, 2, "f32", mem="device")
    m.set_tracks([dict(gain0=1.0)])
    F = m.out_frames(N)
    x = torch.empty((B, N, 2), dtype=torch.float32, device="cuda")
    y = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    xm.synth(x.data_ptr(), "f32", SEED, 0, B, 2, N)
    torch.cuda.synchronize()
    m.process_strided(x.data_ptr(), N * 2, N * 2, y.data_ptr(), F * 2, B, N)
    torch.cuda.synchronize()
    _fast(m)
    for b in (0, B - 1):
        assert bits_equal(y[b].cpu().numpy(), CO.resample_f32(x[b].cpu().numpy(), 160, 147)), b
    assert not bool(y.isnan().any())
    del x, y
    torch.cuda.empty_cache()
