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
    torch.cuda.synchronize()
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


@pytest.mark.parametrize("N", [48000, 48001, 48002, 48003, 160 * 40 + 33])
@pytest.mark.parametrize("convert_out", [False, True])
def test_fast_s16_tracks_into_f32_mix(xm, gpu, N, convert_out):
    """XM_MIXER_IN_CONVERT on the fused kernel: 8 s16 tracks (4-B frames,
    128-B DMA segments) read as x * 2^-15 into the f32 mix; every N mod 4
    (a partial last 4-frame chunk holds the next track's first samples,
    which the copy zeroes), full-scale samples, optionally s16 out."""
    from bench import RAMPS
    B = 3
    x = np.stack([np.stack([O.gen_s16(SEED, 6200 + 8 * b + t, 2, N) for t in range(8)]) for b in range(B)])
    x[:, :, 300:340] = 32767
    x[:, 3:, 700:720] = -32768
    m = xm.Mixer(48000, 44100, 2, "f32", convert_in=True, convert_out=convert_out)
    m.set_tracks(RAMPS)
    y = m.process(x)
    t = m.timing()
    assert t.fast_launches == 1, (t.n_launches, t.fast_launches)
    xf = x.astype(np.float32) * np.float32(2.0 ** -15)
    ref, _ = CO.batch_resample_mix_f32(xf, RAMPS, 147, 160, threads=2)
    assert bits_equal(y, _to_s16(ref) if convert_out else ref)


def test_fast_s16_in_device_strides_and_tables(xm, gpu):
    """Device memory, s16 tracks at padded strides (frames 4-B aligned, not
    16-B) and through a scattered pointer table: the same bits as the
    oracle, on the fused kernel."""
    import torch
    from bench import RAMPS
    N, B, ntr = 9601, 3, 8
    x = np.stack([np.stack([O.gen_s16(SEED, 6300 + 8 * b + t, 2, N) for t in range(ntr)]) for b in range(B)])
    ts, ms = N * 2 + 6, (N * 2 + 6) * ntr + 10
    buf = np.zeros(B * ms, np.int16)
    for b in range(B):
        for t in range(ntr):
            buf[b * ms + t * ts: b * ms + t * ts + 2 * N] = x[b, t].reshape(-1)
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device", convert_in=True)
    m.set_tracks(RAMPS)
    F = m.out_frames(N)
    xd = torch.from_numpy(buf).cuda()
    yd = torch.zeros((B, F * 2 + 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    m.process_strided(xd.data_ptr(), ts, ms, yd.data_ptr(), F * 2 + 4, B, N)
    torch.cuda.synchronize()
    assert m.timing().fast_launches == 1
    xf = x.astype(np.float32) * np.float32(2.0 ** -15)
    ref, _ = CO.batch_resample_mix_f32(xf, RAMPS, 147, 160, threads=2)
    y = yd.cpu().numpy()[:, :2 * F].reshape(B, F, 2)
    assert bits_equal(y, ref)
    # pointer table: every mix's tracks in a scattered order inside the buffer
    perm = [(3 * t + 5) % ntr for t in range(ntr)]
    ins = [xd[b * ms + perm[t] * ts:].data_ptr() for b in range(B) for t in range(ntr)]
    y2 = torch.zeros((B, F, 2), dtype=torch.float32, device="cuda")
    m.process_ptrs(ins, [y2[b].data_ptr() for b in range(B)], B, N)
    torch.cuda.synchronize()
    assert m.timing().fast_launches == 1
    ref2, _ = CO.batch_resample_mix_f32(xf[:, perm], RAMPS, 147, 160, threads=2)
    assert bits_equal(y2.cpu().numpy(), ref2)


Q15_RAMPS = [dict(gain0_q15=29491), dict(gain0_q15=0, gain1_q15=26214, ramp_start=0, ramp_len=4800),
             dict(gain0_q15=22938, gain1_q15=6554, ramp_start=2400, ramp_len=9600), dict(gain0_q15=65535),
             dict(mode=1, ramp_start=1440, ramp_len=9601),
             dict(gain0_q15=0, gain1_q15=32768, ramp_start=14400, ramp_len=9599),
             dict(gain0_q15=32768, gain1_q15=0, ramp_start=43200, ramp_len=4800),
             dict(gain0_q15=9830, gain1_q15=19661, ramp_start=30000, ramp_len=0)]


@pytest.mark.parametrize("N", [48000, 48003, 160 * 40 + 33])
@pytest.mark.parametrize("convert_out", [False, True])
def test_fast_s16_q15_mix(xm, gpu, N, convert_out):
    """s16 tracks into the s16 Q15 mix on the fused kernel: each track
    resampled in fp32 on its integer samples, sat16(rint(r)), times its Q15
    ramp (rising, falling, crossfade-out, step, gain 65535: the ramps' integer
    quotients advance per output without a division), (s*g + 2^14) >> 15,
    int32 sum, sat16; optionally f32 out (sat16 * 2^-15)."""
    B = 3
    x = np.stack([np.stack([O.gen_s16(SEED, 6400 + 8 * b + t, 2, N) for t in range(8)]) for b in range(B)])
    x[:, :, 300:340] = 32767             # full scale: every saturation stage
    x[:, 3:, 700:720] = -32768
    m = xm.Mixer(48000, 44100, 2, "s16", convert_out=convert_out)
    m.set_tracks(Q15_RAMPS)
    y = m.process(x)
    t = m.timing()
    assert t.fast_launches == 1, (t.n_launches, t.fast_launches)
    for b in range(B):
        ref = CO.resample_mix_s16(list(x[b]), Q15_RAMPS, 147, 160)
        if convert_out:
            ref = ref.astype(np.float32) * np.float32(2.0 ** -15)
        assert bits_equal(y[b], ref), b


def test_fast_s16_q15_long_ramps(xm, gpu):
    """Ramps of hundreds of thousands of frames: (q1 - q0) * k passes 2^31,
    so the per-SP start of the incremental quotient needs its 64-bit form;
    rising, falling and crossfade-out ramps, 10 s clips."""
    N, B = 480000, 2
    ramps = [dict(gain0_q15=0, gain1_q15=65535, ramp_start=1000, ramp_len=400000),
             dict(gain0_q15=60000, gain1_q15=100, ramp_start=0, ramp_len=441000),
             dict(mode=1, ramp_start=5000, ramp_len=300001),
             dict(gain0_q15=32768, gain1_q15=1, ramp_start=200000, ramp_len=240000)] * 2
    x = np.stack([np.stack([O.gen_s16(SEED, 6500 + 8 * b + t, 2, N) for t in range(8)]) for b in range(B)])
    m = xm.Mixer(48000, 44100, 2, "s16")
    m.set_tracks(ramps)
    y = m.process(x)
    assert m.timing().fast_launches == 1
    for b in range(B):
        assert bits_equal(y[b], CO.resample_mix_s16(list(x[b]), ramps, 147, 160)), b


def _planar(a):
    """[..., frames, channels] -> [..., channels, frames]"""
    return np.ascontiguousarray(np.swapaxes(a, -1, -2))


@pytest.mark.parametrize("N", [48000, 48001, 48003, 160 * 40 + 33])
def test_fast_planar_mix(xm, gpu, N):
    """XM_MIXER_PLANAR on the fused kernel: planar f32 tracks (plane R at
    +N samples, so for N mod 4 != 0 a partial chunk of plane L holds plane
    R's first samples, zeroed on the copy) and planar mixes (two b32 stores
    per output)."""
    from bench import RAMPS
    B = 3
    x = np.stack([np.stack([O.gen_f32(SEED, 6600 + 8 * b + t, 2, N) for t in range(8)]) for b in range(B)])
    m = xm.Mixer(48000, 44100, 2, "f32", planar=True)
    m.set_tracks(RAMPS)
    y = m.process(_planar(x))
    assert m.timing().fast_launches == 1
    ref, _ = CO.batch_resample_mix_f32(x, RAMPS, 147, 160, threads=2)
    assert bits_equal(y, _planar(ref))


def test_fast_planar_device_pointer_table(xm, gpu):
    """Planar tracks through a scattered pointer table in device memory."""
    import torch
    from bench import RAMPS
    N, B = 9601, 2
    x = np.stack([np.stack([O.gen_f32(SEED, 6700 + 8 * b + t, 2, N) for t in range(8)]) for b in range(B)])
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device", planar=True)
    m.set_tracks(RAMPS)
    F = m.out_frames(N)
    xd = torch.from_numpy(_planar(x)).cuda()               # [B][8][2][N]
    perm = [(5 * t + 1) % 8 for t in range(8)]
    ins = [xd[b, perm[t]].data_ptr() for b in range(B) for t in range(8)]
    y = torch.full((B, 2, F), float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    m.process_ptrs(ins, [y[b].data_ptr() for b in range(B)], B, N)
    torch.cuda.synchronize()
    assert m.timing().fast_launches == 1
    ref, _ = CO.batch_resample_mix_f32(x[:, perm], RAMPS, 147, 160, threads=2)
    assert bits_equal(y.cpu().numpy(), _planar(ref))
