"""The fused kernel at the small-L/M ratios (SURVEY.md
§8(a) a1-a2): 3/2 (32k -> 48k, 16k -> 24k), 2/3 (48k -> 32k) and 1/2
(96k -> 48k): stereo f32 interleaved tracks, mono f32 tracks and mono s16
tracks into the Q15 mix, 1-8 tracks per mix.  A
super-period is P periods (160 or 159 input frames) and every output runs all
T taps of its phase (RatioBase<RID_32/23/12> in csrc/xm_resample_fast.hip).
Every case must run on the fused kernel (XmMixerTiming.fast_launches == 1)
and equal the C oracle bit for bit: track counts (1-track rows and 8-row
mixes with phantom rows), odd and tiny frame counts, lengths around a
super-period edge, padded device strides, scattered pointer tables, and the
s16 store epilogue."""
import numpy as np
import pytest

from conftest import bits_equal

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED

# (in rate, out rate, L, M, input frames per super-period)
RATIOS = [(32000, 48000, 3, 2, 160), (48000, 32000, 2, 3, 159), (96000, 48000, 1, 2, 160)]
IDS = ["3_2", "2_3", "1_2"]


def _F(N, L, M):
    return (N * L + M - 1) // M


def _ramps(nt, F):
    out = []
    for t in range(nt):
        k = t % 6
        if k == 0:
            out.append(dict(gain0=0.9 - 0.05 * t))
        elif k == 1:
            out.append(dict(gain0=0.0, gain1=0.8, ramp_start=41 * t, ramp_len=max(1, F // 3)))
        elif k == 2:
            out.append(dict(mode=1, ramp_start=F // 4, ramp_len=max(1, F // 5)))
        elif k == 3:
            out.append(dict(gain0=0.3, gain1=0.6, ramp_start=F // 2))              # step
        elif k == 4:
            out.append(dict(gain0=1.25, gain1=0.5, ramp_start=0, ramp_len=max(1, F)))
        else:
            out.append(dict(gain0=0.5, gain1=0.0, ramp_start=max(0, F - 900), ramp_len=800))
    return out


def _x(B, nt, N, base):
    return np.stack([np.stack([O.gen_f32(SEED, base + 16 * b + t, 2, N) for t in range(nt)]) for b in range(B)])


def _fast(m):
    t = m.timing()
    assert t.n_launches == 1 and t.fast_launches == 1, (t.n_launches, t.fast_launches)


@pytest.mark.parametrize("ratio", RATIOS, ids=IDS)
@pytest.mark.parametrize("nt", [1, 2, 5, 8])
@pytest.mark.parametrize("odd", [0, 1])
def test_small_track_counts(xm, gpu, ratio, nt, odd):
    fi, fo, L, M, SPI = ratio
    N = 20 * SPI + 37 + odd
    B = 5
    x = _x(B, nt, N, 21000 + 100 * nt + odd)
    ramps = _ramps(nt, _F(N, L, M))
    m = xm.Mixer(fi, fo, 2, "f32")
    m.set_tracks(ramps)
    y = m.process(x)
    _fast(m)
    ref, _ = CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)
    assert bits_equal(y, ref)


@pytest.mark.parametrize("ratio", RATIOS, ids=IDS)
def test_small_short_and_edge_lengths(xm, gpu, ratio):
    """Clips shorter than one super-period or one DMA segment, and lengths
    around super-period edges (the edge SPs redirect chunks past N)."""
    fi, fo, L, M, SPI = ratio
    for N in (1, 2, 7, 31, 33, SPI - 1, SPI, SPI + 1, 2 * SPI - 1, 2 * SPI + 1, 40 * SPI + 13):
        B, nt = 3, 8
        x = _x(B, nt, N, 22000 + N)
        ramps = _ramps(nt, _F(N, L, M))
        m = xm.Mixer(fi, fo, 2, "f32")
        m.set_tracks(ramps)
        y = m.process(x)
        _fast(m)
        ref, _ = CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)
        assert bits_equal(y, ref), N


def test_same_design_other_rates(xm, gpu):
    """16k -> 24k is the 3/2 design (L and M alone define the filter)."""
    N, nt = 16000 + 3, 4
    x = _x(2, nt, N, 23000)
    ramps = _ramps(nt, _F(N, 3, 2))
    m = xm.Mixer(16000, 24000, 2, "f32")
    m.set_tracks(ramps)
    y = m.process(x)
    _fast(m)
    assert bits_equal(y, CO.batch_resample_mix_f32(x, ramps, 3, 2, threads=4)[0])


@pytest.mark.parametrize("ratio", RATIOS, ids=IDS)
def test_small_device_strides_tables_s16_out(xm, gpu, ratio):
    """Padded strides in device memory, a scattered pointer table, and the s16
    store epilogue."""
    import torch
    fi, fo, L, M, SPI = ratio
    nt, N, B = 8, 9001, 9
    x = _x(B, nt, N, 24000)
    ramps = _ramps(nt, _F(N, L, M))
    ref, _ = CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)
    m = xm.Mixer(fi, fo, 2, "f32", mem="device")
    m.set_tracks(ramps)
    F = m.out_frames(N)
    assert F == _F(N, L, M)
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
    ref2, _ = CO.batch_resample_mix_f32(x[:, perm], ramps, L, M, threads=4)
    got = y2.cpu().numpy()
    for b in range(B):
        assert bits_equal(got[(5 * b + 2) % B], ref2[b]), b
    c = xm.Mixer(fi, fo, 2, "f32", convert_out=True)
    c.set_tracks(ramps)
    y3 = c.process(x)
    _fast(c)
    want = np.clip(np.rint(ref.astype(np.float32) * np.float32(32768)), -32768, 32767).astype(np.int16)
    assert bits_equal(y3, want)


def test_small_production_grid_32_48(xm, gpu):
    """The 32k -> 48k bench line's shape (512 mixes x 8 tracks x 10 s): the
    first and last mixes bit-checked, nothing left unwritten."""
    import torch
    B, nt, N = 512, 8, 320000
    ramps = _ramps(nt, _F(N, 3, 2))
    m = xm.Mixer(32000, 48000, 2, "f32", mem="device")
    m.set_tracks(ramps)
    F = m.out_frames(N)
    x = torch.empty((B * nt, N, 2), dtype=torch.float32, device="cuda")
    y = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    xm.synth(x.data_ptr(), "f32", SEED, 0, B * nt, 2, N)
    torch.cuda.synchronize()
    m.process_strided(x.data_ptr(), N * 2, N * 2 * nt, y.data_ptr(), F * 2, B, N)
    torch.cuda.synchronize()
    _fast(m)
    for b in (0, B - 1):
        xb = x[b * nt:(b + 1) * nt].cpu().numpy()[None]
        ref, _ = CO.batch_resample_mix_f32(xb, ramps, 3, 2, threads=8)
        assert bits_equal(y[b].cpu().numpy(), ref[0]), b
    assert not bool(y.isnan().any())
    del x, y
    torch.cuda.empty_cache()


def _xm1(B, nt, N, base, s16=False):
    g = O.gen_s16 if s16 else O.gen_f32
    return np.stack([np.stack([g(SEED, base + 16 * b + t, 1, N) for t in range(nt)]) for b in range(B)])


@pytest.mark.parametrize("ratio", RATIOS, ids=IDS)
@pytest.mark.parametrize("nt", [1, 3, 8])
def test_small_mono_f32(xm, gpu, ratio, nt):
    """Mono f32 tracks at the small ratios (the MONO instantiations: a lane's
    run in two halves riding as the planar pair), odd and even N."""
    fi, fo, L, M, SPI = ratio
    for N in (20 * SPI + 37, 20 * SPI + 38, 2 * SPI - 1):
        B = 11 if nt == 1 else 3
        x = _xm1(B, nt, N, 25000 + N + nt)
        ramps = _ramps(nt, _F(N, L, M))
        m = xm.Mixer(fi, fo, 1, "f32")
        m.set_tracks(ramps)
        y = m.process(x)
        t = m.timing()
        # 3/2 one-track mono rows: the generic kernel (vmcnt bound, see xmg_fast_kern_mono_r32)
        assert t.n_launches == 1 and t.fast_launches == (0 if (L, M, nt) == (3, 2, 1) else 1)
        ref, _ = CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)
        assert bits_equal(y, ref), N


@pytest.mark.parametrize("ratio", RATIOS, ids=IDS)
@pytest.mark.parametrize("nt", [1, 5])
def test_small_mono_s16_q15(xm, gpu, ratio, nt):
    """Mono s16 tracks into the Q15 mix at the small ratios (M16; 2/3 moves
    every other SP origin by one s16 frame), even and (since round 5) odd N
    on the fused kernel."""
    fi, fo, L, M, SPI = ratio
    for N in (20 * SPI + 38, 2 * SPI + 2, 20 * SPI + 37):
        B = 11 if nt == 1 else 3
        x = _xm1(B, nt, N, 26000 + N + nt, s16=True)
        F = _F(N, L, M)
        q = [dict(gain0_q15=32768 - 3000 * t, gain1_q15=1000 * t, ramp_start=37 * t, ramp_len=max(1, F // 3)) for t in range(nt)]
        m = xm.Mixer(fi, fo, 1, "s16")
        m.set_tracks(q)
        y = m.process(x)
        t = m.timing()
        fused = (L, M, nt) != (3, 2, 1)
        assert t.n_launches == 1 and t.fast_launches == (1 if fused else 0), (N, t.fast_launches)
        ref = np.stack([CO.resample_mix_s16(list(x[b]), q, L, M) for b in range(B)])
        assert bits_equal(y, ref), N


# 2/1 and 3/1: 320 and 480 outputs per super-period, 8-track rows only
UPRATIOS = [(24000, 48000, 2, 1, 160), (16000, 48000, 3, 1, 160)]


@pytest.mark.parametrize("ratio", UPRATIOS, ids=["2_1", "3_1"])
@pytest.mark.parametrize("nt", [1, 2, 5, 8])
def test_up_small_mixes(xm, gpu, ratio, nt):
    """Stereo f32 mixes at 2/1 (24k -> 48k) and 3/1 (16k -> 48k) on the fused
    kernel (2-8 tracks; 1-track resample-only batches: 2/1 fused since round
    5, 3/1 the generic kernel), odd and even N, lengths around super-period
    edges."""
    fi, fo, L, M, SPI = ratio
    for N in (20 * SPI + 37, 20 * SPI + 38, SPI - 1, SPI + 1, 2 * SPI + 1, 7):
        B = 3
        x = _x(B, nt, N, 27000 + N + nt)
        ramps = _ramps(nt, _F(N, L, M))
        m = xm.Mixer(fi, fo, 2, "f32")
        m.set_tracks(ramps)
        y = m.process(x)
        t = m.timing()
        assert t.n_launches == 1 and t.fast_launches == (1 if nt >= 2 or L == 2 else 0), (N, t.fast_launches)
        ref, _ = CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)
        assert bits_equal(y, ref), N


@pytest.mark.parametrize("ratio", RATIOS + UPRATIOS, ids=IDS + ["2_1", "3_1"])
@pytest.mark.parametrize("nt", [2, 8])
def test_small_multi_sp_runs(xm, gpu, ratio, nt):
    """Batches large enough that each lane walks several super-periods (R >= 2:
    the carry, the previous SP's last round stored in the next SP, the next
    SP's segment 2 loaded during this one).  Every output of every mix is
    checked; the small-batch tests above run one SP per lane.  (At 2/1 and 3/1
    the next SP's segment-2 DMA once ran past its 8 parts into the exchange
    rows: wrong last rounds at the production bench shape.)"""
    import torch
    fi, fo, L, M, SPI = ratio
    B, N = (64, 48000) if nt == 2 else (48, 96000)   # B * N / 160 SPs > 16384: R >= 2
    x = _x(B, nt, N, 29000 + nt)
    ramps = _ramps(nt, _F(N, L, M))
    m = xm.Mixer(fi, fo, 2, "f32", mem="device")
    m.set_tracks(ramps)
    F = m.out_frames(N)
    xd = torch.from_numpy(x).cuda()
    y = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    m.process_strided(xd.data_ptr(), N * 2, N * 2 * nt, y.data_ptr(), F * 2, B, N)
    torch.cuda.synchronize()
    _fast(m)
    ref, _ = CO.batch_resample_mix_f32(x, ramps, L, M, threads=8)
    assert bits_equal(y.cpu().numpy(), ref)


@pytest.mark.parametrize("ratio", UPRATIOS, ids=["2_1", "3_1"])
def test_up_small_production_grid(xm, gpu, ratio):
    """The 24k -> 48k and 16k -> 48k bench lines' shape (512 mixes x 8 tracks x
    10 s): first and last mixes bit-checked, nothing left unwritten."""
    import torch
    fi, fo, L, M, SPI = ratio
    B, nt, N = 512, 8, fi * 10
    ramps = _ramps(nt, _F(N, L, M))
    m = xm.Mixer(fi, fo, 2, "f32", mem="device")
    m.set_tracks(ramps)
    F = m.out_frames(N)
    x = torch.empty((B * nt, N, 2), dtype=torch.float32, device="cuda")
    y = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    xm.synth(x.data_ptr(), "f32", SEED, 0, B * nt, 2, N)
    torch.cuda.synchronize()
    m.process_strided(x.data_ptr(), N * 2, N * 2 * nt, y.data_ptr(), F * 2, B, N)
    torch.cuda.synchronize()
    _fast(m)
    for b in (0, B - 1):
        xb = x[b * nt:(b + 1) * nt].cpu().numpy()[None]
        ref, _ = CO.batch_resample_mix_f32(xb, ramps, L, M, threads=8)
        assert bits_equal(y[b].cpu().numpy(), ref[0]), b
    assert not bool(y.isnan().any())
    del x, y
    torch.cuda.empty_cache()


@pytest.mark.parametrize("ratio", RATIOS, ids=IDS)
@pytest.mark.parametrize("nt", [4, 8])
def test_small_stereo_s16(xm, gpu, ratio, nt):
    """Stereo s16 tracks at the small ratios (the IO instantiations, 8-track
    rows): the s16 Q15 mix and s16 tracks into the f32 mix, odd and even N."""
    fi, fo, L, M, SPI = ratio
    for N in (20 * SPI + 37, 20 * SPI + 38, SPI + 1):
        B = 3
        xs = np.stack([np.stack([O.gen_s16(SEED, 28000 + N + 16 * b + t, 2, N) for t in range(nt)]) for b in range(B)])
        F = _F(N, L, M)
        q = [dict(gain0_q15=29491 - 1000 * t, gain1_q15=3000 * t, ramp_start=200 * t, ramp_len=max(1, F // 4))
             for t in range(nt)]
        m = xm.Mixer(fi, fo, 2, "s16")
        m.set_tracks(q)
        y = m.process(xs)
        _fast(m)
        for b in range(B):
            assert bits_equal(y[b], CO.resample_mix_s16(list(xs[b]), q, L, M)), (N, b)
        ramps = _ramps(nt, F)
        c = xm.Mixer(fi, fo, 2, "f32", convert_in=True)
        c.set_tracks(ramps)
        yc = c.process(xs)
        _fast(c)
        xf = xs.astype(np.float32) * np.float32(2.0 ** -15)
        assert bits_equal(yc, CO.batch_resample_mix_f32(xf, ramps, L, M, threads=4)[0]), N
