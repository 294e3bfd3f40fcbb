"""Mono s16 tracks on the fused kernel (M16, VERDICT r3 item 5: config 1's own
form): the MONO instantiations with 2-byte stream frames.  At 44.1k -> 48k an
SP origin moves 294 B, so every other SP's segments start 2 B off a dword;
the DMA reads from the dword before and the copy shifts by one frame.  Both
table ratios, the Q15 mix (s16 out) and s16 tracks into the f32 mix
(convert_in), 1-track rows (batches of clips) and 2-8-track mixes, ramps
whose edges fall in either half of a lane's run, short clips and lengths
around super-period edges, strided device memory and pointer tables.  Every
case must run on the fused kernel (XmMixerTiming.fast_launches == 1): since
round 5 odd frame counts too (every other clip 2 B off a dword: each row's
DMA window starts at the dword before its own segment start, and the copy
shifts by that row's delta).  All equal the C oracle bit for bit."""
import numpy as np
import pytest

from conftest import bits_equal

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED
RATES = {(48000, 44100): (147, 160), (44100, 48000): (160, 147)}


def _F(N, L, M):
    return (N * L + M - 1) // M


def _q15(nt, F):
    out = []
    for t in range(nt):
        k = t % 5
        if k == 0:
            out.append(dict(gain0_q15=32768 - 1111 * t))
        elif k == 1:
            out.append(dict(gain0_q15=0, gain1_q15=29491, ramp_start=37 * t, ramp_len=max(1, F // 3)))
        elif k == 2:
            out.append(dict(mode=1, ramp_start=F // 4, ramp_len=max(1, F // 5)))
        elif k == 3:
            out.append(dict(gain0_q15=9830, gain1_q15=19661, ramp_start=F // 2))      # step
        else:
            out.append(dict(gain0_q15=40960, gain1_q15=3, ramp_start=0, ramp_len=max(1, F)))
    return out


def _f32ramps(nt, F):
    return [dict(gain0=0.9 - 0.1 * t, gain1=0.2 + 0.05 * t, ramp_start=29 * t, ramp_len=max(1, F // 2)) for t in range(nt)]


def _xs(B, nt, N, base):
    return np.stack([np.stack([O.gen_s16(SEED, base + 16 * b + t, 1, N) for t in range(nt)]) for b in range(B)])


def _ref_s16(x, ramps, L, M):
    return np.stack([CO.resample_mix_s16(list(x[b]), ramps, L, M) for b in range(x.shape[0])])


def _run(xm, rates, x, ramps, fmt="s16", **kw):
    m = xm.Mixer(*rates, 1, fmt, **kw)
    m.set_tracks(ramps)
    y = m.process(x)
    t = m.timing()
    assert t.n_launches == 1 and t.fast_launches == 1, (t.n_launches, t.fast_launches)
    return y


@pytest.mark.parametrize("rates", list(RATES))
@pytest.mark.parametrize("nt", [1, 2, 5, 8])
@pytest.mark.parametrize("N", [48000, 48002, 48001])
def test_m16_track_counts(xm, gpu, rates, nt, N):
    L, M = RATES[rates]
    B = 11 if nt == 1 else 3          # 11 one-track mixes: the last wave holds 3 of its 8
    x = _xs(B, nt, N, 30000 + 100 * nt)
    q = _q15(nt, _F(N, L, M))
    y = _run(xm, rates, x, q)
    assert bits_equal(y, _ref_s16(x, q, L, M))


@pytest.mark.parametrize("rates", list(RATES))
@pytest.mark.parametrize("nt", [1, 4])
def test_m16_into_f32_mix(xm, gpu, rates, nt):
    """s16 tracks into the f32 mix (XM_MIXER_IN_CONVERT): x * 2^-15 exactly."""
    L, M = RATES[rates]
    N, B = 44100 + 2, 5
    x = _xs(B, nt, N, 31000 + nt)
    ramps = _f32ramps(nt, _F(N, L, M))
    y = _run(xm, rates, x, ramps, fmt="f32", convert_in=True)
    xf = x.astype(np.float32) * np.float32(2.0 ** -15)
    ref, _ = CO.batch_resample_mix_f32(xf, ramps, L, M, threads=4)
    assert bits_equal(y, ref)


@pytest.mark.parametrize("rates", list(RATES))
def test_m16_short_and_edge_lengths(xm, gpu, rates):
    """Clips of one or a few super-periods (the second half of a run may lie
    wholly past the clip), lengths around SP and segment edges."""
    L, M = RATES[rates]
    for N in (2, 8, 30, 146, 148, 160, 162, 294, 296, 322, 4802, 160 * 37 + 6, 1, 7, 161, 4801):
        for nt in (1, 3):
            x = _xs(3, nt, N, 32000 + N + nt)
            q = _q15(nt, _F(N, L, M))
            y = _run(xm, rates, x, q)
            assert bits_equal(y, _ref_s16(x, q, L, M)), (N, nt)


def test_m16_ramps_across_the_half_run(xm, gpu):
    """Q15 ramps that start, end and step in both halves of every lane's run
    (each half has its own gain stepper)."""
    N, B, nt = 96000, 2, 6
    F = _F(N, 160, 147)
    q = [dict(gain0_q15=3000 * t, gain1_q15=32768 - 3000 * t, ramp_start=97 * t + F // 2 - 3000,
              ramp_len=6000 + 11 * t) for t in range(nt)]
    q[3] = dict(gain0_q15=22937, gain1_q15=6554, ramp_start=F // 2 + 5)        # a step just past the middle
    x = _xs(B, nt, N, 33000)
    y = _run(xm, (44100, 48000), x, q)
    assert bits_equal(y, _ref_s16(x, q, 160, 147))


def test_m16_device_strides_and_tables(xm, gpu):
    import torch
    nt, N, B = 5, 9608, 4
    x = _xs(B, nt, N, 34000)
    q = _q15(nt, _F(N, 160, 147))
    ref = _ref_s16(x, q, 160, 147)
    m = xm.Mixer(44100, 48000, 1, "s16", mem="device")
    m.set_tracks(q)
    F = m.out_frames(N)
    ts, ms = N + 6, (N + 6) * nt + 4
    buf = np.zeros(B * ms + 16, np.int16)
    for b in range(B):
        for t in range(nt):
            buf[b * ms + t * ts: b * ms + t * ts + N] = x[b, t].reshape(-1)
    xd = torch.from_numpy(buf).cuda()
    yd = torch.full((B, F + 3), -7, dtype=torch.int16, device="cuda")
    m.process_strided(xd.data_ptr(), ts, ms, yd.data_ptr(), F + 3, B, N)
    torch.cuda.synchronize()
    assert m.timing().fast_launches == 1
    assert bits_equal(yd.cpu().numpy()[:, :F].reshape(B, F, 1), ref)
    assert (yd.cpu().numpy()[:, F:] == -7).all(), "no store past the clip"
    perm = [(3 * t + 2) % nt for t in range(nt)]
    ins = [xd[b * ms + perm[t] * ts:].data_ptr() for b in range(B) for t in range(nt)]
    y2 = torch.full((B, F), -7, dtype=torch.int16, device="cuda")
    outs = [y2[(3 * b + 1) % B].data_ptr() for b in range(B)]
    m.process_ptrs(ins, outs, B, N)
    torch.cuda.synchronize()
    assert m.timing().fast_launches == 1
    ref2 = _ref_s16(x[:, perm], q, 160, 147)
    got = y2.cpu().numpy()
    for b in range(B):
        assert bits_equal(got[(3 * b + 1) % B].reshape(F, 1), ref2[b]), b


def test_m16_config1_batch_production(xm, gpu):
    """2048 mono s16 10 s clips 44.1k -> 48k at unity Q15 gain (config 1's
    own form, batched) in device memory: first and last clip bit-checked
    against the oracle, every output written."""
    import torch
    B, N = 2048, 441000
    m = xm.Mixer(44100, 48000, 1, "s16", mem="device")
    m.set_tracks([dict(gain0_q15=32768)])
    F = m.out_frames(N)
    x = torch.empty((B, N), dtype=torch.int16, device="cuda")
    y = torch.full((B, F), -32768, dtype=torch.int16, device="cuda")
    xm.synth(x.data_ptr(), "s16", SEED, 0, B, 1, N)
    torch.cuda.synchronize()
    m.process_strided(x.data_ptr(), N, N, y.data_ptr(), F, B, N)
    torch.cuda.synchronize()
    assert m.timing().fast_launches == 1
    for b in (0, B - 1):
        assert bits_equal(y[b].cpu().numpy(), CO.resample_s16(x[b].cpu().numpy(), 160, 147)), b
    # every output written: a second run over another sentinel gives the same bits
    y1 = y.clone()
    y.fill_(32767)
    m.process_strided(x.data_ptr(), N, N, y.data_ptr(), F, B, N)
    torch.cuda.synchronize()
    assert bool(torch.equal(y, y1))
    del x, y, y1
    torch.cuda.empty_cache()


@pytest.mark.parametrize("N", [9607, 9609, 9608])
def test_m16_odd_n_device_strides_and_tables(xm, gpu, N):
    """Odd N in device memory: track strides of an odd number of samples (rows
    on every 2-B phase), a scattered pointer table with 2-B aligned entries,
    outputs at odd strides (the exchange-and-store form), both ratios' Q15
    mix and the f32 mix of s16 tracks."""
    import torch
    nt, B = 5, 4
    x = _xs(B, nt, N, 35000 + N)
    for rates, fmt in (((44100, 48000), "s16"), ((48000, 44100), "s16"), ((44100, 48000), "f32")):
        L, M = RATES[rates]
        F = _F(N, L, M)
        q = _q15(nt, F) if fmt == "s16" else _f32ramps(nt, F)
        if fmt == "s16":
            ref = _ref_s16(x, q, L, M)
        else:
            ref, _ = CO.batch_resample_mix_f32(x.astype(np.float32) * np.float32(2.0 ** -15), q, L, M, threads=4)
        m = xm.Mixer(*rates, 1, fmt, mem="device", convert_in=fmt == "f32")
        m.set_tracks(q)
        ts, ms = N + 3, (N + 3) * nt + 1
        buf = np.zeros(B * ms + 16, np.int16)
        for b in range(B):
            for t in range(nt):
                buf[1 + b * ms + t * ts: 1 + b * ms + t * ts + N] = x[b, t].reshape(-1)
        xd = torch.from_numpy(buf).cuda()
        dt = torch.int16 if fmt == "s16" else torch.float32
        yd = torch.full((B, F + 1), -7, dtype=dt, device="cuda")
        m.process_strided(xd[1:].data_ptr(), ts, ms, yd.data_ptr(), F + 1, B, N)
        torch.cuda.synchronize()
        assert m.timing().fast_launches == 1, (rates, fmt)
        assert bits_equal(yd.cpu().numpy()[:, :F].reshape(B, F, 1), ref), (rates, fmt)
        perm = [(3 * t + 2) % nt for t in range(nt)]
        ins = [xd[1 + b * ms + perm[t] * ts:].data_ptr() for b in range(B) for t in range(nt)]
        y2 = torch.full((B, F), -7, dtype=dt, device="cuda")
        outs = [y2[(3 * b + 1) % B].data_ptr() for b in range(B)]
        m.process_ptrs(ins, outs, B, N)
        torch.cuda.synchronize()
        assert m.timing().fast_launches == 1
        ref2 = _ref_s16(x[:, perm], q, L, M) if fmt == "s16" else \
            CO.batch_resample_mix_f32(x[:, perm].astype(np.float32) * np.float32(2.0 ** -15), q, L, M, threads=4)[0]
        got = y2.cpu().numpy()
        for b in range(B):
            assert bits_equal(got[(3 * b + 1) % B].reshape(F, 1), ref2[b]), (rates, fmt, b)


@pytest.mark.parametrize("nt", [1, 5])
def test_m16_odd_n_multi_sp(xm, gpu, monkeypatch, nt):
    """Odd N with lanes walking 2 SP pairs per plane (R = 8): the row delta
    combines with the SP parity in every segment."""
    monkeypatch.setenv("XM_FAST_SPLIT_R", "8")
    N = 147 * (8 * 8 * 5 // 2 + 3) + 37
    B = 11 if nt == 1 else 3
    x = _xs(B, nt, N, 36000 + nt)
    q = _q15(nt, _F(N, 160, 147))
    y = _run(xm, (44100, 48000), x, q)
    assert xm.last_fast_split()[0] == 8
    assert bits_equal(y, _ref_s16(x, q, 160, 147))


def test_m16_config1_batch_odd_n(xm, gpu):
    """Config 1's own form with an odd N, 256 clips, first and last checked,
    every output written."""
    import torch
    B, N = 256, 441001
    m = xm.Mixer(44100, 48000, 1, "s16", mem="device")
    m.set_tracks([dict(gain0_q15=32768)])
    F = m.out_frames(N)
    x = torch.empty((B, N), dtype=torch.int16, device="cuda")
    y = torch.full((B, F), -32768, dtype=torch.int16, device="cuda")
    xm.synth(x.data_ptr(), "s16", SEED, 5, B, 1, N)
    torch.cuda.synchronize()
    m.process_strided(x.data_ptr(), N, N, y.data_ptr(), F, B, N)
    torch.cuda.synchronize()
    assert m.timing().fast_launches == 1
    for b in (0, 1, B - 1):
        assert bits_equal(y[b].cpu().numpy(), CO.resample_s16(x[b].cpu().numpy(), 160, 147)), b
    y1 = y.clone()
    y.fill_(32767)
    m.process_strided(x.data_ptr(), N, N, y.data_ptr(), F, B, N)
    torch.cuda.synchronize()
    assert bool(torch.equal(y, y1))
    del x, y, y1
    torch.cuda.empty_cache()
