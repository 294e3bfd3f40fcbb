"""Mono f32 mixes on the fused kernel (the MONO instantiations, VERDICT r2
item 4): a lane's run of super-periods is cut in two halves that ride as the
two planes of the planar kernel, each with its own clip edges and gains, and
the store step writes the two mono outputs half a run apart.  Both table
ratios, 1-track rows (batches of mono clips) and 2-8-track mixes, odd and
tiny frame counts, ramps whose edges fall in either half, strided device
memory and pointer tables.  Every case must run on the fused kernel
(XmMixerTiming.fast_launches == 1) and equal the C oracle bit for bit."""
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


def _ramps(nt, F):
    out = []
    for t in range(nt):
        k = t % 6
        if k == 0:
            out.append(dict(gain0=0.9 - 0.05 * t))
        elif k == 1:
            out.append(dict(gain0=0.0, gain1=0.8, ramp_start=37 * t, ramp_len=max(1, F // 3)))
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
    return np.stack([np.stack([O.gen_f32(SEED, base + 16 * b + t, 1, N) for t in range(nt)]) for b in range(B)])


def _run(xm, rates, x, ramps):
    m = xm.Mixer(*rates, 1, "f32")
    m.set_tracks(ramps)
    y = m.process(x)
    t = m.timing()
    assert t.n_launches == 1 and t.fast_launches == m.fused, (t.n_launches, t.fast_launches)   # fused: GPU handles
    return y


@pytest.mark.parametrize("rates", list(RATES))
@pytest.mark.parametrize("nt", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("N", [48000, 48001])
def test_mono_track_counts(xm, gpu, rates, nt, N):
    L, M = RATES[rates]
    B = 11 if nt == 1 else 3          # 11 one-track mixes: the last wave holds 3 of its 8
    x = _x(B, nt, N, 20000 + 100 * nt)
    ramps = _ramps(nt, _F(N, L, M))
    y = _run(xm, rates, x, ramps)
    ref, _ = CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)
    assert bits_equal(y, ref)


@pytest.mark.parametrize("rates", list(RATES))
@pytest.mark.parametrize("N", [1, 7, 146, 160, 161, 321, 4801, 160 * 37 + 5])
def test_mono_short_and_edge_lengths(xm, gpu, rates, N):
    """Clips of one or a few super-periods: the second half of a run may lie
    wholly past the clip (its outputs dropped, its loads zero-filled)."""
    L, M = RATES[rates]
    for nt in (1, 4):
        x = _x(3, nt, N, 21000 + N + nt)
        ramps = _ramps(nt, _F(N, L, M))
        y = _run(xm, rates, x, ramps)
        ref, _ = CO.batch_resample_mix_f32(x, ramps, L, M, threads=4)
        assert bits_equal(y, ref), nt


def test_mono_ramp_across_the_half_run(xm, gpu):
    """Ramps that start, end and step in both halves of every lane's run."""
    N, B, nt = 96000, 2, 6
    F = _F(N, 147, 160)
    ramps = [dict(gain0=0.1 * t, gain1=1.0 - 0.1 * t, ramp_start=97 * t + F // 2 - 3000, ramp_len=6000 + 11 * t)
             for t in range(nt)]
    ramps[3] = dict(gain0=0.7, gain1=0.2, ramp_start=F // 2 + 5)          # a step just past the middle
    x = _x(B, nt, N, 22000)
    y = _run(xm, (48000, 44100), x, ramps)
    ref, _ = CO.batch_resample_mix_f32(x, ramps, 147, 160, threads=4)
    assert bits_equal(y, ref)


def test_mono_device_strides_and_tables(xm, gpu):
    import torch
    nt, N, B = 5, 9607, 4
    x = _x(B, nt, N, 23000)
    ramps = _ramps(nt, _F(N, 147, 160))
    ref, _ = CO.batch_resample_mix_f32(x, ramps, 147, 160, threads=4)
    m = xm.Mixer(48000, 44100, 1, "f32", mem="device")
    m.set_tracks(ramps)
    F = m.out_frames(N)
    ts, ms = N + 5, (N + 5) * nt + 3
    buf = np.zeros(B * ms + 16, np.float32)
    for b in range(B):
        for t in range(nt):
            buf[b * ms + t * ts: b * ms + t * ts + N] = x[b, t].reshape(-1)
    xd = torch.from_numpy(buf).cuda()
    yd = torch.full((B, F + 3), float("nan"), dtype=torch.float32, device="cuda")
    m.process_strided(xd.data_ptr(), ts, ms, yd.data_ptr(), F + 3, B, N)
    torch.cuda.synchronize()
    assert m.timing().fast_launches == m.fused
    assert bits_equal(yd.cpu().numpy()[:, :F].reshape(B, F, 1), ref)
    perm = [(3 * t + 2) % nt for t in range(nt)]
    ins = [xd[b * ms + perm[t] * ts:].data_ptr() for b in range(B) for t in range(nt)]
    y2 = torch.full((B, F), float("nan"), dtype=torch.float32, device="cuda")
    outs = [y2[(3 * b + 1) % B].data_ptr() for b in range(B)]
    m.process_ptrs(ins, outs, B, N)
    torch.cuda.synchronize()
    assert m.timing().fast_launches == m.fused
    ref2, _ = CO.batch_resample_mix_f32(x[:, perm], ramps, 147, 160, threads=4)
    got = y2.cpu().numpy()
    for b in range(B):
        assert bits_equal(got[(3 * b + 1) % B].reshape(F, 1), ref2[b]), b


def test_mono_clip_batch_production(xm, gpu):
    """1024 mono 10 s clips 44.1k -> 48k at unity gain (config 1's shape,
    batched) in device memory: first and last clip bit-checked, nothing left
    unwritten."""
    import torch
    B, N = 1024, 441000
    m = xm.Mixer(44100, 48000, 1, "f32", mem="device")
    m.set_tracks([dict(gain0=1.0)])
    F = m.out_frames(N)
    x = torch.empty((B, N), dtype=torch.float32, device="cuda")
    y = torch.full((B, F), float("nan"), dtype=torch.float32, device="cuda")
    xm.synth(x.data_ptr(), "f32", SEED, 0, B, 1, N)
    torch.cuda.synchronize()
    m.process_strided(x.data_ptr(), N, N, y.data_ptr(), F, B, N)
    torch.cuda.synchronize()
    assert m.timing().fast_launches == m.fused
    for b in (0, B - 1):
        assert bits_equal(y[b].cpu().numpy(), CO.resample_f32(x[b].cpu().numpy(), 160, 147)), b
    assert not bool(y.isnan().any())
