"""GPU parity of timeline mixes: tracks of
different input rates and lengths, each placed at its own output frame.
Oracle: each track resampled on its own by the C restatement (pinned to
scipy), zero-padded to its place, then the ordered-sum mix restatement."""
import numpy as np
import pytest

from conftest import bits_equal, ulp_diff

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED


def _ratio(fi, fo):
    from math import gcd
    g = gcd(fi, fo)
    return fo // g, fi // g


def _oracle(xb, rates, offsets, ramps, out_rate, out_frames, s16):
    placed = []
    for x, r, off in zip(xb, rates, offsets):
        L, M = _ratio(r, out_rate)
        if L == M:
            y = x
        else:
            y = CO.resample_s16(x, L, M) if s16 else CO.resample_f32(x, L, M)
        p = np.zeros((out_frames, x.shape[1]), x.dtype)
        lo, hi = max(off, 0), min(off + len(y), out_frames)
        if hi > lo:
            p[lo:hi] = y[lo - off:hi - off]
        placed.append(p)
    return CO.mix_s16(placed, ramps) if s16 else CO.mix_f32(placed, ramps)


RAMPS = [dict(gain0=0.8), dict(gain0=0.0, gain1=1.0, ramp_start=500, ramp_len=2000),
         dict(gain0=1.0, gain1=0.25, ramp_start=3000, ramp_len=900), dict(gain0=0.6),
         dict(mode=1, ramp_start=1000, ramp_len=700)]


@pytest.mark.parametrize("channels", [1, 2])
def test_timeline_f32_mixed_rates_into_44k(xm, gpu, channels):
    out_rate = 44100
    rates = [48000, 44100, 16000, 22050, 48000]
    lens = [4800 + 7, 3000, 1600 + 3, 2205, 9000]
    offsets = [0, 1234, -300, 4000, 9000]          # head cut, gaps, a tail past the end
    out_frames = 10000
    B = 2
    xs = [np.stack([O.gen_f32(SEED, 4000 + 8 * b + t, channels, n) for b in range(B)])
          for t, n in enumerate(lens)]
    m = xm.Mixer(48000, out_rate, channels, "f32")
    m.set_tracks([dict(r, in_rate=rt) for r, rt in zip(RAMPS, rates)])
    y = m.process_timeline(xs, offsets, out_frames)
    for b in range(B):
        ref = _oracle([x[b] for x in xs], rates, offsets, RAMPS, out_rate, out_frames, False)
        assert bits_equal(y[b], ref), (b, ulp_diff(y[b], ref))
    with pytest.raises(xm.XmError):   # uniform-length calls refuse mixed rates
        m.process(np.zeros((1, 5, 100, channels), np.float32))


def test_timeline_s16_voice_bgm_48k(xm, gpu):
    """BGM at 48k, voice at 44.1k and 16k, s16 Q15 with saturation."""
    out_rate = 48000
    rates = [48000, 44100, 16000]
    lens = [12000, 4410 + 1, 1600]
    offsets = [0, 2000, 7000]
    xs = [np.stack([O.gen_s16(SEED, 4100 + 8 * b + t, 2, n) for b in range(3)]) for t, n in enumerate(lens)]
    ramps = [dict(gain0=1.5), dict(gain0=1.9, gain1=0.5, ramp_start=2500, ramp_len=3000), dict(gain0=1.0)]
    ramps = [dict(r, gain0_q15=int(round(r["gain0"] * 32768)),
                  gain1_q15=int(round(r.get("gain1", r["gain0"]) * 32768))) for r in ramps]
    m = xm.Mixer(48000, out_rate, 2, "s16")
    m.set_tracks([dict(r, in_rate=rt) for r, rt in zip(ramps, rates)])
    y = m.process_timeline(xs, offsets, 12000)
    for b in range(3):
        ref = _oracle([x[b] for x in xs], rates, offsets, ramps, out_rate, 12000, True)
        assert bits_equal(y[b], ref), b


def test_timeline_same_rate_equals_process(xm, gpu):
    """All tracks at the mixer rate, offset 0, equal lengths: process_timeline == process."""
    B, N = 2, 9600 + 5
    x = np.stack([np.stack([O.gen_f32(SEED, 4200 + 8 * b + t, 2, N) for t in range(5)]) for b in range(B)])
    m = xm.Mixer(48000, 44100, 2, "f32")
    m.set_tracks(RAMPS)
    want = m.process(x)
    got = m.process_timeline([x[:, t] for t in range(5)], [0] * 5, m.out_frames(N))
    assert bits_equal(got, want)


def test_timeline_device_memory(xm, gpu):
    import ctypes
    import torch
    rates = [48000, 16000]
    lens = [4800, 1600]
    xs = [np.stack([O.gen_f32(SEED, 4300 + t, 2, n)]) for t, n in enumerate(lens)]
    host = xm.Mixer(48000, 44100, 2, "f32")
    host.set_tracks([dict(gain0=0.5, in_rate=rates[0]), dict(gain0=0.7, in_rate=rates[1])])
    want = host.process_timeline(xs, [10, 100], 5000)
    dev = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    dev.set_tracks([dict(gain0=0.5, in_rate=rates[0]), dict(gain0=0.7, in_rate=rates[1])])
    xd = [torch.from_numpy(x[0]).cuda() for x in xs]
    yd = torch.zeros((5000, 2), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ins = (ctypes.c_void_p * 2)(*[t.data_ptr() for t in xd])
    pl = (xm.XmTrackPlacement * 2)(xm.XmTrackPlacement(10, 4800), xm.XmTrackPlacement(100, 1600))
    outs = (ctypes.c_void_p * 1)(yd.data_ptr())
    assert xm._lib.xm_audio_mixer_process_timeline(dev._h, ins, pl, outs, 1, 5000) == 0
    assert bits_equal(yd.cpu().numpy(), want[0])


def test_rate_table_cache_follows_track_list(xm, gpu):
    """Per-track rate tables are kept only while a track uses them: a handle
    that sees more than 64 distinct rates over its life keeps working, and
    the mix after many swaps equals a fresh handle's."""
    m = xm.Mixer(44100, 48000, 1, "f32")
    for r in range(8000, 8000 + 70 * 100, 100):        # 140 distinct rates, two at a time
        m.set_tracks([dict(in_rate=r), dict(in_rate=r + 50, gain0=0.5)])
    x = [np.stack([O.gen_f32(SEED, 7700 + b, 1, 3000)]) for b in range(2)]
    tracks = [dict(in_rate=22050, gain0=0.7), dict(in_rate=16000, gain0=0.4)]
    m.set_tracks(tracks)
    y = m.process_timeline(x, [0, 100], 7000)
    f = xm.Mixer(44100, 48000, 1, "f32")
    f.set_tracks(tracks)
    assert bits_equal(y, f.process_timeline(x, [0, 100], 7000))
