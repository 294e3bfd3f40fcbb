"""GPU parity of the streaming entry points:
xm_audio_mixer_stream_{begin,push,flush} and xm_effects_{stream_reset,
process_stream}.  A signal split into ragged blocks (1-frame, empty, shorter
than the filter history, longer than a kernel chunk) must give, bit for bit,
the oracle's output for the whole signal — and so the whole-signal GPU call."""
import numpy as np
import pytest

from conftest import bits_equal, golden, ulp_diff

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED

RAMPS8 = [
    dict(gain0=0.9), dict(gain0=0.0, gain1=0.8, ramp_start=100, ramp_len=3000),
    dict(gain0=0.7, gain1=0.2, ramp_start=2000, ramp_len=441), dict(gain0=0.5),
    dict(mode=1, ramp_start=3000, ramp_len=800), dict(gain0=0.0, gain1=1.0, ramp_start=3000, ramp_len=800),
    dict(gain0=1.25, gain1=0.75, ramp_start=0, ramp_len=4410), dict(gain0=0.3, gain1=0.6, ramp_start=4000),
]


def _blocks(N, pattern):
    """Block sizes summing to N: the pattern, then 4099-frame blocks, then the rest."""
    out, left = [], N
    for b in pattern:
        b = min(b, left)
        out.append(b)
        left -= b
    while left > 0:
        out.append(min(4099, left))
        left -= out[-1]
    return out


PATTERNS = {
    "ragged": [0, 1, 5, 137, 0, 1000, 17, 2, 33],
    "single_frames": [1] * 40 + [0, 3],
    "one_block": [10 ** 9],
}


def _stream_mix(m, x, sizes):
    B = x.shape[0]
    m.stream_begin(B)
    outs, p = [], 0
    for n in sizes:
        outs.append(m.stream_push(x[:, :, p:p + n]))
        p += n
    assert p == x.shape[2]
    outs.append(m.stream_flush())
    return np.concatenate(outs, axis=1)


@pytest.mark.parametrize("pattern", sorted(PATTERNS))
def test_stream_resample_mix_f32_48_to_44(xm, gpu, pattern):
    B, ntr, N = 2, 8, 9600 + 77
    x = np.stack([np.stack([O.gen_f32(SEED, 3000 + 8 * b + t, 2, N) for t in range(ntr)]) for b in range(B)])
    m = xm.Mixer(48000, 44100, 2, "f32")
    m.set_tracks(RAMPS8)
    y = _stream_mix(m, x, _blocks(N, PATTERNS[pattern]))
    ref, _ = CO.batch_resample_mix_f32(x, RAMPS8, 147, 160, threads=4)
    assert y.shape == ref.shape
    assert bits_equal(y, ref), f"max ulp {ulp_diff(y, ref)}"
    assert bits_equal(y, m.process(x))


def test_stream_resample_s16_44_to_48_mono(xm, gpu):
    N = 8820 + 3
    x = np.stack([O.gen_s16(SEED, 3100 + t, 1, N) for t in range(3)])[None]
    ramps = RAMPS8[1:4]
    m = xm.Mixer(44100, 48000, 1, "s16")
    m.set_tracks(ramps)
    y = _stream_mix(m, x, _blocks(N, PATTERNS["ragged"]))
    ref = CO.resample_mix_s16(list(x[0]), ramps, 160, 147)
    assert bits_equal(y[0], ref.reshape(y[0].shape))


def test_stream_mix_s16_same_rate(xm, gpu):
    """Config 3 mixer (no resampling) streamed: gains at the absolute frame."""
    N = 6000 + 5
    x = np.stack([np.stack([O.gen_s16(SEED, 3200 + 8 * b + t, 2, N) for t in range(8)]) for b in range(2)])
    m = xm.Mixer(48000, 48000, 2, "s16")
    m.set_tracks(RAMPS8)
    y = _stream_mix(m, x, _blocks(N, [0, 1, 7, 301, 2, 999]))
    for b in range(2):
        assert bits_equal(y[b], CO.mix_s16(list(x[b]), RAMPS8).reshape(y[b].shape))


def test_stream_device_memory_strided(xm, gpu):
    import torch
    B, ntr, N = 2, 8, 9600
    x = np.stack([np.stack([O.gen_f32(SEED, 3300 + 8 * b + t, 2, N) for t in range(ntr)]) for b in range(B)])
    ref = xm.Mixer(48000, 44100, 2, "f32")
    ref.set_tracks(RAMPS8)
    want = ref.process(x)
    dev = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    dev.set_tracks(RAMPS8)
    F = dev.out_frames(N)
    xd = torch.from_numpy(x).cuda()
    yd = torch.zeros((B, F, 2), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    dev.stream_begin(B)
    got = 0
    for p0, n in zip(np.cumsum([0] + _blocks(N, [3, 500, 1])[:-1]), _blocks(N, [3, 500, 1])):
        got += dev.stream_push_strided(xd[:, :, int(p0):].data_ptr(), N * 2, ntr * N * 2, n,
                                       yd[:, got:].data_ptr(), F * 2, F - got)
    got += dev.stream_flush_strided(yd[:, got:].data_ptr(), F * 2, F - got)
    assert got == F
    assert bits_equal(yd.cpu().numpy(), want)


def test_stream_mixer_errors(xm, gpu):
    import ctypes
    m = xm.Mixer(48000, 44100, 2, "f32")
    m._st_batch = 1
    with pytest.raises(xm.XmError):   # push before begin
        m.stream_push(np.zeros((1, 1, 10, 2), np.float32))
    m.stream_begin(1)
    x = np.zeros((1, 1, 4000, 2), np.float32)
    y = np.zeros((1, 10, 2), np.float32)
    n = ctypes.c_size_t(0)
    rc = xm._lib.xm_audio_mixer_stream_push(m._h, x.ctypes.data, 8000, 8000, 4000, y.ctypes.data, 20, 10,
                                           ctypes.byref(n))
    assert rc == xm.XM_EINVAL and n.value == 0   # out_cap too small: nothing consumed
    assert m.stream_push(x).shape[1] == -(-4000 * 147 // 160) - 11   # ceil(L*R/M) - rm
    m.set_tracks([dict(gain0=1.0), dict(gain0=1.0)])
    with pytest.raises(xm.XmError):   # track count changed mid-stream
        m.stream_push(np.zeros((1, 2, 10, 2), np.float32))


@pytest.mark.parametrize("channels", [1, 2])
@pytest.mark.parametrize("pattern", ["ragged", "single_frames", "chunk_edges"])
def test_effects_stream_chain(xm, gpu, channels, pattern):
    """biquad x3 -> FIR 63 -> biquad x2, streamed, against the whole-signal oracle."""
    z = golden("effects.npz")
    B, N = 5, 6000 + 11
    x = np.stack([O.gen_f32(SEED, 3400 + b, channels, N) for b in range(B)])
    e = xm.Effects(48000, channels)
    for s in z["sos"][:3]:
        e.add_biquad(s)
    e.add_fir(z["h63"])
    for s in z["sos"][3:]:
        e.add_biquad(s)
    pat = {"ragged": PATTERNS["ragged"], "single_frames": PATTERNS["single_frames"],
           "chunk_edges": [31, 32, 33, 62, 64, 65, 1, 127]}[pattern]
    e.stream_reset(B)
    outs, p = [], 0
    for i, n in enumerate(_blocks(N, pat)):
        outs.append(e.process_stream(x[:, p:p + n], inplace=(i % 3 == 2)))
        p += n
    y = np.concatenate(outs, axis=1)
    for b in range(B):
        r = CO.biquad_f32(CO.fir_f32(CO.biquad_f32(x[b], z["sos"][:3]), z["h63"]), z["sos"][3:])
        assert bits_equal(y[b], r), (b, ulp_diff(y[b], r))
    # the stream ends when the chain changes; a reset restarts from zero state
    e.add_fir(np.array([1.0], np.float32))
    with pytest.raises(xm.XmError):
        e.process_stream(x[:, :10])
    e.stream_reset(B)
    y2 = e.process_stream(x)
    assert bits_equal(y2, e.process(x))


def test_effects_stream_errors(xm, gpu):
    e = xm.Effects(48000, 2)
    e.add_biquad(golden("effects.npz")["sos"][0])
    x = np.zeros((2, 100, 2), np.float32)
    with pytest.raises(xm.XmError):   # no reset
        e.process_stream(x)
    e.stream_reset(3)
    with pytest.raises(xm.XmError):   # clip count differs from the reset
        e.process_stream(x)


def test_stream_device_1frame_reused_buffer(xm, gpu):
    """Device-memory pushes that release no output (1-frame blocks) are still
    synchronous on the handle's own stream: the caller refills ONE input
    buffer between pushes from another stream, and the stream must have read
    every block before the push returned (the nout == 0 path)."""
    import torch
    B, ntr, N = 2, 8, 700
    x = np.stack([np.stack([O.gen_f32(SEED, 4100 + 8 * b + t, 2, N) for t in range(ntr)]) for b in range(B)])
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    m.set_tracks(RAMPS8)
    h = xm.Mixer(48000, 44100, 2, "f32")
    h.set_tracks(RAMPS8)
    want = h.process(x)
    F = h.out_frames(N)
    blk = torch.empty((B, ntr, 1, 2), dtype=torch.float32, device="cuda")
    out = torch.zeros((B, F, 2), dtype=torch.float32, device="cuda")
    side = torch.cuda.Stream()
    m.stream_begin(B)
    pos = 0
    for f in range(N):
        with torch.cuda.stream(side):     # refill the one buffer from another stream
            blk.copy_(torch.from_numpy(x[:, :, f:f + 1]).pin_memory().cuda(non_blocking=True), non_blocking=True)
        side.synchronize()
        o = out[:, pos:]
        pos += m.stream_push_strided(blk.data_ptr(), 2, ntr * 2, 1, o.data_ptr(), F * 2, F - pos)
    o = out[:, pos:]
    pos += m.stream_flush_strided(o.data_ptr(), F * 2, F - pos)
    assert pos == F
    assert bits_equal(out.cpu().numpy(), want)


def test_stream_mixed_rates_mid_stream(xm, gpu):
    """set_tracks with a per-track rate after stream_begin (same track count):
    the next push refuses (XM_ENOSYS) instead of ignoring the rate."""
    m = xm.Mixer(48000, 44100, 2, "f32")
    m.set_tracks(RAMPS8[:2])
    m.stream_begin(1)
    m.stream_push(np.zeros((1, 2, 100, 2), np.float32))
    m.set_tracks([dict(RAMPS8[0]), dict(RAMPS8[1], in_rate=44100)])
    with pytest.raises(xm.XmError) as e:
        m.stream_push(np.zeros((1, 2, 100, 2), np.float32))
    assert e.value.code == xm.XM_ENOSYS


@pytest.mark.parametrize("pattern", ["big_ragged", "sp_edges", "one_block"])
def test_stream_fused_window_path(xm, gpu, pattern):
    """48k->44.1k stereo 8-track streams run their super-period-aligned bulk
    on the fused kernel (a window job: input at the window frame of the
    first aligned output, 32 real lead-in frames, ramps shifted) and the head
    before it on the generic kernel; any split equals the whole-signal call."""
    N = 48000 + 77
    x = np.stack([np.stack([O.gen_f32(SEED, 6100 + 8 * b + t, 2, N) for t in range(8)]) for b in range(2)])
    m = xm.Mixer(48000, 44100, 2, "f32")
    m.set_tracks(RAMPS8)
    want = m.process(x)
    sizes = {"big_ragged": _blocks(N, [7001, 1, 0, 12345, 160 * 30 + 1, 3]),
             "sp_edges": _blocks(N, [160 * 5, 160 * 20 + 32, 160 * 7 - 1, 160 * 40]),
             "one_block": [N]}[pattern]
    m.stream_begin(2)
    outs, p, fast = [], 0, 0
    for n in sizes:
        outs.append(m.stream_push(x[:, :, p:p + n]))
        fast += m.timing().fast_launches
        p += n
    outs.append(m.stream_flush())
    fast += m.timing().fast_launches
    assert fast >= 1, "the fused kernel never ran"
    assert bits_equal(np.concatenate(outs, axis=1), want)


def test_stream_fused_window_split_mode(xm, gpu):
    """1-track unity-gain streams of 16 clips (split mode) in blocks; 9 clips
    (a remainder) stay on the generic kernel, with the same bits."""
    N, B = 9600 * 3 + 5, 16
    x = np.stack([O.gen_f32(SEED, 6200 + b, 2, N)[None] for b in range(B)])
    m = xm.Mixer(48000, 44100, 2, "f32")
    m.set_tracks([dict(gain0=1.0)])
    want = m.process(x)
    m.stream_begin(B)
    outs, p, fast = [], 0, 0
    for n in _blocks(N, [9000, 7, 10000]):
        outs.append(m.stream_push(x[:, :, p:p + n]))
        fast += m.timing().fast_launches
        p += n
    outs.append(m.stream_flush())
    assert fast >= 1
    assert bits_equal(np.concatenate(outs, axis=1), want)
    x9 = x[:9]
    m.stream_begin(9)
    o9 = [m.stream_push(x9[:, :, :15000]), m.stream_push(x9[:, :, 15000:]), m.stream_flush()]
    assert bits_equal(np.concatenate(o9, axis=1), want[:9])


@pytest.mark.parametrize("ntr", [8, 4, 12])
def test_stream_device_direct_bulk(xm, gpu, ntr):
    """Device-memory pushes of a 48k->44.1k stream: each large block's
    super-period-aligned bulk runs on the fused kernel straight from the
    caller's block (no copy into the window); the head before it and small
    blocks run from the window.  Ragged blocks, one and several bulk
    launches, a block too small for a bulk, 4 / 8 / 12 tracks: the
    concatenated releases equal the whole-signal call bit for bit."""
    import torch
    B, N = 3, 48000 + 77
    x = np.stack([np.stack([O.gen_f32(SEED, 6300 + 16 * b + t, 2, N) for t in range(ntr)]) for b in range(B)])
    ramps = (RAMPS8 * 2)[:ntr]
    h = xm.Mixer(48000, 44100, 2, "f32")
    h.set_tracks(ramps)
    want = h.process(x)
    F = h.out_frames(N)
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    m.set_tracks(ramps)
    xd = torch.from_numpy(x).cuda()
    yd = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    m.stream_begin(B)
    got, p, fast = 0, 0, 0
    for n in _blocks(N, [12001, 5, 700, 20000, 3]):
        blk = xd[:, :, p:p + n].contiguous()        # the caller's block in its own buffer
        got += m.stream_push_strided(blk.data_ptr(), n * 2, ntr * n * 2, n, yd[:, got:].data_ptr(), F * 2, F - got)
        fast += m.timing().fast_launches
        p += n
        del blk
    got += m.stream_flush_strided(yd[:, got:].data_ptr(), F * 2, F - got)
    assert got == F
    assert fast >= 2, fast
    assert bits_equal(yd.cpu().numpy(), want)


@pytest.mark.parametrize("pattern", ["big_ragged", "sp_edges", "one_block"])
@pytest.mark.parametrize("ntr", [8, 3, 12])
def test_stream_fused_window_path_44_to_48(xm, gpu, pattern, ntr):
    """44.1k->48k stereo streams (round 5): the super-period-aligned bulk of a
    release runs on the fused UP kernel as a window job (input at the window
    frame 147*ob/160 of the first aligned output, 32 real lead-in frames, SP
    origins alternating parity), the head on the generic kernel; any split
    equals the whole-signal call bit for bit."""
    N = 44100 + 77
    x = np.stack([np.stack([O.gen_f32(SEED, 6400 + 16 * b + t, 2, N) for t in range(ntr)]) for b in range(2)])
    ramps = (RAMPS8 * 2)[:ntr]
    m = xm.Mixer(44100, 48000, 2, "f32")
    m.set_tracks(ramps)
    want = m.process(x)
    sizes = {"big_ragged": _blocks(N, [7001, 1, 0, 12345, 147 * 30 + 1, 3]),
             "sp_edges": _blocks(N, [147 * 5, 147 * 20 + 32, 147 * 7 - 1, 147 * 40]),
             "one_block": [N]}[pattern]
    m.stream_begin(2)
    outs, p, fast = [], 0, 0
    for n in sizes:
        outs.append(m.stream_push(x[:, :, p:p + n]))
        fast += m.timing().fast_launches
        p += n
    outs.append(m.stream_flush())
    fast += m.timing().fast_launches
    assert fast >= 1, "the fused kernel never ran"
    assert bits_equal(np.concatenate(outs, axis=1), want)


@pytest.mark.parametrize("ntr", [8, 5])
def test_stream_device_direct_bulk_44_to_48(xm, gpu, ntr):
    """Device-memory pushes of a 44.1k->48k stream: each large block's aligned
    bulk on the fused UP kernel straight from the caller's block."""
    import torch
    B, N = 3, 44100 + 77
    x = np.stack([np.stack([O.gen_f32(SEED, 6500 + 16 * b + t, 2, N) for t in range(ntr)]) for b in range(B)])
    ramps = (RAMPS8 * 2)[:ntr]
    h = xm.Mixer(44100, 48000, 2, "f32")
    h.set_tracks(ramps)
    want = h.process(x)
    F = h.out_frames(N)
    m = xm.Mixer(44100, 48000, 2, "f32", mem="device")
    m.set_tracks(ramps)
    xd = torch.from_numpy(x).cuda()
    yd = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    m.stream_begin(B)
    got, p, fast = 0, 0, 0
    for n in _blocks(N, [12001, 5, 700, 20000, 3]):
        blk = xd[:, :, p:p + n].contiguous()
        got += m.stream_push_strided(blk.data_ptr(), n * 2, ntr * n * 2, n, yd[:, got:].data_ptr(), F * 2, F - got)
        fast += m.timing().fast_launches
        p += n
        del blk
    got += m.stream_flush_strided(yd[:, got:].data_ptr(), F * 2, F - got)
    assert got == F
    assert fast >= 2, fast
    assert bits_equal(yd.cpu().numpy(), want)
