"""Multi-device mixer handles (SURVEY.md §8(b) n_devices, §8(e)): one
single-device handle and one worker thread per entry of the device list,
batches cut into contiguous mix blocks, and config 5's exchange inside the
library.  On a one-GPU box the list repeats device 0 ([0, 0], [0, 0, 0]):
the blocks still run on separate sub-handles, streams and threads, so the
sharding logic is exercised; the results must equal a one-device handle
(and the oracle) bit for bit.  A [0] list runs config 5's RCCL path with a
one-device communicator."""
import numpy as np
import pytest

from conftest import bits_equal, golden

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


def _x(B, ntr, N, base=0):
    return np.stack([np.stack([O.gen_f32(SEED, base + 8 * b + t, 2, N) for t in range(ntr)]) for b in range(B)])


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_multi_host_batch_equals_single(xm, gpu, devices):
    B, N = 5, 9600 + 11                   # 5 mixes over 2 / 3 devices: ragged blocks
    x = _x(B, 8, N, 100)
    one = xm.Mixer(48000, 44100, 2, "f32")
    one.set_tracks(RAMPS8)
    want = one.process(x)
    m = xm.Mixer(48000, 44100, 2, "f32", devices=devices)
    assert m.n_devices() == len(devices)
    m.set_tracks(RAMPS8)
    y = m.process(x)
    assert bits_equal(y, want)
    ref, _ = CO.batch_resample_mix_f32(x, RAMPS8, 147, 160, threads=4)
    assert bits_equal(y, ref)
    t = m.timing()
    assert t.n_launches >= min(B, len(devices)) and t.kernel_ms > 0
    # a crossfade set on the multi-device handle reaches every device
    m.set_crossfade(4, 5, 1000, 2000)
    one.set_crossfade(4, 5, 1000, 2000)
    assert bits_equal(m.process(x), one.process(x))


def test_multi_device_memory_ptrs_and_sharded(xm, gpu):
    import torch
    B, N = 6, 4800
    x = _x(B, 8, N, 300)
    one = xm.Mixer(48000, 44100, 2, "f32")
    one.set_tracks(RAMPS8)
    want = one.process(x)
    F = one.out_frames(N)
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device", devices=[0, 0])
    m.set_tracks(RAMPS8)
    xd = torch.from_numpy(x).cuda()
    y = torch.zeros((B, F, 2), dtype=torch.float32, device="cuda")
    ins = [xd[b, t].data_ptr() for b in range(B) for t in range(8)]
    outs = [y[b].data_ptr() for b in range(B)]
    m.process_ptrs(ins, outs, B, N)
    assert bits_equal(y.cpu().numpy(), want)
    # resident shards: device d's block at its own base pointer
    y2 = torch.zeros_like(y)
    m.process_sharded([xd[0].data_ptr(), xd[4].data_ptr()], N * 2, 8 * N * 2,
                      [y2[0].data_ptr(), y2[4].data_ptr()], F * 2, [4, 2], N)
    assert bits_equal(y2.cpu().numpy(), want)
    with pytest.raises(xm.XmError) as e:        # one base pointer cannot span devices
        m.process_strided(xd.data_ptr(), N * 2, 8 * N * 2, y.data_ptr(), F * 2, B, N)
    assert e.value.code == xm.XM_EINVAL
    with pytest.raises(xm.XmError) as e:
        m.set_stream(torch.cuda.current_stream().cuda_stream)
    assert e.value.code == xm.XM_ENOSYS


def test_multi_track_effects_config4_shape(xm, gpu):
    """Config 4's chain (resample -> 5-band EQ -> gain -> mix) on a
    multi-device handle: the effects chain is cloned onto every device."""
    z = golden("effects.npz")
    B, N = 3, 4800 + 7
    x = _x(B, 8, N, 500)
    fx = xm.Effects(44100, 2)
    for s in z["sos"]:
        fx.add_biquad(s)
    one = xm.Mixer(48000, 44100, 2, "f32")
    one.set_tracks(RAMPS8)
    one.set_track_effects(fx)
    want = one.process(x)
    m = xm.Mixer(48000, 44100, 2, "f32", devices=[0, 0, 0])
    m.set_tracks(RAMPS8)
    m.set_track_effects(fx)
    assert bits_equal(m.process(x), want)
    for b in range(B):                   # and the oracle's chain
        r = [CO.biquad_f32(CO.resample_f32(x[b, t], 147, 160), z["sos"]) for t in range(8)]
        assert bits_equal(want[b], CO.mix_f32(r, RAMPS8)), b
    m.set_track_effects(None)
    one.set_track_effects(None)
    assert bits_equal(m.process(x), one.process(x))


def test_multi_streaming_and_timeline(xm, gpu):
    B, N = 4, 6000
    x = _x(B, 8, N, 700)
    one = xm.Mixer(48000, 44100, 2, "f32")
    one.set_tracks(RAMPS8)
    want = one.process(x)
    m = xm.Mixer(48000, 44100, 2, "f32", devices=[0, 0, 0])
    m.set_tracks(RAMPS8)
    m.stream_begin(B)
    outs, p = [], 0
    for n in (1, 0, 777, 1500, 3722):
        outs.append(m.stream_push(x[:, :, p:p + n]))
        p += n
    outs.append(m.stream_flush())
    assert bits_equal(np.concatenate(outs, axis=1), want)
    tracks = [x[:, t, : 3000 + 100 * t] for t in range(8)]
    offs = [0, 50, -20, 400, 0, 0, 900, 10]
    assert bits_equal(m.process_timeline(tracks, offs, 4000), one.process_timeline(tracks, offs, 4000))


def test_config_n_devices_range(xm, gpu):
    ndev = xm.device_count()
    m = xm.Mixer(48000, 44100, 2, "f32", n_devices=1)
    assert m.n_devices() == 1
    if ndev == 1:
        with pytest.raises(xm.XmError) as e:      # devices 0 .. 1 on a one-GPU box
            xm.Mixer(48000, 44100, 2, "f32", n_devices=2)
        assert e.value.code == xm.XM_EDEVICE
    with pytest.raises(xm.XmError) as e:
        xm.Mixer(48000, 44100, 2, "f32", devices=[0, ndev])
    assert e.value.code == xm.XM_EDEVICE
    s = xm.Mixer(48000, 48000, 2, "s16", mem="device", devices=[0, 0])
    with pytest.raises(xm.XmError) as e:
        s.process_partial_strided(1, 2, 2, 1, 2, 1, 1)
    assert e.value.code == xm.XM_ENOSYS


_R = [(32768, 32768, 0, 0, 0), (0, 32768, 100, 20000, 0), (65535, 100, 0, 9600, 0), (16384, 16384, 0, 0, 0),
      (0, 0, 5000, 900, 1), (0, 32768, 5000, 900, 0), (40000, 3, 7000, 13, 0), (7, 60000, 4800, 0, 0)]
RAMPS64 = [dict(gain0_q15=q, gain1_q15=q2, ramp_start=s + 17 * i, ramp_len=ln, mode=md)
           for i in range(8) for q, q2, s, ln, md in _R]


@pytest.mark.parametrize("devices,rate_out", [([0], 48000), ([0, 0], 48000), ([0, 0, 0, 0], 48000),
                                              ([0, 0], 44100)])
def test_mix_spanning_in_library(xm, gpu, devices, rate_out):
    """Config 5 through xm_audio_mixer_mix_spanning_s16: device d holds tracks
    [d*64/n, (d+1)*64/n) of every mix and receives the finished mixes it owns.
    [0] exchanges through an RCCL reduce-scatter (one-device communicator),
    repeated devices through device copies + the ordered finish."""
    import torch
    n = len(devices)
    B, N = 4, 9600 + 5
    x = np.stack([np.stack([O.gen_s16(SEED, 6000 + 64 * b + t, 2, N) for t in range(64)]) for b in range(B)])
    x[:, :6, 300:800] = 32767
    x[:, 58:, 1200:1500] = -32768
    one = xm.Mixer(48000, rate_out, 2, "s16")
    one.set_tracks(RAMPS64)
    want = one.process(x)
    if rate_out == 48000:
        assert bits_equal(want, CO.batch_mix_s16(x, RAMPS64, threads=4)[0])
    F = one.out_frames(N)
    m = xm.Mixer(48000, rate_out, 2, "s16", mem="device", devices=devices)
    m.set_tracks(RAMPS64)
    per = 64 // n
    xs = [torch.from_numpy(np.ascontiguousarray(x[:, d * per:(d + 1) * per])).cuda() for d in range(n)]
    ys = [torch.zeros((B // n, F, 2), dtype=torch.int16, device="cuda") for _ in range(n)]
    m.mix_spanning_s16([t.data_ptr() for t in xs], N * 2, per * N * 2, [t.data_ptr() for t in ys], F * 2, B, N)
    got = np.concatenate([t.cpu().numpy() for t in ys])
    assert bits_equal(got, want)
    # the same handle then runs ordinary full-list calls again (its subs go
    # back from their config-5 subsets to the full 64-track list)
    xall = torch.from_numpy(x).cuda()
    yall = torch.zeros((B, F, 2), dtype=torch.int16, device="cuda")
    ins = [xall[b, t].data_ptr() for b in range(B) for t in range(64)]
    m.process_ptrs(ins, [yall[b].data_ptr() for b in range(B)], B, N)
    assert bits_equal(yall.cpu().numpy(), want)
    # and config 5 once more on the same handle
    for t in ys:
        t.zero_()
    m.mix_spanning_s16([t.data_ptr() for t in xs], N * 2, per * N * 2, [t.data_ptr() for t in ys], F * 2, B, N)
    assert bits_equal(np.concatenate([t.cpu().numpy() for t in ys]), want)
    h = xm.Mixer(48000, rate_out, 2, "s16", devices=devices)
    h.set_tracks(RAMPS64)
    assert bits_equal(h.process(x), want)


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_multi_device_effects_chain(xm, gpu, devices):
    """xm_effects_create_multi: a batch of clips cut into contiguous blocks over
    the device list, bit-identical to one device and to the oracle; host and
    device memory, streaming, and effects added after creation."""
    import torch
    z = golden("effects.npz")
    B, N = 7, 4410 + 13
    x = np.stack([O.gen_f32(SEED, 1300 + b, 2, N) for b in range(B)])
    h = np.linspace(-0.25, 0.5, 31).astype(np.float32)
    one = xm.Effects(44100, 2)
    multi = xm.Effects(44100, 2, devices=devices)
    assert multi.n_devices() == len(devices)
    for e in (one, multi):
        for s in z["sos"]:
            e.add_biquad(s)
        e.add_fir(h)
    want = one.process(x)
    assert bits_equal(multi.process(x), want)
    ref = np.stack([CO.fir_f32(CO.biquad_f32(x[b], z["sos"]), h) for b in range(B)])
    assert bits_equal(want, ref)
    md = xm.Effects(44100, 2, mem="device", devices=devices)
    for s in z["sos"]:
        md.add_biquad(s)
    md.add_fir(h)
    xd = torch.from_numpy(x).cuda()
    yd = torch.zeros_like(xd)
    md.process_ptrs([xd[b].data_ptr() for b in range(B)], [yd[b].data_ptr() for b in range(B)], N)
    assert bits_equal(yd.cpu().numpy(), want)
    multi.stream_reset(B)
    parts = [multi.process_stream(x[:, a:b]) for a, b in ((0, 1), (1, 1), (1, 2000), (2000, N))]
    assert bits_equal(np.concatenate(parts, axis=1), want)
    if len(devices) > 1:
        with pytest.raises(xm.XmError) as e:
            multi.set_stream(torch.cuda.current_stream().cuda_stream)
        assert e.value.code == xm.XM_ENOSYS
    else:   # a one-device list is the plain single-device chain: streams allowed
        multi.set_stream(torch.cuda.current_stream().cuda_stream)
        multi.set_stream(None)


@pytest.mark.parametrize("devices,batch,chunks", [([0], 8, 4), ([0], 8, 3), ([0] * 8, 32, 0), ([0] * 8, 32, 2),
                                                  ([0, 0], 12, 3)])
def test_mix_spanning_chunked_exchange(xm, gpu, devices, batch, chunks):
    """Config 5 with the exchange in chunks (xm_audio_mixer_set_span_chunks,
    VERDICT r5 item 4): the owned blocks are cut into K groups; [0] runs K
    RCCL reduce-scatters on the exchange stream beside the next group's
    partials (3 asked of 8 owned mixes: K = 2), repeated devices exchange each
    group by device copies.  Every K equals the one-device 64-track mix."""
    import torch
    n = len(devices)
    B, N = batch, 4800 + 3
    x = np.stack([np.stack([O.gen_s16(SEED, 7000 + 64 * b + t, 2, N) for t in range(64)]) for b in range(B)])
    x[:, :6, 300:800] = 32767
    one = xm.Mixer(48000, 48000, 2, "s16")
    one.set_tracks(RAMPS64)
    want = one.process(x)
    F = one.out_frames(N)
    m = xm.Mixer(48000, 48000, 2, "s16", mem="device", devices=devices)
    m.set_tracks(RAMPS64)
    m.set_span_chunks(chunks)
    per = 64 // n
    xs = [torch.from_numpy(np.ascontiguousarray(x[:, d * per:(d + 1) * per])).cuda() for d in range(n)]
    ys = [torch.full((B // n, F, 2), -5, dtype=torch.int16, device="cuda") for _ in range(n)]
    m.mix_spanning_s16([t.data_ptr() for t in xs], N * 2, per * N * 2, [t.data_ptr() for t in ys], F * 2, B, N)
    assert bits_equal(np.concatenate([t.cpu().numpy() for t in ys]), want)
    with pytest.raises(xm.XmError):
        m.set_span_chunks(65)
