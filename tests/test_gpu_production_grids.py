"""Configs 3, 4 and 5 at the production sizes the bench lines time
(BASELINE.json:9-11; tools/bench_configs.py), so the grids
the smaller parity cases never reach run in the driver's GPU tests too:

  c3  1024 mixes x 8 s16 stereo tracks x 960000 frames (10 s @ 48 kHz),
      Q15 ramps and a crossfade: 15.7 G input samples, past 2^32 elements;
  c4  the per-GPU shard of config 4, 1024 clips = 128 mixes x 8 stereo fp32
      tracks x 480000 frames, resample -> 5-band EQ -> gain -> mix, through
      a multi-device handle over the same GPU twice (devices=[0, 0]);
  c5  512 mixes x 64 s16 tracks x 960000 frames spread over 8 "devices"
      (devices=[0] * 8: 8 tracks each, int32 partials, one exchange, each
      device saturating its block of mixes), mix_spanning_s16.

Each checks the first and the last mix against the C oracle bit for bit and
that no output sample was left unwritten: the outputs are prefilled with two
different patterns in two runs (f32: NaN), and both runs must agree.
"""
import numpy as np
import pytest

from conftest import bits_equal, golden

import c_oracle as CO

pytestmark = pytest.mark.gpu

Q15 = [dict(gain0_q15=a, gain1_q15=b, ramp_start=s, ramp_len=n, mode=md)
       for a, b, s, n, md in [(29491, 29491, 0, 0, 0), (0, 26214, 0, 48000, 0), (22938, 6554, 240000, 96000, 0),
                              (16384, 16384, 0, 0, 0), (0, 0, 144000, 96000, 1), (0, 32768, 144000, 96000, 0),
                              (32768, 0, 432000, 48000, 0), (9830, 19661, 300000, 0, 0)]]


def _free():
    import torch
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def test_config3_production_grid(xm, gpu):
    import torch
    from bench import SEED
    B, ntr, N = 1024, 8, 960000
    x = torch.empty((B, ntr, N, 2), dtype=torch.int16, device="cuda")   # 31.5 GB
    xm.synth(x.data_ptr(), "s16", SEED, 0, B * ntr, 2, N)
    m = xm.Mixer(48000, 48000, 2, "s16", mem="device")
    m.set_tracks(Q15)
    ys = []
    for fill in (0x5555, -0x5556):
        y = torch.full((B, N, 2), fill, dtype=torch.int16, device="cuda")
        torch.cuda.synchronize()
        m.process_strided(x.data_ptr(), N * 2, ntr * N * 2, y.data_ptr(), N * 2, B, N)
        torch.cuda.synchronize()
        ys.append(y)
    assert bool(torch.equal(ys[0], ys[1])), "an output sample was left unwritten"
    for b in (0, B - 1):
        ref, _ = CO.batch_mix_s16(x[b:b + 1].cpu().numpy(), Q15, threads=8)
        assert bits_equal(ys[0][b:b + 1].cpu().numpy(), ref), b
    del x, ys
    _free()


def test_config4_shard_through_multi_device_handle(xm, gpu):
    import torch
    from bench import RAMPS, SEED
    sos = golden("effects.npz")["sos"]
    B, ntr, N = 128, 8, 480000
    devs = [0, 0]
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device", devices=devs)
    m.set_tracks(RAMPS)
    e = xm.Effects(44100, 2)
    for s in sos:
        e.add_biquad(s)
    m.set_track_effects(e)
    F = m.out_frames(N)
    x = torch.empty((B, ntr, N, 2), dtype=torch.float32, device="cuda")
    xm.synth(x.data_ptr(), "f32", SEED, 0, B * ntr, 2, N)
    y = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    half = B // 2   # block d of the shard on handle device d (both GPU 0)
    m.process_sharded([x[:half].data_ptr(), x[half:].data_ptr()], N * 2, ntr * N * 2,
                      [y[:half].data_ptr(), y[half:].data_ptr()], F * 2, [half, B - half], N)
    torch.cuda.synchronize()
    assert not bool(y.isnan().any()), "an output frame was left unwritten"
    for b in (0, B - 1):
        xb = x[b].cpu().numpy()
        r = [CO.biquad_f32(CO.resample_f32(t, 147, 160), sos) for t in xb]
        assert bits_equal(y[b].cpu().numpy(), CO.mix_f32(r, RAMPS)), b
    del x, y
    _free()


def test_config4_time_block_pipeline(xm, gpu):
    """One device at config 4's clip length: the time-block pipeline (8 blocks
    of whole super-periods: block resample, biquad with carried states and the
    gained mix per block, on CU-masked streams; src/xm_audio_mixer.c
    run_fx_pipelined) is the path taken (24 launches) and every output equals
    the oracle bit for bit, with ramps and steps that start and end inside
    blocks and across their edges."""
    import torch
    from bench import SEED
    sos = golden("effects.npz")["sos"]
    B, ntr, N = 2, 8, 480000
    F = 441000
    edge = (F // 32 + 146) // 147 * 147          # the first block edge
    ramps = [dict(gain0=0.9),
             dict(gain0=0.0, gain1=0.8, ramp_start=edge - 700, ramp_len=1400),
             dict(mode=1, ramp_start=3 * edge - 5, ramp_len=9 * edge),
             dict(gain0=0.3, gain1=0.6, ramp_start=7 * edge),
             dict(gain0=1.25, gain1=0.5, ramp_start=0, ramp_len=F),
             dict(gain0=0.5, gain1=0.0, ramp_start=F - 2 * edge - 3, ramp_len=2 * edge),
             dict(gain0=0.7),
             dict(gain0=0.2, gain1=0.9, ramp_start=edge, ramp_len=1)]
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    m.set_tracks(ramps)
    e = xm.Effects(44100, 2)
    for s in sos:
        e.add_biquad(s)
    m.set_track_effects(e)
    assert m.out_frames(N) == F
    x = torch.empty((B, ntr, N, 2), dtype=torch.float32, device="cuda")
    xm.synth(x.data_ptr(), "f32", SEED, 77, B * ntr, 2, N)
    y = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    m.process_strided(x.data_ptr(), N * 2, ntr * N * 2, y.data_ptr(), F * 2, B, N)
    torch.cuda.synchronize()
    assert m.timing().n_launches == 24, m.timing().n_launches
    for b in range(B):
        xb = x[b].cpu().numpy()
        r = [CO.biquad_f32(CO.resample_f32(t, 147, 160), sos) for t in xb]
        assert bits_equal(y[b].cpu().numpy(), CO.mix_f32(r, ramps)), b
    del x, y
    _free()


def test_config5_production_grid_mix_spanning(xm, gpu):
    import torch
    from bench import RAMPS64, SEED
    B, ntr, N, n = 512, 64, 960000, 8
    per = ntr // n
    devs = [0] * n
    m = xm.Mixer(48000, 48000, 2, "s16", mem="device", devices=devs)
    m.set_tracks(RAMPS64)
    xs = []
    for d in range(n):   # device d: tracks [8d, 8d + 8) of every mix, 7.9 GB each
        x = torch.empty((B, per, N, 2), dtype=torch.int16, device="cuda")
        xm.synth(x.data_ptr(), "s16", SEED, d * B * per, B * per, 2, N)
        xs.append(x)
    nb = B // n
    outs = {}
    for fill in (0x5555, -0x5556):
        ys = [torch.full((nb, N, 2), fill, dtype=torch.int16, device="cuda") for _ in range(n)]
        torch.cuda.synchronize()
        m.mix_spanning_s16([x.data_ptr() for x in xs], N * 2, per * N * 2, [y.data_ptr() for y in ys], N * 2, B, N)
        torch.cuda.synchronize()
        outs[fill] = ys
    for a, b in zip(outs[0x5555], outs[-0x5556]):
        assert bool(torch.equal(a, b)), "an output sample was left unwritten"
    ys = outs[0x5555]
    for g in (0, B - 1):   # global mix g: its 64 tracks are row g of every device's block
        tracks = np.concatenate([xs[d][g].cpu().numpy() for d in range(n)])
        ref, _ = CO.batch_mix_s16(tracks[None], RAMPS64, threads=8)
        assert bits_equal(ys[g // nb][g % nb].cpu().numpy(), ref[0]), g
    del xs, outs, ys
    _free()
