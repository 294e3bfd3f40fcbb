"""GPU parity: the HIP path (through the C ABI) against the oracle.

Bar (BASELINE.json:5): bit-exact for s16 mix/gain and — stricter than the
north_star's ±1 ULP float32 allowance — bit-exact for fp32 resample / mix /
biquad / FIR, since the kernels keep scipy's separately-rounded order.
Small cases compare with the committed scipy golden vectors; larger ones
with the C restatement (oracle/xm_oracle.c), itself pinned to those vectors
by tests/test_oracle.py.
"""
import hashlib
import json

import numpy as np
import pytest

from conftest import bits_equal, golden, manifest, ulp_diff

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED


def _resample_cases():
    z = golden("resample.npz")
    return sorted(k[:-6] for k in z.files if k.endswith("__meta"))


@pytest.mark.parametrize("name", _resample_cases())
def test_resample_f32_golden(xm, gpu, name):
    z = golden("resample.npz")
    fi, fo, N, Cc, clip = (int(v) for v in z[f"{name}__meta"])
    x = O.gen_f32(SEED, clip, Cc, N)
    m = xm.Mixer(fi, fo, Cc, "f32")
    y = m.process(x[None, None])[0]
    ref = z[f"{name}__y"].reshape(y.shape)
    assert bits_equal(y, ref), f"max ulp {ulp_diff(y, ref)}"


@pytest.mark.parametrize("kind", ["silence", "fullscale", "denormal", "impulse"])
def test_resample_f32_special(xm, gpu, kind):
    z = golden("resample.npz")
    x, ref = z[f"special_{kind}__x"], z[f"special_{kind}__y"]
    y = xm.Mixer(48000, 44100, 2, "f32").process(x[None, None])[0]
    assert bits_equal(y, ref)


def test_resample_s16_saturating(xm, gpu):
    z = golden("resample_s16.npz")
    y = xm.Mixer(48000, 44100, 2, "s16").process(z["x"][None, None])[0]
    assert bits_equal(y, z["y"])


def test_config1_s16_44k_to_48k_full_clip(xm, gpu):
    """BASELINE.json:7: single mono 44.1k->48k s16, 10 s — GPU equals the CPU path."""
    x = O.gen_s16(SEED, 0, 1, 441000)
    y = xm.Mixer(44100, 48000, 1, "s16").process(x[None, None])[0]
    assert y.shape == (480000, 1)
    assert hashlib.sha256(y.tobytes()).hexdigest() == manifest()["config1_sha256"]


def test_mix_s16_8track_golden(xm, gpu):
    """Config 3 shape: 8-track s16 mix with ramps, crossfade and saturation."""
    z = golden("mix.npz")
    ramps = json.loads(str(z["s16_mix8__ramps"]))
    tr = [O.gen_s16(SEED, 200 + t, 2, 4800) for t in range(8)]
    tr[0][10:20] = 32767
    tr[1][10:20] = 32767
    tr[2][30:40] = -32768
    m = xm.Mixer(48000, 48000, 2, "s16")
    m.set_tracks(ramps)
    y = m.process(np.stack(tr)[None])[0]
    assert bits_equal(y, z["s16_mix8__y"])


def test_resample_mix_s16_golden(xm, gpu):
    z = golden("mix.npz")
    ramps = json.loads(str(z["s16_mix8__ramps"]))[:4]
    tr = [O.gen_s16(SEED, 200 + t, 2, 4800) for t in range(4)]
    tr[0][10:20] = 32767
    tr[1][10:20] = 32767
    tr[2][30:40] = -32768
    m = xm.Mixer(48000, 44100, 2, "s16")
    m.set_tracks(ramps)
    assert bits_equal(m.process(np.stack(tr)[None])[0], z["s16_resample4__y"])


def test_resample_mix_f32_golden(xm, gpu):
    """Headline op at fixture size: resample 48k->44.1k + 8-track ramped mix."""
    z = golden("mix.npz")
    ramps = json.loads(str(z["f32_resample8__ramps"]))
    xs = np.stack([O.gen_f32(SEED, 100 + t, 2, 4800) for t in range(8)])
    m = xm.Mixer(48000, 44100, 2, "f32")
    m.set_tracks(ramps)
    y = m.process(xs[None])[0]
    assert bits_equal(y, z["f32_resample8__y"]), f"max ulp {ulp_diff(y, z['f32_resample8__y'])}"


HEADLINE_RAMPS = [
    dict(gain0=0.9), dict(gain0=0.0, gain1=0.8, ramp_start=1000, ramp_len=30000),
    dict(gain0=0.7, gain1=0.2, ramp_start=20000, ramp_len=4410), dict(gain0=0.5),
    dict(mode=1, ramp_start=30000, ramp_len=8000), dict(gain0=0.0, gain1=1.0, ramp_start=30000, ramp_len=8000),
    dict(gain0=1.25, gain1=0.75, ramp_start=0, ramp_len=44100), dict(gain0=0.3, gain1=0.6, ramp_start=40000),
]


@pytest.mark.parametrize("frames", [48000, 48000 + 77])
def test_resample_mix_f32_vs_c_oracle_batch(xm, gpu, frames):
    """4 mixes x 8 tracks x ~1 s stereo, every output bit-compared with the C oracle."""
    B, ntr = 4, 8
    x = np.stack([np.stack([O.gen_f32(SEED, 1000 + 8 * b + t, 2, frames) for t in range(ntr)]) for b in range(B)])
    m = xm.Mixer(48000, 44100, 2, "f32")
    m.set_tracks(HEADLINE_RAMPS)
    y = m.process(x)
    ref, _ = CO.batch_resample_mix_f32(x, HEADLINE_RAMPS, 147, 160, threads=8)
    assert bits_equal(y, ref), f"max ulp {ulp_diff(y, ref)}"


def test_resample_44_to_48_mix_vs_c_oracle(xm, gpu):
    x = np.stack([O.gen_f32(SEED, 500 + t, 2, 44100) for t in range(3)])[None]
    ramps = HEADLINE_RAMPS[:3]
    m = xm.Mixer(44100, 48000, 2, "f32")
    m.set_tracks(ramps)
    y = m.process(x)[0]
    assert bits_equal(y, CO.resample_mix_f32(list(x[0]), ramps, 160, 147))


def test_mono_and_identity_ratio(xm, gpu):
    x = np.stack([O.gen_f32(SEED, 600 + t, 1, 3000) for t in range(5)])[None]
    ramps = HEADLINE_RAMPS[:5]
    m = xm.Mixer(48000, 44100, 1, "f32")
    m.set_tracks(ramps)
    assert bits_equal(m.process(x)[0], CO.resample_mix_f32(list(x[0]), ramps, 147, 160))
    m2 = xm.Mixer(48000, 48000, 1, "f32")
    m2.set_tracks(ramps)
    assert bits_equal(m2.process(x)[0], CO.mix_f32(list(x[0]), ramps))


def test_large_s16_mix_vs_c_oracle(xm, gpu):
    """Config 3 arithmetic on 16 mixes x 8 tracks x 2 s stereo."""
    B, ntr, F = 16, 8, 96000
    x = np.stack([np.stack([O.gen_s16(SEED, 3000 + 8 * b + t, 2, F) for t in range(ntr)]) for b in range(B)])
    ramps = [dict(gain0_q15=q, gain1_q15=q2, ramp_start=s, ramp_len=ln, mode=md)
             for q, q2, s, ln, md in [(32768, 32768, 0, 0, 0), (0, 32768, 100, 20000, 0), (65535, 100, 0, 96000, 0),
                                      (16384, 16384, 0, 0, 0), (0, 0, 50000, 9000, 1), (0, 32768, 50000, 9000, 0),
                                      (40000, 3, 70000, 13, 0), (7, 60000, 48000, 0, 0)]]
    m = xm.Mixer(48000, 48000, 2, "s16")
    m.set_tracks(ramps)
    y = m.process(x)
    ref, _ = CO.batch_mix_s16(x, ramps, threads=8)
    assert bits_equal(y, ref)


def test_crossfade_helper(xm, gpu):
    x = np.stack([O.gen_f32(SEED, 700 + t, 2, 4800) for t in range(2)])[None]
    m = xm.Mixer(48000, 44100, 2, "f32")
    m.set_tracks([dict(gain0=1.0), dict(gain0=1.0)])
    m.set_crossfade(0, 1, 1000, 2000)
    ramps = [dict(mode=1, ramp_start=1000, ramp_len=2000), dict(gain0=0.0, gain1=1.0, ramp_start=1000, ramp_len=2000)]
    assert bits_equal(m.process(x)[0], CO.resample_mix_f32(list(x[0]), ramps, 147, 160))


def test_ragged_lengths(xm, gpu):
    for N in (1, 2, 22, 23, 159, 160, 161, 321, 1001):
        x = np.stack([O.gen_f32(SEED, 800 + t, 2, N) for t in range(3)])[None]
        m = xm.Mixer(48000, 44100, 2, "f32")
        m.set_tracks(HEADLINE_RAMPS[:3])
        y = m.process(x)[0]
        assert bits_equal(y, CO.resample_mix_f32(list(x[0]), HEADLINE_RAMPS[:3], 147, 160)), N


def test_empty_inputs(xm, gpu):
    m = xm.Mixer(48000, 44100, 2, "f32")
    y = m.process(np.zeros((1, 1, 0, 2), np.float32))
    assert y.shape == (1, 0, 2)
    y = m.process(np.zeros((0, 1, 100, 2), np.float32))
    assert y.shape == (0, 92, 2)


def test_effects_biquad_fir_golden(xm, gpu):
    z = golden("effects.npz")
    e = xm.Effects(48000, 2)
    for b in z["bands"]:
        e.add_eq_band(int(b[0]), float(b[2]), float(b[3]), float(b[4]))
    for i in range(5):
        assert bits_equal(e.biquad(i), z["sos"][i])
    assert bits_equal(e.process(z["x"][None])[0], z["y_biquad"])
    f = xm.Effects(48000, 2)
    f.add_fir(z["h63"])
    assert bits_equal(f.process(z["x"][None])[0], z["y_fir63"])
    assert bits_equal(f.process(z["x"][None].copy(), inplace=True)[0], z["y_fir63"])
    g = xm.Effects(48000, 1)
    g.add_fir(z["h7"])
    assert bits_equal(g.process(z["x"][None, :1000, :1])[0, :, 0], z["y_fir7_mono"])


@pytest.mark.parametrize("C", [1, 2])
def test_fir_tap_counts_vs_c_oracle(xm, gpu, C):
    """The register-blocked FIR over every shape of its tap loop: fewer taps
    than one 7-tap block, whole 14-tap iterations, a trailing whole block and
    a remainder, and more taps than one tile; clip lengths off the 1792-frame
    tile and the 16-B grid."""
    rng = np.random.default_rng(11)
    for K in (1, 2, 6, 7, 8, 13, 14, 15, 20, 21, 27, 28, 35, 63, 64, 127, 255, 2000):
        for N in (1, 5, 1791 + K, 4001):
            x = O.gen_f32(SEED, 3000 + K, C, N)
            h = rng.standard_normal(K).astype(np.float32) / K
            e = xm.Effects(48000, C)
            e.add_fir(h)
            y = e.process(x[None])[0]
            assert bits_equal(y, CO.fir_f32(x, h)), (K, N)


def test_effects_chain_vs_c_oracle(xm, gpu):
    z = golden("effects.npz")
    x = np.stack([O.gen_f32(SEED, 900 + b, 2, 20000) for b in range(6)])
    e = xm.Effects(48000, 2)
    for s in z["sos"][:3]:
        e.add_biquad(s)
    e.add_fir(z["h63"])
    for s in z["sos"][3:]:
        e.add_biquad(s)
    y = e.process(x)
    for b in range(6):
        r = CO.biquad_f32(CO.fir_f32(CO.biquad_f32(x[b], z["sos"][:3]), z["h63"]), z["sos"][3:])
        assert bits_equal(y[b], r), b


def test_mixer_with_track_eq_vs_c_oracle(xm, gpu):
    """Config 4 chain: resample -> 5-band EQ -> gain -> ordered mix."""
    z = golden("effects.npz")
    x = np.stack([O.gen_f32(SEED, 950 + t, 2, 9600) for t in range(4)])[None]
    ramps = HEADLINE_RAMPS[:4]
    e = xm.Effects(44100, 2)
    for s in z["sos"]:
        e.add_biquad(s)
    m = xm.Mixer(48000, 44100, 2, "f32")
    m.set_tracks(ramps)
    m.set_track_effects(e)
    y = m.process(x)[0]
    r = [CO.biquad_f32(CO.resample_f32(t, 147, 160), z["sos"]) for t in x[0]]
    assert bits_equal(y, CO.mix_f32(r, ramps))


def test_mixer_with_track_biquad_fir_chain(xm, gpu):
    """Per-track chain with FIR stages (ping-pong track buffers): resample ->
    biquad x2 -> FIR 63 -> biquad -> FIR 7 -> gain -> ordered mix."""
    z = golden("effects.npz")
    x = np.stack([O.gen_f32(SEED, 970 + t, 2, 9600 + 3) for t in range(3)])[None]
    ramps = HEADLINE_RAMPS[:3]
    e = xm.Effects(44100, 2)
    e.add_biquad(z["sos"][0])
    e.add_biquad(z["sos"][1])
    e.add_fir(z["h63"])
    e.add_biquad(z["sos"][2])
    e.add_fir(z["h7"])
    m = xm.Mixer(48000, 44100, 2, "f32")
    m.set_tracks(ramps)
    m.set_track_effects(e)
    y = m.process(x)[0]
    r = [CO.fir_f32(CO.biquad_f32(CO.fir_f32(CO.biquad_f32(CO.resample_f32(t, 147, 160), z["sos"][:2]), z["h63"]),
                                  z["sos"][2:3]), z["h7"]) for t in x[0]]
    assert bits_equal(y, CO.mix_f32(r, ramps))


def test_device_memory_strided_and_ptrs(xm, gpu):
    """XM_MEM_DEVICE through torch-allocated HBM: strided, pointer tables and a
    caller stream all give the host-mode bits."""
    import torch
    B, ntr, N = 3, 8, 9600
    x = np.stack([np.stack([O.gen_f32(SEED, 1200 + 8 * b + t, 2, N) for t in range(ntr)]) for b in range(B)])
    host = xm.Mixer(48000, 44100, 2, "f32")
    host.set_tracks(HEADLINE_RAMPS)
    ref = host.process(x)
    dev = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    dev.set_tracks(HEADLINE_RAMPS)
    F = dev.out_frames(N)
    xd = torch.from_numpy(x).cuda()
    yd = torch.zeros((B, F, 2), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    dev.process_strided(xd.data_ptr(), N * 2, ntr * N * 2, yd.data_ptr(), F * 2, B, N)
    assert bits_equal(yd.cpu().numpy(), ref)
    # permuted pointer table (non-strided)
    perm = [2, 0, 1]
    yd2 = torch.zeros_like(yd)
    ins = [xd[b, t].data_ptr() for b in perm for t in range(ntr)]
    outs = [yd2[i].data_ptr() for i in range(B)]
    dev.process_ptrs(ins, outs, B, N)
    assert bits_equal(yd2.cpu().numpy(), ref[perm])
    # caller stream: stream-ordered, asynchronous
    s = torch.cuda.Stream()
    yd3 = torch.zeros_like(yd)
    dev.set_stream(s.cuda_stream)
    dev.process_strided(xd.data_ptr(), N * 2, ntr * N * 2, yd3.data_ptr(), F * 2, B, N)
    s.synchronize()
    dev.set_stream(None)
    assert bits_equal(yd3.cpu().numpy(), ref)


def test_synth_matches_oracle_generator(xm, gpu):
    import torch
    t = torch.empty((3, 1000, 2), dtype=torch.float32, device="cuda")
    xm.synth(t.data_ptr(), "f32", SEED, 4094, 3, 2, 1000)
    for c in range(3):
        assert bits_equal(t[c].cpu().numpy(), O.gen_f32(SEED, 4094 + c, 2, 1000))
    s = torch.empty((2, 777, 1), dtype=torch.int16, device="cuda")
    xm.synth(s.data_ptr(), "s16", SEED, 5, 2, 1, 777)
    assert bits_equal(s[0].cpu().numpy(), O.gen_s16(SEED, 5, 1, 777))


def test_errors(xm, gpu):
    m = xm.Mixer(48000, 44100, 2, "f32")
    with pytest.raises(xm.XmError) as e:
        m.set_tracks([dict(gain0_q15=70000)])
    assert e.value.code == xm.XM_EINVAL
    with pytest.raises(xm.XmError):
        m.set_tracks([dict()] * 65)
    m.set_tracks([dict(in_rate=22050)])   # another rate: only process_timeline takes it
    with pytest.raises(xm.XmError) as e:
        m.process(np.zeros((1, 1, 100, 2), np.float32))
    assert e.value.code == xm.XM_ENOSYS
    with pytest.raises(xm.XmError):
        xm.Mixer(48000, 44100, 2, "f32", device=99)
    e2 = xm.Effects(48000, 2)
    with pytest.raises(xm.XmError):
        e2.add_biquad([1, 0, 0, 2, 0, 0])   # a0 != 1


@pytest.mark.parametrize("n_sos", [1, 2, 5, 8, 15, 16, 40, 64, 70])
@pytest.mark.parametrize("channels", [1, 2])
def test_biquad_cascade_shapes(xm, gpu, n_sos, channels):
    """Section-pipelined biquad kernel (lane = clip x section): every cascade
    length up to XM_MAX_SOS = 64 in one pass (70: split in two), more clips
    than one workgroup holds, ragged lengths
    around the 64-granule chunk (128 stereo / 256 mono frames: whole chunks,
    a partial last chunk, one frame past a chunk), bit-compared with the C
    oracle (sosfilt order)."""
    z = golden("effects.npz")
    rng = np.random.default_rng(n_sos * 10 + channels)
    sos = np.concatenate([z["sos"]] * (n_sos // len(z["sos"]) + 1))[:n_sos]   # > 64: the stager splits
    e = xm.Effects(48000, channels)
    for s in sos:
        e.add_biquad(s)
    ch = 256 // channels
    # clips per workgroup: k_biquad_mf (<= 16 sections, (16 / n_sos) groups
    # of 4 / channels clips) or k_biquad_pipe (64 / n_sos)
    kpw = min(16 // n_sos * (4 // channels), 16) if n_sos <= 16 else min(64 // n_sos, 16)
    for B, N in [(1, 1), (3, 31), (2 * kpw + 1, 33), (17, 1000), (5, ch), (kpw, 2 * ch), (3, 3 * ch + 1),
                 (kpw + 1, 4 * ch - 1)]:
        x = (rng.standard_normal((B, N, channels)) * 0.5).astype(np.float32)
        y = e.process(x)
        for b in range(B):
            assert bits_equal(y[b], CO.biquad_f32(x[b], sos)), (B, N, b)


@pytest.mark.parametrize("B,N", [(8, 4800), (9, 48000), (17, 9602), (3, 4800), (16, 480000)])
def test_resample_only_batches(xm, gpu, B, N):
    """Config 2 shape: 1-track unity-gain resampling of a batch of clips (the
    fast kernel's split mode takes 8 clips per pseudo-mix, the remainder and
    batches under 8 run the generic kernel); every clip bit-compared."""
    x = np.stack([O.gen_f32(SEED, 3100 + b, 2, N) for b in range(B)])[:, None]
    m = xm.Mixer(48000, 44100, 2, "f32")
    y = m.process(x)
    idx = range(B) if N < 100000 else (0, 7, 8, 15)
    for b in idx:
        assert bits_equal(y[b], CO.resample_f32(x[b, 0], 147, 160)), b


SPAN_RAMPS = [dict(gain0_q15=q, gain1_q15=q2, ramp_start=s, ramp_len=ln, mode=md)
              for q, q2, s, ln, md in [(32768, 32768, 0, 0, 0), (0, 32768, 100, 20000, 0), (65535, 100, 0, 9600, 0),
                                       (16384, 16384, 0, 0, 0), (0, 0, 5000, 900, 1), (0, 32768, 5000, 900, 0),
                                       (40000, 3, 7000, 13, 0), (7, 60000, 4800, 0, 0)] * 2]


@pytest.mark.parametrize("rate_out", [48000, 44100])
def test_partial_finish_s16_spanning(xm, gpu, rate_out):
    """Config 5 kernels: the 16 tracks of every mix split over two handles (as
    over two devices); int32 partials (vs the numpy oracle), summed by
    finish_s16 in part order, equal the one-handle 16-track mix bit for bit.
    rate_out 44100 runs the partial through the resampling (generic) kernel."""
    import torch
    B, N, ntr = 3, 9600, 16
    x = np.stack([np.stack([O.gen_s16(SEED, 5000 + 16 * b + t, 2, N) for t in range(ntr)]) for b in range(B)])
    x[:, :4, 100:300] = 32767       # the full mix saturates there
    full = xm.Mixer(48000, rate_out, 2, "s16")
    full.set_tracks(SPAN_RAMPS)
    ref = full.process(x)
    F = full.out_frames(N)
    xd = torch.from_numpy(x).cuda()
    parts = torch.zeros((2, B, F * 2), dtype=torch.int32, device="cuda")
    for h in range(2):
        m = xm.Mixer(48000, rate_out, 2, "s16", mem="device")
        m.set_tracks(SPAN_RAMPS[8 * h: 8 * h + 8])
        xh = xd[:, 8 * h: 8 * h + 8].contiguous()
        m.process_partial_strided(xh.data_ptr(), N * 2, 8 * N * 2, parts[h].data_ptr(), F * 2, B, N)
        torch.cuda.synchronize()
        if rate_out == 48000:
            for b in range(B):
                want = O.mix_s16_partial(list(x[b, 8 * h: 8 * h + 8]), SPAN_RAMPS[8 * h: 8 * h + 8]).reshape(-1)
                assert bits_equal(parts[h, b].cpu().numpy(), want), (h, b)
    y = torch.empty((B, F, 2), dtype=torch.int16, device="cuda")
    m.finish_s16(parts.data_ptr(), 2, B * F * 2, F * 2, y.data_ptr(), F * 2, B, F)
    assert bits_equal(y.cpu().numpy(), ref)
    if rate_out == 48000:
        assert bits_equal(ref, CO.batch_mix_s16(x, SPAN_RAMPS, threads=4)[0])
    # the exchange's own form: one pre-summed partial, saturate only
    summed = (parts[0] + parts[1]).contiguous()
    y1 = torch.empty_like(y)
    m.finish_s16(summed.data_ptr(), 1, 0, F * 2, y1.data_ptr(), F * 2, B, F)
    assert bits_equal(y1.cpu().numpy(), ref)


def test_partial_errors(xm, gpu):
    m = xm.Mixer(48000, 48000, 2, "f32", mem="device")
    with pytest.raises(xm.XmError) as e:
        m.process_partial_strided(1, 2, 2, 1, 2, 1, 1)
    assert e.value.code == xm.XM_ENOSYS
    h = xm.Mixer(48000, 48000, 2, "s16")     # host memory: not supported
    with pytest.raises(xm.XmError) as e:
        h.finish_s16(1, 1, 0, 2, 1, 2, 1, 1)
    assert e.value.code == xm.XM_ENOSYS


@pytest.mark.parametrize("n_sos", [5, 20])
@pytest.mark.parametrize("channels", [1, 2])
def test_biquad_silence_zeros_and_denormals(xm, gpu, n_sos, channels):
    """Signed zeros, exact silence and denormals through the cascade: bursts
    followed by long silences, so every section's state decays through the
    denormal range to zero; -0 and denormal input samples; a clip of pure
    -0.  The feed-forward products (matrix core in k_biquad_mf, VALU in
    k_biquad_pipe for 20 sections) must keep IEEE signed zeros and gradual
    underflow: bit-compared with the C oracle."""
    z = golden("effects.npz")
    sos = np.concatenate([z["sos"]] * (n_sos // len(z["sos"]) + 1))[:n_sos]
    e = xm.Effects(48000, channels)
    for s in sos:
        e.add_biquad(s)
    rng = np.random.default_rng(4242 + n_sos + channels)
    B, N = 6, 60000
    x = np.zeros((B, N, channels), np.float32)
    x[0, :500] = rng.standard_normal((500, channels)) * 0.5
    x[1, 100:101] = 1.0                                   # an impulse, then 59899 frames of silence
    x[2] = -0.0
    x[3, ::7] = -0.0
    x[3, 3::11] = rng.standard_normal((len(range(3, N, 11)), channels)) * 1e-39   # denormal samples
    x[4, :2000] = rng.standard_normal((2000, channels)) * 1e-3
    x[4, 30000:30050] = 1e-38
    x[5] = rng.standard_normal((N, channels)) * 0.25
    x[5, 20000:] = 0.0
    y = e.process(x)
    tiny = 0
    for b in range(B):
        want = CO.biquad_f32(x[b], sos)
        tiny += int(np.count_nonzero((want != 0) & (np.abs(want) < np.finfo(np.float32).tiny)))
        assert bits_equal(y[b], want), b
    assert tiny > 0   # the oracle's outputs do pass through the denormal range


def test_biquad_pointer_tables_unaligned_and_far_apart(xm, gpu):
    """The biquad kernel's two addressing forms: clips within 4 GB of the
    wave's lowest one (wave-uniform base + 32-bit offsets) and clips further
    apart (per-access 64-bit bases), with float-aligned (not 16-B aligned)
    clip starts, out of place and in place."""
    import torch
    z = golden("effects.npz")
    sos = np.concatenate([z["sos"]] * 2)[:5]
    e = xm.Effects(48000, 2, mem="device")
    for s in sos:
        e.add_biquad(s)
    N, B = 1000, 5
    rng = np.random.default_rng(77)
    x = (rng.standard_normal((B, N, 2)) * 0.5).astype(np.float32)
    want = [CO.biquad_f32(x[b], sos) for b in range(B)]
    big = torch.zeros(((5 << 30) // 4,), dtype=torch.float32, device="cuda")   # 5 GiB
    small = torch.zeros((2 * N + 8,), dtype=torch.float32, device="cuda")
    dst = torch.zeros((B * (N * 2 + 8),), dtype=torch.float32, device="cuda")
    # clip starts: odd float offsets; clips 1 and 3 more than 4 GB above clip 0
    offs = [1, (4 << 30) // 4 + 3, 4 * N + 5, (4 << 30) // 4 + 2 * N + 11]
    views = [big[o:o + 2 * N] for o in offs] + [small[3:3 + 2 * N]]
    for b, v in enumerate(views):
        v.copy_(torch.from_numpy(x[b].reshape(-1)))
    outs = [dst[(b + 1) * (2 * N + 8) - 2 * N - 1:(b + 1) * (2 * N + 8) - 1] for b in range(B - 1)]
    outs.append(big[7 * N + 1:9 * N + 1])
    torch.cuda.synchronize()
    e.process_ptrs([v.data_ptr() for v in views], [o.data_ptr() for o in outs], N)
    torch.cuda.synchronize()
    for b in range(B):
        assert bits_equal(outs[b].cpu().numpy().reshape(N, 2), want[b]), b
    # in place, the same far-apart table
    e.process_ptrs([v.data_ptr() for v in views], [v.data_ptr() for v in views], N)
    torch.cuda.synchronize()
    for b in range(B):
        assert bits_equal(views[b].cpu().numpy().reshape(N, 2), want[b]), b
    del big, small, dst
    torch.cuda.empty_cache()
