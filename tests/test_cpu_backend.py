"""CPU suite: the library's host CPU backend (SURVEY.md §8(b) "n_devices
(0 = CPU)", §1 layer L0-cpu; src/cpu/) through the C ABI, with no GPU.

It is product code (it shares nothing with oracle/), so it gets the same
bar as the kernels: bit-exact against the scipy golden vectors and the C
oracle.  Besides the tests below, this module re-runs the host-memory parity
tests of the GPU suites (tests/test_gpu_*.py) with every handle created on
the CPU backend: the `xm` fixture is overridden here by a view of xmaudio
whose Mixer / Effects / synth default to device="cpu", and `gpu` asks for no
device.  Tests that need torch device memory, several devices, or assert
which gfx950 kernel ran are not re-run (they are GPU tests by nature).
"""
import hashlib
import json

import numpy as np
import pytest

from conftest import bits_equal, golden, manifest

import c_oracle as CO
import np_oracle as O

SEED = O.SEED


class _CpuXm:
    """xmaudio with every handle on the CPU backend unless told otherwise."""

    def __init__(self, mod):
        self._m = mod

    def __getattr__(self, name):
        return getattr(self._m, name)

    def Mixer(self, *a, **k):
        if "devices" not in k and k.get("n_devices", 1) in (0, 1):
            k.setdefault("device", "cpu")
        return self._m.Mixer(*a, **k)

    def Effects(self, *a, **k):
        if "devices" not in k:
            k.setdefault("device", "cpu")
        return self._m.Effects(*a, **k)

    def synth(self, *a, **k):
        k.setdefault("device", "cpu")
        return self._m.synth(*a, **k)


@pytest.fixture(scope="module")
def xm():
    import xmaudio
    return _CpuXm(xmaudio)


@pytest.fixture(scope="module")
def gpu():
    return None   # the re-run GPU-suite tests need no device here


# ---- the GPU suites' host-memory tests, re-run on the CPU backend --------
from test_gpu_parity import (  # noqa: E402,F401
    test_resample_f32_golden, test_resample_f32_special, test_resample_s16_saturating,
    test_config1_s16_44k_to_48k_full_clip, test_mix_s16_8track_golden, test_resample_mix_s16_golden,
    test_resample_mix_f32_golden, test_resample_mix_f32_vs_c_oracle_batch, test_resample_44_to_48_mix_vs_c_oracle,
    test_mono_and_identity_ratio, test_large_s16_mix_vs_c_oracle, test_crossfade_helper, test_ragged_lengths,
    test_empty_inputs, test_effects_biquad_fir_golden, test_fir_tap_counts_vs_c_oracle,
    test_effects_chain_vs_c_oracle, test_mixer_with_track_eq_vs_c_oracle, test_mixer_with_track_biquad_fir_chain,
    test_biquad_cascade_shapes, test_resample_only_batches, test_biquad_silence_zeros_and_denormals,
)
from test_gpu_convert import (  # noqa: E402,F401
    test_f32_mix_to_s16_out, test_s16_mix_to_f32_out, test_convert_with_track_effects_and_timeline,
    test_f32_tracks_into_s16_mix, test_planar_f32_headline_shape_and_effects, test_in_convert_planar_unsupported_calls,
)
from test_gpu_fast_mono import (  # noqa: E402,F401
    test_mono_track_counts, test_mono_short_and_edge_lengths, test_mono_ramp_across_the_half_run,
)
from test_gpu_fast_up import (  # noqa: E402,F401
    test_up_track_counts, test_up_short_and_edge_lengths, test_up_special_inputs, test_up_s16_and_planar,
)
from test_gpu_timeline import (  # noqa: E402,F401
    test_timeline_f32_mixed_rates_into_44k, test_timeline_s16_voice_bgm_48k, test_timeline_same_rate_equals_process,
    test_rate_table_cache_follows_track_list,
)
from test_gpu_streaming import (  # noqa: E402,F401
    test_stream_resample_mix_f32_48_to_44, test_stream_resample_s16_44_to_48_mono, test_stream_mix_s16_same_rate,
    test_stream_mixer_errors, test_effects_stream_chain, test_effects_stream_errors, test_stream_mixed_rates_mid_stream,
)
from test_gpu_golden_fused import (  # noqa: E402,F401
    test_fused_mix_equals_scipy, test_fused_rows_equal_scipy,
)


# ---- the CPU backend through the C ABI itself ----------------------------
def test_config1_through_the_c_api(xm):
    """BASELINE.json:7 ("single mono 44.1 kHz->48 kHz s16 resample on the
    reference CPU path, no GPU"): xm_audio_mixer_create with n_devices = 0
    reproduces the committed config-1 digest, pinned to scipy."""
    import ctypes as C
    lib = xm._lib
    cfg = xm.XmMixerConfig(44100, 48000, 1, xm.XM_FMT_S16, xm.XM_MEM_HOST, 0, 0, 0)   # n_devices = 0
    st = C.c_int(7)
    h = lib.xm_audio_mixer_create_ex(C.byref(cfg), C.byref(st))
    assert h and st.value == 0
    try:
        assert lib.xm_audio_mixer_n_devices(h) == 1
        x = O.gen_s16(SEED, 0, 1, 441000)
        assert lib.xm_audio_mixer_out_frames(h, 441000) == 480000
        y = np.empty(480000, np.int16)
        ins = (C.c_void_p * 1)(x.ctypes.data)
        outs = (C.c_void_p * 1)(y.ctypes.data)
        assert lib.xm_audio_mixer_process_batch(h, ins, outs, 1, 441000) == 0
        assert hashlib.sha256(y.tobytes()).hexdigest() == manifest()["config1_sha256"]
        z = golden("config1.npz")
        assert bits_equal(y[:4096, None], z["y_head"]) and bits_equal(y[-4096:, None], z["y_tail"])
        t = xm.XmMixerTiming()
        assert lib.xm_audio_mixer_get_timing(h, C.byref(t)) == 0
        assert t.n_launches == 1 and t.fast_launches == 0 and t.kernel_ms >= 0.0
    finally:
        hp = C.c_void_p(h)
        lib.xm_audio_mixer_freep(C.byref(hp))
        assert hp.value is None


def test_synth_matches_generator_golden(xm):
    z = golden("generator.npz")
    a = np.empty((1, 512, 2), np.float32)
    xm.synth(a.ctypes.data, "f32", SEED, 0, 1, 2, 512)
    assert bits_equal(a[0], z["f32_clip0_st"])
    m = np.empty((1, 512, 1), np.float32)
    xm.synth(m.ctypes.data, "f32", SEED, 77, 1, 1, 512)
    assert bits_equal(m[0], z["f32_clip77_mono"])
    s = np.empty((1, 512, 2), np.int16)
    xm.synth(s.ctypes.data, "s16", SEED, 5, 1, 2, 512)
    assert bits_equal(s[0], z["s16_clip5_st"])
    b = np.empty((3, 777, 2), np.float32)
    xm.synth(b.ctypes.data, "f32", SEED, 4094, 3, 2, 777)
    for c in range(3):
        assert bits_equal(b[c], O.gen_f32(SEED, 4094 + c, 2, 777))


@pytest.mark.parametrize("n_mix,frames", [(3, 4800 + 5), (17, 1601)])
def test_headline_shape_strided_and_pointer_batches(xm, n_mix, frames):
    """The headline op (48k->44.1k, 8 ramped tracks) in both call forms; the
    mem kind does not matter on the CPU (host pointers either way)."""
    ramps = json.loads(str(golden("mix.npz")["f32_resample8__ramps"]))
    x = np.stack([np.stack([O.gen_f32(SEED, 9000 + 8 * b + t, 2, frames) for t in range(8)]) for b in range(n_mix)])
    ref, _ = CO.batch_resample_mix_f32(x, ramps, 147, 160, threads=4)
    for mem in ("host", "device"):
        m = xm.Mixer(48000, 44100, 2, "f32", mem=mem)
        m.set_tracks(ramps)
        assert bits_equal(m.process(x), ref), mem
        F = m.out_frames(frames)
        y = np.zeros((n_mix, F, 2), np.float32)
        m.process_strided(x.ctypes.data, frames * 2, 8 * frames * 2, y.ctypes.data, F * 2, n_mix, frames)
        assert bits_equal(y, ref), mem
        perm = list(range(n_mix))[::-1]
        y2 = np.zeros_like(y)
        m.process_ptrs([x[b, t].ctypes.data for b in perm for t in range(8)], [y2[i].ctypes.data for i in range(n_mix)],
                       n_mix, frames)
        assert bits_equal(y2, ref[perm]), mem


def test_partial_and_finish_s16(xm):
    """Config 5's two calls on the CPU backend (host pointers): the int32
    partials of two track halves, summed in part order and saturated, equal
    the one-call 16-track mix."""
    from test_gpu_parity import SPAN_RAMPS
    B, N, ntr = 3, 4800, 16
    x = np.stack([np.stack([O.gen_s16(SEED, 5000 + 16 * b + t, 2, N) for t in range(ntr)]) for b in range(B)])
    x[:, :4, 100:300] = 32767
    full = xm.Mixer(48000, 48000, 2, "s16")
    full.set_tracks(SPAN_RAMPS)
    ref = full.process(x)
    assert bits_equal(ref, CO.batch_mix_s16(x, SPAN_RAMPS, threads=4)[0])
    parts = np.zeros((2, B, N * 2), np.int32)
    for h in range(2):
        m = xm.Mixer(48000, 48000, 2, "s16", mem="device")
        m.set_tracks(SPAN_RAMPS[8 * h: 8 * h + 8])
        xh = np.ascontiguousarray(x[:, 8 * h: 8 * h + 8])
        m.process_partial_strided(xh.ctypes.data, N * 2, 8 * N * 2, parts[h].ctypes.data, N * 2, B, N)
        for b in range(B):
            want = O.mix_s16_partial(list(x[b, 8 * h: 8 * h + 8]), SPAN_RAMPS[8 * h: 8 * h + 8]).reshape(-1)
            assert bits_equal(parts[h, b], want), (h, b)
    y = np.empty((B, N, 2), np.int16)
    m.finish_s16(parts.ctypes.data, 2, B * N * 2, N * 2, y.ctypes.data, N * 2, B, N)
    assert bits_equal(y, ref)
    ms = xm.Mixer(48000, 48000, 2, "s16")
    ms.set_tracks(SPAN_RAMPS)
    y2 = np.empty_like(y)
    ms.mix_spanning_s16([x.ctypes.data], N * 2, ntr * N * 2, [y2.ctypes.data], N * 2, B, N)   # one "device": no exchange
    assert bits_equal(y2, ref)


def test_cpu_effects_create_forms(xm):
    """xm_effects_create(rate, ch, 0) and XM_DEVICE_CPU make CPU chains; a
    CPU chain attaches to a CPU mixer; set_stream is accepted and ignored."""
    lib = xm._lib
    h = lib.xm_effects_create(48000, 2, 0)
    assert h
    import ctypes as C
    assert lib.xm_effects_n_devices(h) == 1
    hp = C.c_void_p(h)
    lib.xm_effects_freep(C.byref(hp))
    z = golden("effects.npz")
    e = xm.Effects(44100, 2)
    for s in z["sos"]:
        e.add_biquad(s)
    e.set_stream(12345)   # no stream on the CPU: a no-op
    m = xm.Mixer(48000, 44100, 2, "f32")
    m.set_stream(12345)
    m.set_track_effects(e)
    x = np.stack([O.gen_f32(SEED, 950 + t, 2, 9600) for t in range(2)])[None]
    m.set_tracks([dict(gain0=0.5), dict(gain0=0.25)])
    y = m.process(x)[0]
    r = [CO.biquad_f32(CO.resample_f32(t, 147, 160), z["sos"]) for t in x[0]]
    assert bits_equal(y, CO.mix_f32(r, [dict(gain0=0.5), dict(gain0=0.25)]))


def test_gpu_handles_never_fall_back_to_the_cpu(xm):
    """No GPU: a GPU handle (n_devices >= 1, a device list, a device
    ordinal) still fails with XM_EDEVICE; only n_devices = 0 / XM_DEVICE_CPU
    selects the CPU backend."""
    if xm.device_count() > 0:
        pytest.skip("GPU present")
    for kw in (dict(device=0), dict(n_devices=1, device=0), dict(n_devices=2, device=0), dict(devices=[0])):
        with pytest.raises(xm.XmError) as e:
            xm._m.Mixer(48000, 44100, 2, "f32", **kw)
        assert e.value.code == xm.XM_EDEVICE, kw
    with pytest.raises(xm.XmError) as e:
        xm._m.Effects(48000, 2, device=0)
    assert e.value.code == xm.XM_EDEVICE
    a = np.empty((1, 16, 2), np.float32)
    with pytest.raises(xm.XmError):
        xm._m.synth(a.ctypes.data, "f32", SEED, 0, 1, 2, 16, device=0)
