"""API edge cases found by review, through the C ABI.

CPU suite (no GPU): the CPU backend's create-time selection, effects range
checks, fork-safety of its worker pool, and process_batch with per-track
effects, irregular mix strides and scattered outputs (bit-exact against the C
oracle).  The GPU form of the last case is in test_gpu_api_edges.py.
"""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import bits_equal, golden

import c_oracle as CO
import np_oracle as O

SEED = O.SEED
RAMPS3 = [dict(gain0=0.5), dict(gain0=0.0, gain1=0.8, ramp_start=300, ramp_len=2000), dict(mode=1, ramp_start=900, ramp_len=700)]


@pytest.fixture(scope="module")
def xm():
    import xmaudio
    return xmaudio


def _create(xm, **kw):
    cfg = xm.XmMixerConfig(kw.get("in_rate", 48000), kw.get("out_rate", 44100), 2, xm.XM_FMT_F32,
                           kw["mem"], kw["device"], 0, kw["n_devices"])
    st = C.c_int(7)
    h = xm._lib.xm_audio_mixer_create_ex(C.byref(cfg), C.byref(st))
    if h:
        hp = C.c_void_p(h)
        xm._lib.xm_audio_mixer_freep(C.byref(hp))
    return st.value


def test_cpu_selection_is_explicit_for_device_memory(xm):
    """n_devices = 0 selects the host CPU backend.  Device
    memory on it must be asked for by device = XM_DEVICE_CPU; a zero-device
    config that names a GPU ordinal with XM_MEM_DEVICE would hand HBM pointers
    to the host, so create refuses it (XM_EINVAL) instead of running."""
    assert _create(xm, mem=xm.XM_MEM_HOST, device=0, n_devices=0) == 0
    assert _create(xm, mem=xm.XM_MEM_HOST, device=xm.XM_DEVICE_CPU, n_devices=0) == 0
    assert _create(xm, mem=xm.XM_MEM_DEVICE, device=xm.XM_DEVICE_CPU, n_devices=0) == 0
    assert _create(xm, mem=xm.XM_MEM_DEVICE, device=xm.XM_DEVICE_CPU, n_devices=1) == 0
    assert _create(xm, mem=xm.XM_MEM_DEVICE, device=0, n_devices=0) == xm.XM_EINVAL
    assert _create(xm, mem=xm.XM_MEM_HOST, device=-5, n_devices=0) == xm.XM_EINVAL
    assert _create(xm, mem=xm.XM_MEM_HOST, device=0, n_devices=-1) == xm.XM_EINVAL
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device", device="cpu")
    assert m.backend == "cpu"


def test_effects_create_device_count_range(xm):
    """xm_effects_create(rate, ch, n) returns NULL outside [0, 16]."""
    lib = xm._lib
    for n in (-1, -16, 17):
        assert not lib.xm_effects_create(48000, 2, n), n
    h = lib.xm_effects_create(48000, 2, 0)
    assert h
    hp = C.c_void_p(h)
    lib.xm_effects_freep(C.byref(hp))


def _fx_irregular_case(xm, device, alloc, to_np):
    """process_batch with effects, batch > 1, mixes (ntr + 1) tracks apart
    (in_mix_stride != ntr * in_track_stride: the track-table branch of the
    effects path) and separately allocated outputs (an output pointer table):
    every mix bit-exact against the oracle, and no input overwritten."""
    z = golden("effects.npz")
    B, ntr, N = 3, 3, 4800 + 7
    x = np.stack([np.stack([O.gen_f32(SEED, 3100 + 4 * b + t, 2, N) for t in range(ntr + 1)]) for b in range(B)])
    e = xm.Effects(44100, 2, device=device)
    e.add_biquad(z["sos"][0])
    e.add_fir(z["h7"])
    e.add_biquad(z["sos"][1])
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device", device=device)
    m.set_tracks(RAMPS3)
    m.set_track_effects(e)
    F = m.out_frames(N)
    xd = alloc(x)
    outs = [alloc(np.zeros((F, 2), np.float32)) for _ in range(B)]
    ins = [xd.ptr(b, t) for b in range(B) for t in range(ntr)]
    m.process_ptrs(ins, [o.ptr() for o in outs], B, N)
    for b in range(B):
        r = [CO.biquad_f32(CO.fir_f32(CO.biquad_f32(CO.resample_f32(x[b, t], 147, 160), z["sos"][:1]), z["h7"]),
                           z["sos"][1:2]) for t in range(ntr)]
        assert bits_equal(to_np(outs[b]), CO.mix_f32(r, RAMPS3)), b
    assert bits_equal(to_np(xd), x)   # the mixdown went to the outputs, not into the tracks


class _HostBuf:
    def __init__(self, a):
        self.a = np.ascontiguousarray(a)

    def ptr(self, *idx):
        return self.a[idx].ctypes.data if idx else self.a.ctypes.data


def test_effects_irregular_strides_scattered_outputs_cpu(xm):
    _fx_irregular_case(xm, "cpu", _HostBuf, lambda b: b.a)


@pytest.mark.skipif(not hasattr(os, "fork"), reason="needs fork()")
def test_cpu_pool_survives_fork(xm):
    """A child forked after the parent used the CPU backend's worker pool
    runs its own parallel calls (Python multiprocessing's fork start method):
    the child's mix completes and is bit-exact; the parent's pool still works."""
    B, N = 6, 9600
    x = np.stack([np.stack([O.gen_f32(SEED, 3300 + 8 * b + t, 2, N) for t in range(3)]) for b in range(B)])
    ref, _ = CO.batch_resample_mix_f32(x, RAMPS3, 147, 160, threads=4)
    m = xm.Mixer(48000, 44100, 2, "f32", device="cpu")
    m.set_tracks(RAMPS3)
    assert bits_equal(m.process(x), ref)   # the pool exists now
    pid = os.fork()
    if pid == 0:   # child: exit code 0 iff its own mix is right
        code = 1
        try:
            import signal
            signal.alarm(60)   # a pool waiting on the parent's workers would hang: fail instead
            code = 0 if bits_equal(m.process(x), ref) else 2
        finally:
            os._exit(code)
    _, status = os.waitpid(pid, 0)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0, status
    assert bits_equal(m.process(x), ref)
