"""ctypes wrapper of the C restatement (oracle/build/libxm_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg; never by the product library.  Build with
`make -C oracle` (or __graft_entry__.build()).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libxm_oracle.so")
GOLDEN = os.path.join(os.path.dirname(_HERE), "tests", "golden")


class _Ramp(C.Structure):   # == XmGainRamp in include/xm_audio_common.h
    _fields_ = [("gain0", C.c_float), ("gain1", C.c_float), ("gain0_q15", C.c_int32),
                ("gain1_q15", C.c_int32), ("ramp_start", C.c_int64), ("ramp_len", C.c_int64),
                ("mode", C.c_int32), ("reserved", C.c_int32)]


def _ramps(rs):
    arr = (_Ramp * len(rs))()
    for a, r in zip(arr, rs):
        a.gain0 = r.get("gain0", 1.0)
        a.gain1 = r.get("gain1", a.gain0)
        a.gain0_q15 = r.get("gain0_q15", 32768)
        a.gain1_q15 = r.get("gain1_q15", a.gain0_q15)
        a.ramp_start = r.get("ramp_start", 0)
        a.ramp_len = r.get("ramp_len", 0)
        a.mode = r.get("mode", 0)
    return arr


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built (make -C oracle)")
        _lib = C.CDLL(LIB_PATH)
        vp, sz, i = C.c_void_p, C.c_size_t, C.c_int
        _lib.xo_gen_f32.argtypes = [C.c_uint64, C.c_uint64, i, sz, vp]
        _lib.xo_gen_s16.argtypes = [C.c_uint64, C.c_uint64, i, sz, vp]
        _lib.xo_resample_f32.argtypes = [vp, i, i, i, i, vp, sz, i, vp]
        _lib.xo_resample_s16.argtypes = [vp, i, i, i, i, vp, sz, i, vp]
        _lib.xo_mix_s16.argtypes = [vp, vp, i, sz, i, vp]
        _lib.xo_mix_f32.argtypes = [vp, vp, i, sz, i, vp]
        _lib.xo_resample_mix_f32.argtypes = [vp, i, i, i, i, vp, vp, i, sz, i, vp]
        _lib.xo_resample_mix_s16.argtypes = [vp, i, i, i, i, vp, vp, i, sz, i, vp]
        _lib.xo_biquad_f32.argtypes = [vp, i, vp, sz, i, vp]
        _lib.xo_fir_f32.argtypes = [vp, i, vp, sz, i, vp]
        _lib.xo_batch_resample_mix_f32.argtypes = [vp, i, i, i, i, vp, vp, i, sz, sz, i, vp, i]
        _lib.xo_batch_resample_mix_f32.restype = i
        _lib.xo_batch_mix_s16.argtypes = [vp, vp, i, sz, sz, i, vp, i]
        _lib.xo_batch_mix_s16.restype = i
    return _lib


def table(L: int, M: int):
    """scipy-generated table committed in tests/golden/tables.npz."""
    z = np.load(os.path.join(GOLDEN, "tables.npz"))
    H = np.ascontiguousarray(z[f"H_{L}_{M}"], np.float32)
    meta = z[f"meta_{L}_{M}"]
    return H, int(meta[2]), int(meta[3])   # H, T, rm


def _p(a):
    return a.ctypes.data


def gen_f32(seed, clip, channels, frames):
    y = np.empty((frames, channels), np.float32)
    lib().xo_gen_f32(seed, clip, channels, frames, _p(y))
    return y


def gen_s16(seed, clip, channels, frames):
    y = np.empty((frames, channels), np.int16)
    lib().xo_gen_s16(seed, clip, channels, frames, _p(y))
    return y


def resample_f32(x, L, M, H=None, rm=None):
    if H is None:
        H, _, rm = table(L, M)
    x = np.ascontiguousarray(x, np.float32)
    x2 = x if x.ndim == 2 else x[:, None]
    N, Cc = x2.shape
    y = np.empty(((N * L + M - 1) // M, Cc), np.float32)
    lib().xo_resample_f32(_p(H), L, M, H.shape[1], rm, _p(x2), N, Cc, _p(y))
    return y if x.ndim == 2 else y[:, 0]


def resample_s16(x, L, M):
    H, _, rm = table(L, M)
    x = np.ascontiguousarray(x, np.int16)
    x2 = x if x.ndim == 2 else x[:, None]
    N, Cc = x2.shape
    y = np.empty(((N * L + M - 1) // M, Cc), np.int16)
    lib().xo_resample_s16(_p(H), L, M, H.shape[1], rm, _p(x2), N, Cc, _p(y))
    return y if x.ndim == 2 else y[:, 0]


def mix_s16(tracks, ramps):
    ts = [np.ascontiguousarray(t, np.int16) for t in tracks]
    F, Cc = ts[0].shape
    ptrs = (C.c_void_p * len(ts))(*[_p(t) for t in ts])
    y = np.empty((F, Cc), np.int16)
    lib().xo_mix_s16(ptrs, _ramps(ramps), len(ts), F, Cc, _p(y))
    return y


def mix_f32(tracks, ramps):
    ts = [np.ascontiguousarray(t, np.float32) for t in tracks]
    F, Cc = ts[0].shape
    ptrs = (C.c_void_p * len(ts))(*[_p(t) for t in ts])
    y = np.empty((F, Cc), np.float32)
    lib().xo_mix_f32(ptrs, _ramps(ramps), len(ts), F, Cc, _p(y))
    return y


def resample_mix_f32(tracks, ramps, L, M):
    H, T, rm = table(L, M)
    ts = [np.ascontiguousarray(t, np.float32) for t in tracks]
    N, Cc = ts[0].shape
    ptrs = (C.c_void_p * len(ts))(*[_p(t) for t in ts])
    y = np.empty(((N * L + M - 1) // M, Cc), np.float32)
    lib().xo_resample_mix_f32(_p(H), L, M, T, rm, ptrs, _ramps(ramps), len(ts), N, Cc, _p(y))
    return y


def resample_mix_s16(tracks, ramps, L, M):
    H, T, rm = table(L, M)
    ts = [np.ascontiguousarray(t, np.int16) for t in tracks]
    N, Cc = ts[0].shape
    ptrs = (C.c_void_p * len(ts))(*[_p(t) for t in ts])
    y = np.empty(((N * L + M - 1) // M, Cc), np.int16)
    lib().xo_resample_mix_s16(_p(H), L, M, T, rm, ptrs, _ramps(ramps), len(ts), N, Cc, _p(y))
    return y


def biquad_f32(x, sos):
    x = np.ascontiguousarray(x, np.float32)
    sos = np.ascontiguousarray(sos, np.float32)
    x2 = x if x.ndim == 2 else x[:, None]
    y = np.empty_like(x2)
    lib().xo_biquad_f32(_p(sos), sos.shape[0], _p(x2), x2.shape[0], x2.shape[1], _p(y))
    return y if x.ndim == 2 else y[:, 0]


def fir_f32(x, h):
    x = np.ascontiguousarray(x, np.float32)
    h = np.ascontiguousarray(h, np.float32)
    x2 = x if x.ndim == 2 else x[:, None]
    y = np.empty_like(x2)
    lib().xo_fir_f32(_p(h), len(h), _p(x2), x2.shape[0], x2.shape[1], _p(y))
    return y if x.ndim == 2 else y[:, 0]


def batch_resample_mix_f32(x, ramps, L, M, threads=1):
    """x: [nmix, ntr, N, C] float32 -> ([nmix, Fout, C], threads used)."""
    H, T, rm = table(L, M)
    x = np.ascontiguousarray(x, np.float32)
    nmix, ntr, N, Cc = x.shape
    y = np.empty((nmix, (N * L + M - 1) // M, Cc), np.float32)
    used = lib().xo_batch_resample_mix_f32(_p(H), L, M, T, rm, _p(x), _ramps(ramps), ntr, nmix, N, Cc,
                                           _p(y), threads)
    return y, used


def batch_mix_s16(x, ramps, threads=1):
    x = np.ascontiguousarray(x, np.int16)
    nmix, ntr, F, Cc = x.shape
    y = np.empty((nmix, F, Cc), np.int16)
    used = lib().xo_batch_mix_s16(_p(x), _ramps(ramps), ntr, nmix, F, Cc, _p(y), threads)
    return y, used
