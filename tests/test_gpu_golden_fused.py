"""The fused kernels against scipy directly, at every ratio they serve
(VERDICT r5 item 2).

tests/golden/resample_fused.npz holds scipy 1.15.3 `resample_poly` outputs
(tools/gen_golden.py FUSED_CASES) at 320/147, 2/1, 3/1, 1/2, 2/3, 3/2 and
147/320, stereo and mono, with lengths around the super-period edges, and
mono s16 at odd N at 160/147 and 147/160 (config 1's form).  Until round 5
the fused kernels at these ratios were checked only against the C oracle;
here each golden clip runs through the C ABI in two shapes and must equal
scipy's output bit for bit:
  * an 8-track mix whose track 0 is the golden clip at unity gain and whose
    other tracks are other clips at gain 0 (f32: 1·r + 0·r' + ... == r, the
    final +0 keeps the sign of zero; Q15: (s·32768 + 2¹⁴) >> 15 == s and
    (s·0 + 2¹⁴) >> 15 == 0), every mix of the batch the same;
  * a batch of 1-track rows (resample only) of the golden clip.
Where a fused kernel serves the shape the call must be
one fused launch (`fast_launches == 1`); the other shapes run on the generic
kernel and are checked against the same goldens.  tests/test_cpu_backend.py
re-runs both tests on the host CPU backend.
"""
import numpy as np
import pytest

from conftest import bits_equal, golden

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
SEED = O.SEED


def _cases():
    z = golden("resample_fused.npz")
    return sorted(k[:-6] for k in z.files if k.endswith("__meta"))


def _case(name):
    z = golden("resample_fused.npz")
    fi, fo, N, Cc, clip, bits = (int(v) for v in z[f"{name}__meta"])
    s16 = bits == 16
    x = CO.gen_s16(SEED, clip, Cc, N) if s16 else CO.gen_f32(SEED, clip, Cc, N)
    return fi, fo, N, Cc, s16, x, z[f"{name}__y"]


# fused shapes by (L, M): DESIGN.md §4.1 (kernels) and §8 (what stays generic)
_TABLE = {(147, 160), (160, 147)}
_SMALL = {(3, 2), (2, 3), (1, 2)}
_UPS = {(2, 1), (3, 1)}


def _fused_mix(L, M, Cc, s16):
    if s16:   # Q15 mixes: stereo (IO 2; 2/1, 3/1, 320/147 since round 6) and mono (M16)
        return (L, M) != (147, 320) if Cc == 2 else (L, M) in _TABLE | _SMALL
    if Cc == 2:
        return True   # every ratio here: k_rs147_mix (RID), RID_U2, k_rs_d2_mix
    return (L, M) != (147, 320)   # mono f32: 147/320 mono stays generic


def _fused_row(L, M, Cc, s16):
    if s16:
        return Cc == 1 and (L, M) in _TABLE | _SMALL   # M16 one-track rows
    if Cc == 2:
        return (L, M) != (3, 1)   # 3/1 stereo 1-track rows stay generic
    return (L, M) != (147, 320)


def _unity(s16):
    return dict(gain0_q15=32768) if s16 else dict(gain0=1.0)


def _zero(s16):
    return dict(gain0_q15=0) if s16 else dict(gain0=0.0)


def _check_fast(m, fused):
    t = m.timing()
    assert t.n_launches == 1, t.n_launches
    assert t.fast_launches == (m.fused if fused else 0), (t.fast_launches, fused)


@pytest.mark.parametrize("name", _cases())
def test_fused_mix_equals_scipy(xm, gpu, name):
    fi, fo, N, Cc, s16, x, y = _case(name)
    L, M = O.reduce_ratio(fi, fo)
    B, nt = 3, 8
    gen = CO.gen_s16 if s16 else CO.gen_f32
    xb = np.stack([np.stack([x] + [gen(SEED, 90000 + 16 * b + t, Cc, N) for t in range(1, nt)]) for b in range(B)])
    m = xm.Mixer(fi, fo, Cc, "s16" if s16 else "f32")
    m.set_tracks([_unity(s16)] + [_zero(s16)] * (nt - 1))
    out = m.process(xb)
    _check_fast(m, _fused_mix(L, M, Cc, s16))
    for b in range(B):
        assert bits_equal(out[b], y), (name, b)


@pytest.mark.parametrize("name", _cases())
def test_fused_rows_equal_scipy(xm, gpu, name):
    fi, fo, N, Cc, s16, x, y = _case(name)
    L, M = O.reduce_ratio(fi, fo)
    B = 9   # one full wave of 8 one-track rows and one more
    m = xm.Mixer(fi, fo, Cc, "s16" if s16 else "f32")
    m.set_tracks([_unity(s16)])
    out = m.process(np.stack([x[None]] * B))
    _check_fast(m, _fused_row(L, M, Cc, s16))
    for b in range(B):
        assert bits_equal(out[b], y), (name, b)


@pytest.mark.parametrize("name", [n for n in _cases() if int(n.rsplit("_", 1)[1]) > 1000])
def test_fused_multi_sp_equals_scipy(xm, gpu, name, monkeypatch):
    """The longer golden clips with every lane walking several super-periods
    (XM_FAST_SPLIT_R; mono runs are cut in two halves, so R >= 4)."""
    fi, fo, N, Cc, s16, x, y = _case(name)
    L, M = O.reduce_ratio(fi, fo)
    monkeypatch.setenv("XM_FAST_SPLIT_R", "4" if Cc == 1 else "2")
    gen = CO.gen_s16 if s16 else CO.gen_f32
    xb = np.stack([np.stack([x] + [gen(SEED, 91000 + t, Cc, N) for t in range(1, 8)])] * 2)
    m = xm.Mixer(fi, fo, Cc, "s16" if s16 else "f32")
    m.set_tracks([_unity(s16)] + [_zero(s16)] * 7)
    out = m.process(xb)
    _check_fast(m, _fused_mix(L, M, Cc, s16))
    for b in range(2):
        assert bits_equal(out[b], y), (name, b)
