"""Split mode (2-8 clips or mixes per wave, 48k -> 44.1k, f32) with output
rows off the 64-B grid (round 6).  Config 2's segment stores write whole
64-B output segments on each row's own address grid; rows whose stride is
not a multiple of 64 B (most clip lengths: F x 8 B) go to the odd kernels,
where every row of a wave has its own phase.  Each case must be one fused
launch, equal the C oracle bit for bit, and leave the padding between rows
untouched: strides F + d frames for d = 1..9, even and odd N, 1-track rows
(config 2's form) and 2- and 4-track mixes, clips with several super-period
runs per lane, and an output base 8 B off the grid; then 1-track rows at
the other ratios (2/1, 3/2, 1/2 on the odd kernels' segment stores; 2/3,
320/147 and 160/147, which have one kernel, on their plain stores)."""
import numpy as np
import pytest

from conftest import bits_equal

import c_oracle as CO
import np_oracle as O

pytestmark = pytest.mark.gpu
RAMPS = [dict(gain0=0.9), dict(gain0=0.0, gain1=0.8, ramp_start=41, ramp_len=3000),
         dict(mode=1, ramp_start=900, ramp_len=700), dict(gain0=0.3, gain1=0.6, ramp_start=5000)]


def _run(xm, ntr, B, N, d, base=0, split_r=None, monkeypatch=None, fi=48000, fo=44100):
    import torch
    from bench import SEED
    if split_r:
        monkeypatch.setenv("XM_FAST_SPLIT_R", str(split_r))
    m = xm.Mixer(fi, fo, 2, "f32", mem="device")
    ramps = [dict(gain0=1.0)] if ntr == 1 else RAMPS[:ntr]
    m.set_tracks(ramps)
    F = m.out_frames(N)
    st = F + d                                   # output stride in frames
    x = torch.empty((B, ntr, N, 2), dtype=torch.float32, device="cuda")
    xm.synth(x.data_ptr(), "f32", SEED, 300 + 7 * d + N % 5, B * ntr, 2, N)
    yb = torch.full((B * st * 2 + base + 64,), float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    m.process_strided(x.data_ptr(), N * 2, ntr * N * 2, yb[base:].data_ptr(), st * 2, B, N)
    torch.cuda.synchronize()
    t = m.timing()
    assert t.n_launches == 1 and t.fast_launches == 1, (t.n_launches, t.fast_launches)
    y = yb.cpu().numpy()[base:base + B * st * 2].reshape(B, st, 2)
    L, M = O.reduce_ratio(fi, fo)
    ref, _ = CO.batch_resample_mix_f32(x.cpu().numpy(), ramps, L, M, threads=4)
    for b in range(B):
        assert bits_equal(y[b, :F], ref[b]), (ntr, N, d, b)
        assert np.isnan(y[b, F:]).all(), ("padding written", ntr, N, d, b)
    assert np.isnan(yb.cpu().numpy()[:base]).all() and np.isnan(yb.cpu().numpy()[base + B * st * 2:]).all()


@pytest.mark.parametrize("d", [1, 2, 3, 4, 5, 7, 9])
@pytest.mark.parametrize("N", [48000, 48001])
def test_split_rows_off_grid(xm, gpu, N, d):
    """Config 2's form: 1-track rows, 8 per wave (17 rows: a partial wave)."""
    _run(xm, 1, 17, N, d)


@pytest.mark.parametrize("ntr", [2, 4])
@pytest.mark.parametrize("d", [1, 3, 8])
def test_split_mixes_off_grid(xm, gpu, ntr, d):
    """2- and 4-track mixes, 4 and 2 per wave."""
    _run(xm, ntr, 9, 48000, d)


@pytest.mark.parametrize("base", [2, 8])
def test_split_rows_base_and_stride_off_grid(xm, gpu, base):
    """An output base 8 and 32 B off the grid as well (base in floats)."""
    _run(xm, 1, 16, 48000, 3, base=base)


@pytest.mark.parametrize("R", [2, 5])
def test_split_rows_off_grid_multi_sp(xm, gpu, R, monkeypatch):
    """Lanes walking several super-periods: the open segment at each run's end."""
    _run(xm, 1, 16, 96000, 5, split_r=R, monkeypatch=monkeypatch)


@pytest.mark.parametrize("d", [1, 3, 4, 8])
@pytest.mark.parametrize("fi,fo,N", [(24000, 48000, 24000), (24000, 48000, 24001), (32000, 48000, 32000),
                                     (96000, 48000, 96000), (48000, 32000, 48000), (22050, 48000, 22050),
                                     (44100, 48000, 44100)])
def test_split_rows_off_grid_other_ratios(xm, gpu, fi, fo, N, d):
    _run(xm, 1, 17, N, d, fi=fi, fo=fo)


@pytest.mark.parametrize("fi,fo", [(24000, 48000), (32000, 48000), (96000, 48000)])
def test_split_rows_off_grid_other_ratios_base_multi_sp(xm, gpu, fi, fo, monkeypatch):
    _run(xm, 1, 16, 4 * fi, 5, base=2, split_r=3, monkeypatch=monkeypatch, fi=fi, fo=fo)
