"""The headline workload at its production size (BASELINE.json:2, bench.py):
512 mixes x 8 stereo fp32 tracks x 480000 frames, 48 kHz -> 44.1 kHz + gain
ramps + ordered track sum, in HBM.  This is the grid the bench times
(pick_split: 94 super-periods per lane, 4 tasks per mix, 2048 waves), which
the smaller parity cases do not reach; the first and the last mix (the last
waves of the grid) are bit-compared with the C oracle, and the fused kernel
must be the one that ran."""
import numpy as np
import pytest

from conftest import bits_equal

import c_oracle as CO

pytestmark = pytest.mark.gpu


def _run(xm, B, N, ramps):
    import torch
    from bench import SEED
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    m.set_tracks(ramps)
    F = m.out_frames(N)
    x = torch.empty((B, 8, N, 2), dtype=torch.float32, device="cuda")
    y = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    xm.synth(x.data_ptr(), "f32", SEED, 0, B * 8, 2, N)
    torch.cuda.synchronize()
    m.process_strided(x.data_ptr(), N * 2, 8 * N * 2, y.data_ptr(), F * 2, B, N)
    t = m.timing()
    assert t.n_launches == 1 and t.fast_launches == 1, (t.n_launches, t.fast_launches)
    return x, y


@pytest.mark.parametrize("B", [512, 64])
def test_headline_grid_first_last_mix(xm, gpu, B):
    from bench import RAMPS
    N = 480000
    x, y = _run(xm, B, N, RAMPS)
    idx = [0, B - 1]
    ref, _ = CO.batch_resample_mix_f32(x[idx].cpu().numpy(), RAMPS, 147, 160, threads=2)
    got = y[idx].cpu().numpy()
    assert bits_equal(got, ref)
    # no output frame was left unwritten anywhere in the batch
    assert not bool(y.isnan().any())


@pytest.mark.parametrize("N", [48001, 160 * 300 + 1, 160 * 300 + 33, 4801, 441001])
def test_fast_kernel_odd_lengths(xm, gpu, N):
    """Odd frame counts stay on the fused kernel: the last chunk (frames N-1,
    N) is loaded and frame N (the next track's first sample or padding) is
    zeroed on the copy.  Lengths around a super-period edge and at a DMA
    segment edge; every mix bit-compared with the oracle."""
    from bench import RAMPS
    B = 3
    x, y = _run(xm, B, N, RAMPS)
    ref, _ = CO.batch_resample_mix_f32(x.cpu().numpy(), RAMPS, 147, 160, threads=2)
    assert bits_equal(y.cpu().numpy(), ref)


@pytest.mark.parametrize("N", [48001, 9601])
def test_fast_split_odd_lengths(xm, gpu, N):
    """Resample-only (config 2 split mode, 8 clips per pseudo-mix) with odd N:
    per-clip outputs, no leakage between neighbouring clips."""
    import torch
    from bench import SEED
    B = 16
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    m.set_tracks([dict(gain0=1.0)])
    F = m.out_frames(N)
    x = torch.empty((B, N, 2), dtype=torch.float32, device="cuda")
    xm.synth(x.data_ptr(), "f32", SEED, 77, B, 2, N)
    y = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    m.process_strided(x.data_ptr(), N * 2, N * 2, y.data_ptr(), F * 2, B, N)
    t = m.timing()
    assert t.fast_launches == 1, (t.n_launches, t.fast_launches)
    xs = x.cpu().numpy()
    got = y.cpu().numpy()
    for b in (0, 7, 8, 15):
        assert bits_equal(got[b], CO.resample_f32(xs[b], 147, 160)), b


@pytest.mark.parametrize("N", [48000, 48001])
def test_fast_kernel_pointer_tables_4gb_apart(xm, gpu, N):
    """Tracks of one mix 4.5 GB apart (the two ends of one 4.6 GB tensor) and
    mixes mixing near and far tracks: the FAR kernel (a 64-bit base per track
    row), bit-exact, fast_launches == 1; 5 mixes leave padding waves."""
    import torch
    from bench import RAMPS, SEED
    B = 5
    fl = 2 * N
    big = torch.empty(4_600_000_000 // 4, dtype=torch.float32, device="cuda")
    # track t of mix b at the low end for even t, the high end for odd t
    lo = [b * 8 * fl + t * fl for b in range(B) for t in range(8)]
    hi = [big.numel() - (1 + b * 8 + t) * fl for b in range(B) for t in range(8)]
    offs = [lo[i] if i % 2 == 0 else hi[i] for i in range(B * 8)]
    offs[3 * 8 + 5] = lo[3 * 8 + 5]   # mix 3: one more low track
    for i, o in enumerate(offs):
        xm.synth(big[o:].data_ptr(), "f32", SEED, 900 + i, 1, 2, N)
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    m.set_tracks(RAMPS)
    F = m.out_frames(N)
    y = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    m.process_ptrs([big[o:].data_ptr() for o in offs], [y[b].data_ptr() for b in range(B)], B, N)
    torch.cuda.synchronize()
    t = m.timing()
    assert t.n_launches == 1 and t.fast_launches == 1, (t.n_launches, t.fast_launches)
    assert (max(offs) - min(offs)) * 4 > 4 << 30
    got = y.cpu().numpy()
    for b in range(B):
        tracks = [big[offs[b * 8 + t]: offs[b * 8 + t] + fl].view(N, 2).cpu().numpy() for t in range(8)]
        assert bits_equal(got[b], CO.resample_mix_f32(tracks, RAMPS, 147, 160)), b
    del big
    torch.cuda.empty_cache()


@pytest.mark.parametrize("own_alloc", [False, True])
@pytest.mark.parametrize("N", [48000, 48001])
def test_fast_kernel_pointer_tables(xm, gpu, N, own_alloc):
    """Irregular per-track pointer tables stay on the fused kernel (one
    buffer resource per mix based at its lowest track, per-track offsets
    from the table; a mix whose tracks span 2 GB or more runs the FAR
    kernel, one resource per track): tracks in scattered order inside one
    tensor, plus (with own_alloc) one mix whose tracks are separate
    allocations; outputs through a table too."""
    import torch
    from bench import RAMPS, SEED
    B = 4
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    m.set_tracks(RAMPS)
    F = m.out_frames(N)
    x = torch.empty((B, 8, N, 2), dtype=torch.float32, device="cuda")
    xm.synth(x.data_ptr(), "f32", SEED, 300, B * 8, 2, N)
    own = [x[B - 1, t].clone() if own_alloc else x[B - 1, t] for t in range(8)]   # the last mix: its own allocations
    perm = [(3 * t + 5) % 8 for t in range(8)]
    ins = [x[b, perm[t]].data_ptr() for b in range(B - 1) for t in range(8)] + [o.data_ptr() for o in own]
    y = torch.full((B + 2, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    outs = [y[(5 * b) % (B + 2)].data_ptr() for b in range(B)]
    torch.cuda.synchronize()
    m.process_ptrs(ins, outs, B, N)
    torch.cuda.synchronize()
    t = m.timing()
    assert t.n_launches == 1 and t.fast_launches == 1, (t.n_launches, t.fast_launches)
    xs = x.cpu().numpy()
    got = y.cpu().numpy()
    for b in range(B):
        tracks = [xs[b, perm[t]] for t in range(8)] if b < B - 1 else [xs[b, t] for t in range(8)]
        assert bits_equal(got[(5 * b) % (B + 2)], CO.resample_mix_f32(tracks, RAMPS, 147, 160)), b


def test_fast_split_pointer_table(xm, gpu):
    """Resample-only with an input pointer table (clips in a scattered order)."""
    import torch
    from bench import SEED
    B, N = 16, 9600 + 1
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    m.set_tracks([dict(gain0=1.0)])
    F = m.out_frames(N)
    x = torch.empty((B, N, 2), dtype=torch.float32, device="cuda")
    xm.synth(x.data_ptr(), "f32", SEED, 900, B, 2, N)
    y = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    perm = [(5 * b + 3) % B for b in range(B)]
    m.process_ptrs([x[perm[b]].data_ptr() for b in range(B)], [y[b].data_ptr() for b in range(B)], B, N)
    torch.cuda.synchronize()
    assert m.timing().fast_launches == 1
    xs, got = x.cpu().numpy(), y.cpu().numpy()
    for b in (0, 5, 15):
        assert bits_equal(got[b], CO.resample_f32(xs[perm[b]], 147, 160)), b


def test_split_production_grid_first_last_clip(xm, gpu):
    """Config 2 at its production size (BASELINE.json:8): 4096 stereo 10 s
    fp32 clips resampled 48k -> 44.1k in split mode (8 clips per pseudo-mix
    on the fused kernel, 512 pseudo-mixes); the first and last clip of each
    end of the grid bit-compared with the oracle, nothing left unwritten."""
    import torch
    from bench import SEED
    B, N = 4096, 480000
    m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
    m.set_tracks([dict(gain0=1.0)])
    F = m.out_frames(N)
    x = torch.empty((B, N, 2), dtype=torch.float32, device="cuda")
    xm.synth(x.data_ptr(), "f32", SEED, 0, B, 2, N)
    y = torch.full((B, F, 2), float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    m.process_strided(x.data_ptr(), N * 2, N * 2, y.data_ptr(), F * 2, B, N)
    torch.cuda.synchronize()
    t = m.timing()
    assert t.n_launches == 1 and t.fast_launches == 1, (t.n_launches, t.fast_launches)
    for b in (0, 7, 8, B - 8, B - 1):
        assert bits_equal(y[b].cpu().numpy(), CO.resample_f32(x[b].cpu().numpy(), 147, 160)), b
    assert not bool(y.isnan().any())
