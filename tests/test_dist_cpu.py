"""Multi-rank path on CPU (gloo, world size 2): the same rank plumbing bench.py
uses on GPUs (xmaudio.dist).  Each rank mixes ITS block of mixes, identified by
global clip ids, with the C oracle (this host has no GPU), and the union of the
rank outputs must equal one process doing every mix; the job time is the max
over ranks.  No collective touches the data path: only barriers, the timing
all-reduce and, here, a digest gather for the check."""
import hashlib
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

MIXES_PER_RANK, NT, N = 2, 8, 4802


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(first_mix, n_mix):
    import c_oracle as CO
    from bench import SEED
    x = np.empty((n_mix, NT, N, 2), np.float32)
    for b in range(n_mix):
        for t in range(NT):
            x[b, t] = CO.gen_f32(SEED, (first_mix + b) * NT + t, 2, N)
    return x


def _digests(y):
    return [hashlib.sha256(np.ascontiguousarray(y[b]).tobytes()).hexdigest() for b in range(y.shape[0])]


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    for p in (os.path.join(ROOT, "xm-audio-utils_amd"), os.path.join(ROOT, "oracle"), ROOT):
        sys.path.insert(0, p)
    import torch.distributed as dist
    import c_oracle as CO
    from bench import RAMPS
    from xmaudio import dist as xd

    rk = xd.from_env()
    xd.init(rk, "gloo")
    first, n = xd.mix_block(rk, MIXES_PER_RANK)
    assert xd.first_clip(rk, MIXES_PER_RANK, NT) == first * NT
    y, _ = CO.batch_resample_mix_f32(_inputs(first, n), RAMPS, 147, 160, threads=1)
    gathered = [None] * rk.world
    dist.all_gather_object(gathered, _digests(y))
    slowest = xd.max_over_ranks(rk, float(rank + 1))
    xd.barrier(rk)
    xd.finish(rk)
    q.put((rank, gathered, slowest))


def test_two_rank_shards_union_equals_single_process():
    import c_oracle as CO
    from bench import RAMPS
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    y_all, _ = CO.batch_resample_mix_f32(_inputs(0, world * MIXES_PER_RANK), RAMPS, 147, 160, threads=2)
    want = _digests(y_all)
    for rank, gathered, slowest in res:
        assert slowest == float(world)                       # max over ranks
        assert sum(gathered, []) == want                     # rank r owns mixes [2r, 2r+2)


# ---- config 5 (BASELINE.json:11): tracks of every mix spread over the ranks
B5, NT5, F5 = 4, 64, 3001
_R5 = [(32768, 32768, 0, 0, 0), (0, 32768, 100, 2000, 0), (65535, 100, 0, 3001, 0),
       (16384, 16384, 0, 0, 0), (0, 0, 500, 900, 1), (0, 32768, 500, 900, 0),
       (40000, 3, 2000, 13, 0), (7, 60000, 1500, 0, 0)]
RAMPS5 = [dict(gain0_q15=q, gain1_q15=q2, ramp_start=s, ramp_len=ln, mode=md) for q, q2, s, ln, md in _R5 * 8]


def _tracks5(b):
    import np_oracle as O
    from bench import SEED
    tr = [O.gen_s16(SEED, 64 * b + t, 2, F5) for t in range(NT5)]
    for t in range(6):              # loud tracks: the 64-track sum saturates
        tr[t][50:150] = 32767
        tr[NT5 - 1 - t][400:480] = -32768
    return tr


class _OracleMixer:
    """CPU stand-in for the two config-5 entry points of xmaudio.Mixer
    (process_partial_strided / finish_s16: same pointer-and-stride
    signatures, host memory), so the gloo test drives xmaudio.dist's own
    mix_spanning_s16 end to end.  The kernels themselves are GPU-tested."""

    def __init__(self, ramps):
        self.ramps = ramps

    def out_frames(self, n):
        return n                    # 48 kHz -> 48 kHz

    @staticmethod
    def _view(ptr, dtype, n):
        import ctypes
        return np.ctypeslib.as_array((ctypes.c_byte * (n * np.dtype(dtype).itemsize)).from_address(ptr)).view(dtype)

    def process_partial_strided(self, in_ptr, ts, ms, part_ptr, pms, batch, frames):
        import np_oracle as O
        C = 2
        x = self._view(in_ptr, np.int16, batch * ms)
        part = self._view(part_ptr, np.int32, batch * pms)
        for b in range(batch):
            tracks = [x[b * ms + t * ts: b * ms + t * ts + frames * C].reshape(frames, C)
                      for t in range(len(self.ramps))]
            part[b * pms: b * pms + frames * C] = O.mix_s16_partial(tracks, self.ramps).reshape(-1)

    def finish_s16(self, parts_ptr, n_parts, part_stride, pms, out_ptr, oms, batch, out_frames):
        import np_oracle as O
        assert n_parts == 1
        S = out_frames * 2
        p = self._view(parts_ptr, np.int32, batch * pms)
        o = self._view(out_ptr, np.int16, batch * oms)
        for b in range(batch):
            o[b * oms: b * oms + S] = O.sat16(p[b * pms: b * pms + S].astype(np.int64))


def _worker5(rank, world, port, q, chunks=1):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    for p in (os.path.join(ROOT, "xm-audio-utils_amd"), os.path.join(ROOT, "oracle"), ROOT):
        sys.path.insert(0, p)
    import torch
    from xmaudio import dist as xd

    rk = xd.from_env()
    xd.init(rk, "gloo")
    per = NT5 // world
    mine = range(per * rank, per * (rank + 1))        # this rank's tracks of every mix
    x = torch.from_numpy(np.stack([np.stack([_tracks5(b)[t] for t in mine]) for b in range(B5)]))
    y = xd.mix_spanning_s16(rk, _OracleMixer([RAMPS5[t] for t in mine]), x, chunks=chunks)
    first, n = xd.owned_mixes(rk, B5)
    assert y.shape == (n, F5, 2)
    xd.finish(rk)
    q.put((rank, first, y.numpy()))


@pytest.mark.parametrize("chunks", [1, 2])
def test_two_rank_spanning_mixdown_equals_full_mix(chunks):
    """Config 5 exchange on CPU: each rank holds half of the 64 tracks of every
    mix, forms the int32 Q15 partial, the partials meet in reduce-scatters
    (RCCL on GPUs, gloo here; chunks = 2: two asynchronous reduce-scatters,
    each overlapping the next chunk's partials) and the owner saturates: every
    mix equals the one-process 64-track mix bit for bit, saturation included."""
    import np_oracle as O
    from xmaudio import dist as xd
    assert xd.span_chunks(chunks, B5 // 2) == chunks
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker5, args=(r, world, port, q, chunks)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = {}
    for rank, first, y in res:
        for i in range(y.shape[0]):
            got[first + i] = y[i]
    assert sorted(got) == list(range(B5))
    sat = 0
    for b in range(B5):
        want = O.mix_s16(_tracks5(b), RAMPS5)
        sat += int(np.sum(np.abs(want.astype(np.int32)) >= 32767))
        assert np.array_equal(got[b], want), b
    assert sat > 0                  # the test exercises saturation
