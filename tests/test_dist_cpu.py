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
