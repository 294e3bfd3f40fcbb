"""Rank plumbing for multi-GPU runs.

Mixes are independent, so N GPUs are N processes, each owning a contiguous
block of mixes (bench.py: 4096 clips in total split over the ranks, strong
scaling) with no collective in the data path.  torch.distributed (RCCL = backend "nccl" on ROCm, or "gloo"
on CPU for tests) is used for the start/stop barriers and the max-over-ranks
wall time, and for the one real exchange of the path: config 5
(BASELINE.json:11), where the tracks of every mix are spread over the ranks
and the int32 partial sums meet in a reduce-scatter (reduce_partials).
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass(frozen=True)
class Rank:
    rank: int
    world: int
    local: int


def from_env() -> Rank:
    """RANK / WORLD_SIZE / LOCAL_RANK as torchrun sets them (single process: 0/1/0)."""
    return Rank(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                int(os.environ.get("LOCAL_RANK", "0")))


def init(r: Rank, backend: str, device=None) -> None:
    """Join the process group (no-op for world 1); rendezvous on 127.0.0.1."""
    if r.world <= 1:
        return
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if device is not None:
        dist.init_process_group(backend, device_id=device)
    else:
        dist.init_process_group(backend)


def mix_block(r: Rank, mixes_per_rank: int) -> tuple[int, int]:
    """(first global mix, count) owned by this rank."""
    return r.rank * mixes_per_rank, mixes_per_rank


def first_clip(r: Rank, mixes_per_rank: int, tracks: int) -> int:
    """Global clip id of track 0 of this rank's first mix (clip = mix*tracks + track)."""
    return mix_block(r, mixes_per_rank)[0] * tracks


def owned_mixes(r: Rank, batch: int) -> tuple[int, int]:
    """Config 5: (first, count) of the mixes rank r finishes after the exchange."""
    if batch % r.world:
        raise ValueError(f"batch {batch} does not divide over {r.world} ranks")
    n = batch // r.world
    return r.rank * n, n


def reduce_partials(r: Rank, part):
    """Config 5 exchange.  `part` is this rank's [batch, S] int32 Q15 partial
    (xm_audio_mixer_process_partial_s16 over the tracks it holds); returns the
    [batch/world, S] block of the mixes owned_mixes() gives this rank, summed
    over every rank, from one reduce-scatter (RCCL over xGMI on GPUs, gloo in
    the CPU tests: the same call on every backend).  int32 sums of <= 64 Q15
    terms cannot overflow, so any order is exact and the collective's own
    schedule cannot change a bit."""
    if r.world <= 1:
        return part
    import torch
    import torch.distributed as dist
    _, n = owned_mixes(r, part.shape[0])
    part = part.contiguous()
    out = torch.empty((n,) + tuple(part.shape[1:]), dtype=part.dtype, device=part.device)
    dist.reduce_scatter_tensor(out, part, op=dist.ReduceOp.SUM)
    return out


def partial_s16(mixer, x):
    """This rank's int32 partial of every mix: x [batch, tracks_here, frames, C]
    int16 (mixer.set_tracks holds those tracks' ramps) -> [batch, out_frames*C]."""
    import torch
    B, T, F, C = x.shape
    Fo = mixer.out_frames(F)
    x = x.contiguous()
    part = torch.empty((B, Fo * C), dtype=torch.int32, device=x.device)
    mixer.process_partial_strided(x.data_ptr(), F * C, T * F * C, part.data_ptr(), Fo * C, B, F)
    return part


def finish_block_s16(mixer, blk, channels, out=None):
    """Saturate a summed [n, out_frames*C] int32 block to [n, out_frames, C] int16."""
    import torch
    blk = blk.contiguous()
    n, S = blk.shape
    Fo = S // channels
    if out is None:
        out = torch.empty((n, Fo, channels), dtype=torch.int16, device=blk.device)
    mixer.finish_s16(blk.data_ptr(), 1, 0, S, out.data_ptr(), S, n, Fo)
    return out


def span_chunks(asked: int, owned: int) -> int:
    """The largest chunk count <= asked (0: 4) that divides the owned block
    (xm_audio_mixer_set_span_chunks' rule)."""
    k = min(asked if asked > 0 else 4, max(owned, 1))
    while k > 1 and owned % k:
        k -= 1
    return max(k, 1)


def mix_spanning_s16(r: Rank, mixer, x, out=None, chunks: int = 0):
    """Config 5 on this rank.  x: [batch, tracks_here, frames, C] int16 in HBM,
    this rank's tracks of every mix (mixer.set_tracks holds their ramps).
    Returns [batch/world, out_frames, C] int16: the finished mixes
    owned_mixes() gives this rank (partial -> reduce-scatter -> finish).

    The exchange runs in K chunks (span_chunks(chunks, batch/world)): chunk k
    is mixes q*n + k*cb .. + cb of every owner q (n = batch/world, cb = n/K);
    its partial is formed owner by owner into a [world*cb, S] buffer and its
    reduce-scatter is issued asynchronously, so it crosses the links while
    chunk k+1's partials compute (the in-library form does the same,
    src/xm_mixer_multi.c).  int32 sums are exact in any order: every K gives
    the same bits."""
    if r.world <= 1:
        return finish_block_s16(mixer, partial_s16(mixer, x), x.shape[3], out)
    import torch
    import torch.distributed as dist
    B, T, F, C = x.shape
    _, n = owned_mixes(r, B)
    K = span_chunks(chunks, n)
    cb = n // K
    S = mixer.out_frames(F) * C
    x = x.contiguous()
    blk = torch.empty((n, S), dtype=torch.int32, device=x.device)
    pending = []
    for k in range(K):
        buf = torch.empty((r.world * cb, S), dtype=torch.int32, device=x.device)
        for q in range(r.world):
            m0 = q * n + k * cb
            mixer.process_partial_strided(x[m0].data_ptr(), F * C, T * F * C, buf[q * cb].data_ptr(), S, cb, F)
        work = dist.reduce_scatter_tensor(blk[k * cb:(k + 1) * cb], buf, op=dist.ReduceOp.SUM, async_op=True)
        pending.append((work, buf))
    for work, _ in pending:
        work.wait()
    return finish_block_s16(mixer, blk, C, out)


def barrier(r: Rank) -> None:
    if r.world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(r: Rank, value: float, device="cpu") -> float:
    """The slowest rank's value (the job's wall time)."""
    if r.world <= 1:
        return float(value)
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def min_over_ranks(r: Rank, flag: bool, device="cpu") -> bool:
    """True only if `flag` holds on every rank (the job's parity bit)."""
    if r.world <= 1:
        return bool(flag)
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def finish(r: Rank) -> None:
    if r.world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
