"""Rank plumbing for multi-GPU runs.

Mixes are independent, so N GPUs are N processes, each owning a contiguous
block of mixes (weak scaling: a fixed block per rank) with no collective in
the data path.  torch.distributed (RCCL = backend "nccl" on ROCm, or "gloo"
on CPU for tests) is used only for the start/stop barriers and the
max-over-ranks wall time.
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


def finish(r: Rank) -> None:
    if r.world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
