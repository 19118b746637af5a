"""Data parallel over RCCL/xGMI: one process per GPU, replicated
parameters, one gradient all-reduce per step inside the engine, exact global-mean CE.

The RCCL communicator lives in libcapgen (the count / CE all-reduces on the engine's critical
stream, the gradient buckets' reduce-scatter / all-gather on its bucket stream; at world > 1 the
forward is issued eagerly, so every collective is a plain stream call); torch.distributed is only
the bootstrap channel that carries rank 0's 128-byte unique id.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_rank_world():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def broadcast_unique_id(uid: bytes | None, rank: int) -> bytes:
    """Rank 0's RCCL unique id to every rank over the existing process group."""
    obj = [uid if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def init_engine_dp(engine, rank: int, world: int, unique_id=None):
    """Bootstrap the engine's communicator: rank 0 makes the RCCL unique id (`unique_id`, default
    Engine.dp_unique_id), the process group carries it to every rank, every rank calls dp_init."""
    if unique_id is None:
        from .engine import Engine
        unique_id = Engine.dp_unique_id
    uid = unique_id() if rank == 0 else None
    uid = broadcast_unique_id(uid, rank) if world > 1 else uid
    engine.dp_init(uid, rank, world)


def local_target_count(captions: torch.Tensor, pad_idx: int = 0) -> int:
    """Non-pad targets of this rank's batch: caption[:, 1:] != pad (model.py:89,76)."""
    return int((captions[:, 1:] != pad_idx).sum().item())


def global_target_count(captions: torch.Tensor, pad_idx: int = 0) -> int:
    """Sum of non-pad targets over all ranks: the denominator of the reference's
    CrossEntropyLoss(mean) over the global batch.  Averaging per-rank means would NOT
    match single-process training at the global batch."""
    n = torch.tensor([local_target_count(captions, pad_idx)], dtype=torch.float64)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(n)
    return int(n.item())


def shard_seed(base: int, rank: int) -> int:
    """Per-rank synthetic-data seed (1000 + rank)."""
    return base + rank
