"""Config 5: independent cell graphs sharded over GPUs, mappings gathered over RCCL.

A single solve does not shard, so multi-GPU throughput comes
from independent graphs — cluster cells or what-if variants of one cell. Each
rank owns the graphs ``g ≡ rank (mod world)`` (round-robin, SURVEY §8d config
5), solves them concurrently on its own GPU (``native.solve_many``: one context
and stream per graph, native worker threads), and only after the solves does a
single collective move data: every rank's task→PU buffer, a fixed
``[slots, tasks]`` int64 block (PU node id per task, 0 = unscheduled or
padding), is all-gathered, then reordered by graph id. ``dist`` may be a
``torch.distributed`` group on RCCL (``nccl``, GPU tensors) or ``gloo`` (CPU
tensors, used by the CPU tests).
"""
from __future__ import annotations

import math

import numpy as np


def assign(num_graphs: int, world: int, rank: int) -> list[int]:
    """Graph ids owned by ``rank``: g ≡ rank (mod world)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    return list(range(rank, num_graphs, world))


def slots_per_rank(num_graphs: int, world: int) -> int:
    return max(1, math.ceil(num_graphs / world))


def owner(g: int, world: int) -> tuple[int, int]:
    """(rank, local slot) holding graph g in the gathered buffer."""
    return g % world, g // world


def pack(maps: list[np.ndarray], slots: int, tasks: int) -> np.ndarray:
    """Stack per-graph task→PU vectors (length ≤ tasks) into a zero-padded
    [slots, tasks] int64 block (host side; the GPU path fills the block on
    device through ``ks_get_task_pu_device``)."""
    out = np.zeros((slots, tasks), np.int64)
    for i, m in enumerate(maps):
        m = np.asarray(m, np.int64)
        out[i, :m.shape[0]] = m
    return out


def gather(block, num_graphs: int, dist, group=None):
    """All-gather the per-rank ``[slots, tasks]`` blocks (a torch tensor on the
    collective's device) and return ``[num_graphs, tasks]`` ordered by graph id."""
    import torch

    world = dist.get_world_size(group)
    parts = [torch.empty_like(block) for _ in range(world)]
    dist.all_gather(parts, block.contiguous(), group=group)
    full = torch.stack(parts, 0)                              # [world, slots, tasks]
    idx = torch.arange(num_graphs, device=block.device)
    return full[idx % world, idx // world]
