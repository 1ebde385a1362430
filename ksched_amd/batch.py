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


def union(graphs):
    """Disjoint union of cell graphs as ONE flow network (node ids offset per
    graph). The min-cost flow of a disjoint union is the union of the parts'
    optima, so one device solve fills the GPU with every cell at once instead
    of many small latency-bound solves. Returns (graph, node_offset[k+1],
    arc_offset[k+1]); graph i owns ids node_offset[i]+1 .. node_offset[i+1]."""
    from .gen import Graph

    noff = np.zeros(len(graphs) + 1, np.int64)
    aoff = np.zeros(len(graphs) + 1, np.int64)
    for i, g in enumerate(graphs):
        noff[i + 1] = noff[i] + g.n
        aoff[i + 1] = aoff[i] + g.m
    cat = lambda f: np.concatenate([f(g) for g in graphs]) if graphs else np.zeros(0, np.int64)
    src = cat(lambda g: g.src) + np.repeat(noff[:-1], [g.m for g in graphs])
    dst = cat(lambda g: g.dst) + np.repeat(noff[:-1], [g.m for g in graphs])
    u = Graph(cat(lambda g: g.ntype).astype(np.int32), cat(lambda g: g.supply), src, dst,
              cat(lambda g: g.low), cat(lambda g: g.cap), cat(lambda g: g.cost),
              cat(lambda g: g.arc_types()).astype(np.int32))
    return u, noff, aoff


def split_costs(u, noff, flows) -> np.ndarray:
    """Per-part total cost from the union's positive-flow records (ks_flow:
    src, dst, flow), Σ flow·cost over each part's arcs."""
    n = int(noff[-1]) + 1
    key = u.src.astype(np.int64) * n + u.dst.astype(np.int64)
    order = np.argsort(key, kind="stable")
    fk = flows["src"].astype(np.int64) * n + flows["dst"].astype(np.int64)
    idx = order[np.searchsorted(key, fk, sorter=order)]
    part = np.searchsorted(noff, flows["src"].astype(np.int64), side="left") - 1
    out = np.zeros(len(noff) - 1, np.int64)
    np.add.at(out, part, flows["flow"].astype(np.int64) * u.cost[idx])
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
