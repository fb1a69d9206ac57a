"""Multi-rank plumbing.

-m local shards with no exchange at all: rank r owns a contiguous site range.
The Lynch path (-R, likelihood_ratio, bayes) has exactly one exchange: the
per-rank unique-profile histograms are all-gathered and merged, every rank
then runs the same deterministic estimate and looks up its own sites.  The
payload is O(U) (~10^4 profiles x 16 B at 30x), i.e. latency-bound, so one
all_gather of the packed table is the whole protocol.  With the "nccl"
backend (RCCL on ROCm) the tables travel over xGMI; with "gloo" over the
host (CPU tests).
"""
from __future__ import annotations

import numpy as np


def shard_range(n_total: int, rank: int, world: int):
    """Contiguous, line-aligned site range of `rank` (same split as build/sid)."""
    return n_total * rank // world, n_total * (rank + 1) // world


def merge_profile_tables(tables):
    """Sum counts of equal keys; keys sorted (lexicographic profile_t order)."""
    keys = np.concatenate([np.asarray(k, np.uint64) for k, _ in tables]) if tables else np.zeros(0, np.uint64)
    cnts = np.concatenate([np.asarray(c, np.uint64) for _, c in tables]) if tables else np.zeros(0, np.uint64)
    if len(keys) == 0:
        return keys, cnts
    order = np.argsort(keys, kind="stable")
    keys, cnts = keys[order], cnts[order]
    first = np.ones(len(keys), bool)
    first[1:] = keys[1:] != keys[:-1]
    idx = np.flatnonzero(first)
    return keys[idx], np.add.reduceat(cnts, idx).astype(np.uint64)


def allgather_profile_table(keys: np.ndarray, cnts: np.ndarray, device=None):
    """All-gather every rank's (keys, counts) and return the merged table."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    dev = device if device is not None else torch.device("cpu")
    n = torch.tensor([len(keys)], dtype=torch.int64, device=dev)
    ns = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(ns, n)
    ns = [int(x.item()) for x in ns]
    m = max(ns) if ns else 0
    packed = np.zeros((max(m, 1), 2), np.uint64)
    packed[: len(keys), 0] = keys
    packed[: len(keys), 1] = cnts
    t = torch.from_numpy(packed.view(np.int64)).to(dev)
    outs = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    tables = []
    for r, o in enumerate(outs):
        a = o.cpu().numpy().view(np.uint64)[: ns[r]]
        tables.append((a[:, 0], a[:, 1]))
    return merge_profile_tables(tables)
