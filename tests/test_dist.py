"""Multi-rank path on CPU: world_size-2 gloo process group exchanging the
Lynch-path profile histograms (the only collective of the path), and the
site-range sharding used by build/sid and bench.py."""
import os
import socket

import numpy as np
import pytest


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def host_table(counts):
    # test-side reference histogram (numpy), not a product path
    import sid_amd
    keys = sid_amd.profile_key(counts)
    u, c = np.unique(keys, return_counts=True)
    return u.astype(np.uint64), c.astype(np.uint64)


def _worker(rank, world, port, n, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist

    import sid_amd
    from sid_amd.dist import allgather_profile_table, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(n, rank, world)
    counts = sid_amd.synth_counts_host(3, hi - lo, 30.0, first=lo)
    k, c = host_table(counts)
    mk, mc = allgather_profile_table(k, c)
    q.put((rank, lo, hi, mk.tolist(), mc.tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_profile_allgather(sid, world):
    import torch.multiprocessing as mp
    n = 30011
    port = free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    # shards are disjoint and cover [0, n)
    assert [r[1] for r in res] == [0, n // 2] and res[-1][2] == n
    k, c = host_table(sid.synth_counts_host(3, n, 30.0))
    for r in res:
        assert r[3] == k.tolist() and r[4] == c.tolist()


def test_merge_tables_sums_counts():
    from sid_amd.dist import merge_profile_tables
    a = (np.array([5, 1, 9], np.uint64), np.array([1, 2, 3], np.uint64))
    b = (np.array([9, 2], np.uint64), np.array([10, 20], np.uint64))
    k, c = merge_profile_tables([a, b])
    assert k.tolist() == [1, 2, 5, 9] and c.tolist() == [2, 20, 1, 13]


def test_shard_range_cover():
    from sid_amd.dist import shard_range
    for n in (0, 1, 7, 50_000_000):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
