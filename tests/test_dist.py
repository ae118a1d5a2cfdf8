"""CPU: the multi-GPU prompt-sharding path (hip_llama.cpp_amd/dist.py) on world_size-2 gloo.

Covers what bench.py / the N-GPU decode does besides the kernels: rank 0 owns the weights and
broadcasts them in chunks, prompts are sharded with no data-path collective, the slowest rank's
time is reported."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from __graft_entry__ import _pkg
    _pkg()
    from hip_llama_cpp_amd import dist as D
    # weights: only rank 0 has them; chunked broadcast (tiny chunks exercise the loop)
    n = 1000003
    arena = torch.arange(n, dtype=torch.float32) if rank == 0 else torch.zeros(n, dtype=torch.float32)
    D.broadcast_arena(arena, src=0, chunk_elems=65536)
    ok_bcast = bool(torch.equal(arena, torch.arange(n, dtype=torch.float32)))
    # prompts: contiguous shards, disjoint, covering
    a, b = D.shard(64, world, rank)
    slowest = D.max_over_ranks(1.0 + rank)
    total = D.sum_over_ranks(b - a)
    q.put((rank, ok_bcast, (a, b), slowest, total))
    dist.destroy_process_group()


def test_world2_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get() for _ in range(world))
    assert all(r[1] for r in res), "broadcast did not replicate the arena"
    shards = [r[2] for r in res]
    assert shards == [(0, 32), (32, 64)]
    assert all(r[3] == 2.0 for r in res)      # max over ranks
    assert all(r[4] == 64 for r in res)       # every prompt owned exactly once


@pytest.mark.parametrize("n,world", [(64, 8), (7, 3), (1, 4), (0, 2), (130, 8)])
def test_shard_partition(n, world):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from __graft_entry__ import _pkg
    _pkg()
    from hip_llama_cpp_amd import dist as D
    spans = [D.shard(n, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a0, b0), (a1, b1) in zip(spans, spans[1:]):
        assert b0 == a1
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1
