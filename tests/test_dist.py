"""CPU: the multi-GPU prompt-sharding path (hip_llama.cpp_amd/dist.py) on world_size-2 gloo.

Covers what bench.py / the N-GPU decode does besides the kernels: rank 0 owns the weights and
broadcasts them in chunks, prompts are sharded with no data-path collective, the slowest rank's
time is reported."""
import os
import socket

import numpy as np
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


V = 32000
TOK = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tokenizer.bin")
PROMPTS = ["Once upon a time", "The serene landscape", "", "A brief message:", "x" * 40, "Why?",
           "Lily and Ben", "In a small town", "The cat sat"]


def _fake_logits(token, pos):
    r = np.random.default_rng(int(token) * 100003 + int(pos))
    lg = (r.standard_normal(V) * 2.5).astype(np.float32)
    lg[2] = np.float32(-4.0 + 0.25 * pos)  # EOS likelier with position: varied lengths
    return lg


def _fake_step(worker, toks, pos):
    return np.stack([_fake_logits(t, p) for t, p in zip(toks, pos)])


def _serve_worker(rank, world, port, src, out, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from __graft_entry__ import _pkg
    _pkg()
    from hip_llama_cpp_amd import dist as D
    gen = D.serve_sharded(src, out, TOK, V, 2, _fake_step, 27, 48, workdir=os.path.dirname(out))
    q.put((rank, gen))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_serve_sharded_equals_single_process(tmp_path, world):
    """dist.serve_sharded: the test-mode request file (src/llama.cpp:891-1083) served by `world`
    gloo ranks, each scheduling its prompt shard through the host scheduler with a CPU step
    callback; rank 0's gathered output file is byte-identical to the single-process run and the
    generated-token count is the same."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from __graft_entry__ import _pkg
    _pkg()
    from hip_llama_cpp_amd import host as H
    src = tmp_path / "in.txt"
    src.write_bytes((f"{len(PROMPTS)}\n" + "\n".join(PROMPTS) + "\n").encode())
    r = H.Requests(str(src), 27, 48)
    want_gen = r.serve(TOK, V, 1, 2, _fake_step)
    ref = tmp_path / "ref.txt"
    r.write(str(ref))
    out = tmp_path / "out.txt"
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_serve_worker, args=(k, world, port, str(src), str(out), q)) for k in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    res = sorted(q.get() for _ in range(world))
    assert all(g == want_gen for _, g in res)
    assert out.read_bytes() == ref.read_bytes()
