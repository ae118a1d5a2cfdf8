"""Prompt sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

The reference runs one OpenMP thread per GPU, each with a full weight replica and a shared
request counter (src/llama.cpp:891-1083, "data parallelism"); every GPU uploads the whole
model from host memory (src/models.cpp:86-125).  Here:

* prompts are independent, so they are dealt to ranks without any data-path collective
  (weak scaling): :func:`shard` gives rank r a contiguous slice, sizes differing by <= 1;
* the weights are produced once (loaded / synthesised on rank 0) and replicated with
  RCCL broadcasts over xGMI in large chunks (:func:`broadcast_arena`);
* the only other collective is the timing reduction (:func:`max_over_ranks`).
"""
import torch
import torch.distributed as dist


def shard(n_items, world, rank):
    """Contiguous [start, stop) of n_items for rank (the first n_items % world ranks get one more)."""
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def broadcast_arena(t, src=0, chunk_elems=1 << 28):
    """Broadcast a flat tensor from src in chunks (1 GiB of fp32 per collective by default:
    large enough to run at link rate, small enough for RCCL's int32 element counts)."""
    n = t.numel()
    for s in range(0, n, chunk_elems):
        dist.broadcast(t[s:s + chunk_elems], src=src)


def max_over_ranks(value, device=None):
    """Max of a Python float over all ranks (the bench reports the slowest rank's time)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, device=None):
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def serve_sharded(requests_path, out_path, tokenizer_path, vocab_size, batch, step, max_token_len, max_seq_len,
                  temperature=None, topp=0.9, prefill=None, workdir=".", native=None, outputs=None):
    """The reference's test mode (test_data_parallelism, src/llama.cpp:891-1083) with one process
    per GPU instead of one thread per GPU: every rank parses the request file
    (read_inputfile, src/llama.cpp:424-453), serves the contiguous shard :func:`shard` gives it
    through the host scheduler (``host.Requests.serve``: ``batch`` slots refilled from the shard,
    one sampler per request) with its own ``step`` / ``prefill`` callbacks, and rank 0 gathers
    the generated strings in request order and writes the output file (write_outputfile,
    src/llama.cpp:455-505).  Every request is sampled independently (seed 314028 each), so the
    file equals the single-process one byte for byte.  Returns the reference's num_gen_tokens
    summed over ranks.  The only collectives are the object gather and that sum.
    ``native`` = (step address, prefill address or 0, ctx) drives the scheduler with native
    callbacks instead of ``step`` / ``prefill`` (host.Requests.serve_native).  On rank 0 the
    gathered responses (bytes, request order) are appended to ``outputs`` when it is a list."""
    import os

    from . import host as H
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    full = H.Requests(requests_path, max_token_len, max_seq_len)
    n = len(full)
    a, b = shard(n, world, rank)
    mine = [full.prompt(i) for i in range(a, b)]
    del full
    outs, gen = [], 0
    if mine:
        part = os.path.join(workdir, f".shard_{os.getpid()}_{rank}.txt")
        with open(part, "wb") as f:
            f.write(f"{len(mine)}\n".encode() + b"".join(p + b"\n" for p in mine))
        try:
            r = H.Requests(part, max_token_len, max_seq_len)
        finally:
            os.remove(part)
        if temperature is not None:
            r.set_sampling(temperature, topp)
        if native is not None:
            gen = r.serve_native(tokenizer_path, vocab_size, 1, batch, *native)
        else:
            gen = r.serve(tokenizer_path, vocab_size, 1, batch, step, prefill)
        outs = [r.output(i) for i in range(len(mine))]
    if world > 1:
        parts = [None] * world
        dist.all_gather_object(parts, outs)
        outs = [o for p in parts for o in p]
        gen = int(sum_over_ranks(gen))
    if rank == 0:
        with open(out_path, "wb") as f:
            f.write(f"{n}\n".encode() + b"".join(o + b"\n" for o in outs))
        if outputs is not None:
            outputs.extend(outs)
    return gen
