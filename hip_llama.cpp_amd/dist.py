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
