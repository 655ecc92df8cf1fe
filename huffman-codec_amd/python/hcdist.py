"""Multi-GPU plumbing for batched streams: one process per GPU, torch.distributed over RCCL
(backend "nccl" on ROCm) or gloo (CPU tests).

Streams are independent (no state is shared between HuffTree instances, transform.cpp:366),
so the data path has no collective: rank r owns streams [r*S, (r+1)*S) and generates, encodes
and decodes them locally. Collectives appear only after the data path:
  * reduce_counters  all-reduce of verification counters (and MAX of step time)
  * gather_sizes     all-gather of every stream's encoded length
  * gather_encoded   the encoded payloads of all ranks into rank 0 (packed back to back)
"""
import torch
import torch.distributed as dist


def shard(rank, world, per_rank):
    """Global stream indices owned by `rank` (weak scaling: per_rank streams each)."""
    return range(rank * per_rank, (rank + 1) * per_rank)


def reduce_counters(values, op="sum", device=None):
    t = torch.as_tensor(values, dtype=torch.float64 if op == "max" else torch.int64, device=device)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return t


def gather_sizes(lens):
    """All-gather the per-stream encoded sizes: returns a (world * S,) tensor on every rank."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return lens.clone()
    parts = [torch.empty_like(lens) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, lens)
    return torch.cat(parts)


def pack(buf, offs, lens):
    """Concatenate the byte ranges buf[offs[i]:offs[i]+lens[i]] (device gather, no host copy)."""
    idx = torch.repeat_interleave(offs, lens) + (
        torch.arange(int(lens.sum()), device=buf.device) -
        torch.repeat_interleave(torch.cumsum(lens, 0) - lens, lens))
    return buf[idx]


def gather_encoded(buf, offs, lens):
    """Encoded streams of every rank, packed back to back in global stream order, on rank 0
    (None elsewhere), with the all-gathered sizes. One all-gather of sizes, then one padded
    all-gather of the packed payloads (RCCL ring over xGMI)."""
    packed = pack(buf, offs, lens)
    sizes = gather_sizes(lens)
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return packed, sizes
    world = dist.get_world_size()
    per_rank = sizes.view(world, -1).sum(1)
    cap = int(per_rank.max())
    pad = torch.zeros(cap, dtype=torch.uint8, device=buf.device)
    pad[: packed.numel()] = packed
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    if dist.get_rank() != 0:
        return None, sizes
    return torch.cat([p[: int(n)] for p, n in zip(parts, per_rank)]), sizes
