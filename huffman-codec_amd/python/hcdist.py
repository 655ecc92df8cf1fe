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
    """Global stream indices owned by `rank`: the contiguous range [rank * per_rank, (rank + 1) * per_rank).
    bench.py fixes per_rank (one C5 batch per GPU: weak scaling) by default, and with
    --total-streams splits a fixed total over the ranks (strong scaling: per_rank = total / world)."""
    return range(rank * per_rank, (rank + 1) * per_rank)


def reduce_counters(values, op="sum", device=None):
    t = torch.as_tensor(values, dtype=torch.float64 if op == "max" else torch.int64, device=device)
    if dist.is_initialized():  # world 1 too: the collective runs (RCCL on a one-GPU box)
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return t


def gather_sizes(lens):
    """All-gather the per-stream encoded sizes: returns a (world * S,) tensor on every rank."""
    if not dist.is_initialized():
        return lens.clone()
    parts = [torch.empty_like(lens) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, lens)
    return torch.cat(parts)


def pack(buf, offs, lens):
    """Concatenate the byte ranges buf[offs[i]:offs[i]+lens[i]]. On the GPU this is the
    hc_pack_batch kernel (no index tensors: 16-byte copies straight into the packed buffer);
    CPU tensors (the gloo tests) are sliced on the host."""
    total = int(lens.sum())
    out = torch.empty(total, dtype=torch.uint8, device=buf.device)
    if total == 0:
        return out
    dst = torch.cumsum(lens, 0) - lens
    if buf.is_cuda:
        import hcodec
        hcodec.pack_batch(buf, offs.contiguous(), lens.contiguous(), out, dst.contiguous())
    else:
        for o, n, d in zip(offs.tolist(), lens.tolist(), dst.tolist()):
            out[d:d + n] = buf[o:o + n]
    return out


def gather_encoded(buf, offs, lens):
    """Encoded streams of every rank, packed back to back in global stream order, on rank 0
    (None elsewhere), with the all-gathered sizes. Each rank packs its shard on the device,
    then sends it straight to rank 0 (one point-to-point transfer per rank, all posted at once
    by batch_isend_irecv: over xGMI every rank's shard travels on its own link to GPU 0; no
    rank receives any payload but rank 0, and nothing is padded)."""
    packed = pack(buf, offs, lens)
    sizes = gather_sizes(lens)
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return packed, sizes
    world, rank = dist.get_world_size(), dist.get_rank()
    per_rank = sizes.view(world, -1).sum(1).tolist()
    if rank != 0:
        if per_rank[rank]:
            for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, packed, 0)]):
                w.wait()
        return None, sizes
    out = torch.empty(sum(per_rank), dtype=torch.uint8, device=buf.device)
    out[:per_rank[0]] = packed
    ops, at = [], per_rank[0]
    for r in range(1, world):
        if per_rank[r]:
            ops.append(dist.P2POp(dist.irecv, out[at:at + per_rank[r]], r))
        at += per_rank[r]
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return out, sizes
