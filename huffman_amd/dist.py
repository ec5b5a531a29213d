"""Multi-GPU sharding of the hot path (one process per GPU, torch.distributed).

SURVEY.md 8(e): for the output to stay the ONE stream the 1-GPU encoder
writes, every rank must use the global codebook, so the path has exactly two
small exchange steps, plus an optional reassembly:

  1. all-reduce of the 65 536 x u64 histogram (512 KiB)        -> global codebook
  2. all-gather of each rank's payload bit count (8 B per rank) -> global bit offset
  3. (optional) payload reassembly at a writer rank: shards are packed at their
     global bit offsets into word-aligned local buffers; adjacent shards share
     at most one 32-bit boundary word, merged with OR.

Shard g holds the bytes [g*S, (g+1)*S) of the input with S even, so no
symbol straddles two ranks. Decode needs no collective: each rank decodes
its own symbols from its own payload (its index holds absolute local bits).
Over RCCL ("nccl" backend on ROCm) the exchanges ride xGMI; the tests use gloo.
"""
import numpy as np
import torch
import torch.distributed as dist


def shard_range(n_total, world, rank):
    """Byte range of rank `rank`: equal, even-sized shards (the last takes the rest)."""
    per = (n_total // world) & ~1
    beg = per * rank
    end = n_total if rank == world - 1 else beg + per
    return beg, end


def global_histogram(hist_local, group=None):
    """hist_local: int64 tensor [65536] on this rank's device. Returns a new
    tensor with the all-reduced (global) histogram."""
    h = hist_local.clone()
    dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
    return h


def shard_bit_offsets(payload_bits_local, device, group=None):
    """All-gather of per-rank payload bits -> (exclusive prefix for this rank, all totals)."""
    world = dist.get_world_size(group)
    mine = torch.tensor([payload_bits_local], dtype=torch.int64, device=device)
    allv = torch.zeros(world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(allv, mine, group=group)
    totals = [int(v) for v in allv.cpu()]
    rank = dist.get_rank(group)
    return sum(totals[:rank]), totals


def local_geometry(header_bits, shard_bit_offset, payload_bits_local, first_shard):
    """Where a shard's bits live. Returns (global_word0, start_bit, words): the
    local buffer's word 0 is global payload word `global_word0`; the shard's
    first bit is local bit `start_bit`."""
    stream_bit = header_bits % 8 + shard_bit_offset
    start = stream_bit if first_shard else stream_bit % 32
    word0 = 0 if first_shard else stream_bit // 32
    words = (start + payload_bits_local + 31) // 32
    return word0, start, words


def reassemble(shards, word0s, total_payload_bits, header_bits):
    """OR-merge word-aligned shard buffers (uint8 numpy arrays, big-endian bit
    order inside bytes) into the payload byte stream of the whole file."""
    nbytes = (header_bits % 8 + total_payload_bits + 7) // 8
    words = (nbytes + 3) // 4 + 1
    out = np.zeros(words * 4, dtype=np.uint8)
    for buf, w0 in zip(shards, word0s):
        b = np.asarray(buf, dtype=np.uint8)
        lo = 4 * w0
        hi = min(lo + b.size, out.size)
        out[lo:hi] |= b[:hi - lo]
    return out[:nbytes]


def gather_to(payload, nbytes_local, dst=0, group=None):
    """Gather every rank's first `nbytes_local` payload bytes to rank `dst`
    (padded to the largest shard). Returns the list of numpy buffers on dst,
    None elsewhere."""
    world = dist.get_world_size(group)
    dev = payload.device
    sizes = torch.zeros(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(sizes, torch.tensor([nbytes_local], dtype=torch.int64, device=dev), group=group)
    mx = int(sizes.max())
    pad = torch.zeros(mx, dtype=torch.uint8, device=dev)
    pad[:nbytes_local] = payload[:nbytes_local]
    bufs = [torch.zeros(mx, dtype=torch.uint8, device=dev) for _ in range(world)] if dist.get_rank(group) == dst \
        else None
    dist.gather(pad, bufs, dst=dst, group=group)
    if bufs is None:
        return None
    return [b[:int(s)].cpu().numpy() for b, s in zip(bufs, sizes)]
