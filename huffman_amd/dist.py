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
symbol straddles two ranks; the last shard takes the rest, and when the
stream is odd its final raw byte is broadcast to rank 0 for the header
(odd_last_byte). Decode needs no collective: each rank decodes
its own symbols from its own payload (its index holds absolute local bits).
Over RCCL ("nccl" backend on ROCm) the exchanges ride xGMI; the tests use gloo.
"""
import numpy as np
import torch
import torch.distributed as dist


def _global(group, r):
    """Global rank of rank `r` of `group`: torch.distributed's src/dst/peer
    arguments are global ranks even when a group is passed."""
    return r if group is None else dist.get_global_rank(group, r)


def shard_range(n_total, world, rank):
    """Byte range of rank `rank`: equal, even-sized shards (the last takes the rest)."""
    per = (n_total // world) & ~1
    beg = per * rank
    end = n_total if rank == world - 1 else beg + per
    return beg, end


def odd_last_byte(shard, n_total, group=None):
    """The raw trailing byte of an odd-length stream, on every rank.

    With n_total odd the last rank's shard ends in the byte that is not coded
    (Compressor.cu:339-351); rank 0 writes it into the header
    (Compressor.cu:438-443), so it is broadcast from the last rank. 0 when
    n_total is even. `shard`: this rank's bytes (numpy array or tensor)."""
    if n_total % 2 == 0:
        return 0
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = shard.device if isinstance(shard, torch.Tensor) else torch.device("cpu")
    if dist.get_backend(group) == "nccl" and dev.type != "cuda":
        dev = torch.device("cuda", torch.cuda.current_device())
    v = torch.zeros(1, dtype=torch.int64, device=dev)
    if rank == world - 1:
        assert len(shard) % 2 == 1, "the last shard of an odd stream holds the odd byte"
        v[0] = int(shard[-1])
    dist.broadcast(v, src=_global(group, world - 1), group=group)
    return int(v.item())


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
    dist.gather(pad, bufs, dst=_global(group, dst), group=group)
    if bufs is None:
        return None
    return [b[:int(s)].cpu().numpy() for b, s in zip(bufs, sizes)]


_P2P_CHUNK = 1 << 30  # bytes per point-to-point message


def _chunks(a, b):
    """[a, b) in messages of at most _P2P_CHUNK bytes (the same split on both sides)."""
    while a < b:
        e = min(b, a + _P2P_CHUNK)
        yield a, e
        a = e


def reassemble_on_device(payload, local_bytes, word0, dst=0, group=None, via_host=False):
    """gather every shard's word-aligned payload buffer
    into ONE payload stream on rank `dst`, on the device.

    payload: uint8 CUDA tensor of this shard (word 0 = global payload word `word0`);
    local_bytes: its bytes that hold bits. Shard bodies (bytes [4, n)) land in
    place by point-to-point receives (RCCL over xGMI, all posted at once); the
    shards' first words, which share bits with the previous shard's last word,
    are ORed in afterwards. via_host: the same exchange through host copies
    (gloo; bench.py --rehearse on one GPU). Returns the stream tensor on dst
    (None elsewhere) and the stream's byte count."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = payload.device
    mine = torch.tensor([local_bytes, word0], dtype=torch.int64)
    if via_host:
        parts = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(parts, mine, group=group)
        meta = torch.stack(parts)
    else:
        meta = torch.zeros(world, 2, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(meta.view(-1), mine.to(dev), group=group)
        meta = meta.cpu()
    nb = [int(v) for v in meta[:, 0]]
    w0 = [int(v) for v in meta[:, 1]]
    total = max(4 * w + n for w, n in zip(w0, nb))
    head_n = [min(4, n) for n in nb]
    gdst = _global(group, dst)
    if rank != dst:
        if via_host:  # the same messages as the RCCL path, through host copies
            for a, b in _chunks(4, nb[rank]):
                dist.send(payload[a:b].cpu(), gdst, group=group)
            dist.send(payload[:4].cpu(), gdst, group=group)
        else:
            ops = [dist.P2POp(dist.isend, payload[:4], gdst, group=group)]
            for a, b in _chunks(4, nb[rank]):
                ops.append(dist.P2POp(dist.isend, payload[a:b], gdst, group=group))
            for r in dist.batch_isend_irecv(ops):
                r.wait()
        return None, total
    out = torch.zeros((total + 3) // 4 * 4, dtype=torch.uint8, device=dev)
    heads = torch.zeros(world, 4, dtype=torch.uint8, device=dev)
    ops = []
    for r in range(world):
        body = out[4 * w0[r] + 4:4 * w0[r] + nb[r]] if nb[r] > 4 else None
        if r == dst:
            heads[r] = payload[:4]
            if body is not None:
                body.copy_(payload[4:nb[r]])
        elif via_host:
            for a, b in _chunks(4, nb[r]):
                tmp = torch.empty(b - a, dtype=torch.uint8)
                dist.recv(tmp, _global(group, r), group=group)
                out[4 * w0[r] + a:4 * w0[r] + b].copy_(tmp)
            tmp = torch.empty(4, dtype=torch.uint8)
            dist.recv(tmp, _global(group, r), group=group)
            heads[r] = tmp
        else:
            ops.append(dist.P2POp(dist.irecv, heads[r], _global(group, r), group=group))
            for a, b in _chunks(4, nb[r]):
                ops.append(dist.P2POp(dist.irecv, out[4 * w0[r] + a:4 * w0[r] + b], _global(group, r), group=group))
    if ops:
        for q in dist.batch_isend_irecv(ops):
            q.wait()
    for r in range(world):  # after every body: heads OR into the previous shard's last word
        if head_n[r]:
            seg = out[4 * w0[r]:4 * w0[r] + head_n[r]]
            seg.bitwise_or_(heads[r, :head_n[r]])
    return out, total


# ---- one index-less stream decoded by every rank ----------------------------------
# A reference `.compressed` payload carries no index (Compressor.cu:427-601) and the reference decodes
# it serially (Decompressor.cu:259-291). Split over ranks, every rank decodes one PART of the payload
# bits, found by self-synchronisation: rank r walks its part from 1024 bits before it (its walked
# entry is the first codeword start on that path at or after the part's first bit), counts its
# codewords and finds its exit (the first codeword start at or after its end). The true entry of
# rank r is rank r - 1's true exit: one all-gather of (codewords, exit, entry used) per round; a rank
# whose entry disagrees walks again from the true one (its exit may move, so rounds repeat: at most
# world - 1, typically none). Rank r's first output symbol is the sum of the codewords before it.

UNKNOWN_ENTRY = (1 << 64) - 1


def part_range(payload_bits, world, rank, align=128):
    """Payload bits [begin, end) (after the stream's first bit) of rank `rank`'s part: equal parts,
    boundaries on `align` bits, the last non-empty part takes the rest. A payload shorter than `world`
    aligned parts has fewer parts: the ranks past them get the empty part [payload_bits, payload_bits)."""
    parts = max(1, min(world, payload_bits // align))
    if rank >= parts:
        return payload_bits, payload_bits
    per = (payload_bits // parts) // align * align
    beg = per * rank
    end = payload_bits if rank == parts - 1 else beg + per
    return beg, end


def decode_indexless_split(scan, refix, decode, nsym, device, group=None, empty=False):
    """The exchange of a split index-less decode. Per-rank engines (every bit a stream bit, the same
    coordinates on every rank):
      scan() -> (codewords, exit, walked entry) of this rank's part (rank 0: from the stream's start)
      refix(entry) -> (codewords, exit, entry) of the part walked from a given true entry
      decode(first, nsym_from_first) -> decodes the part's codewords (at most nsym_from_first)
    On the GPU these are hz_indexless_scan / hz_indexless_refix / hz_indexless_decode (bench.py,
    tests/test_gpu_dist.py); tests/test_dist.py drives the same exchange with the CPU oracle's walk.
    empty: this rank's part is empty (part_range past the parts of a short payload): no engine is
    called, the rank passes the previous part's exit on and still joins every all-gather.
    Returns (first symbol of this rank, its codewords, rounds of refixes)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    count, exit_, entry = (0, UNKNOWN_ENTRY, UNKNOWN_ENTRY) if empty else scan()
    rounds = 0
    while True:
        mine = torch.tensor([count, exit_ & ((1 << 63) - 1), exit_ >> 63, entry & ((1 << 63) - 1), entry >> 63,
                             1 if empty else 0], dtype=torch.int64, device=device)
        allv = torch.zeros(world * 6, dtype=torch.int64, device=device)
        dist.all_gather_into_tensor(allv, mine, group=group)
        v = allv.view(world, 6).cpu().tolist()
        counts = [int(x[0]) for x in v]
        exits = [int(x[1]) | (int(x[2]) << 63) for x in v]
        entries = [int(x[3]) | (int(x[4]) << 63) for x in v]
        void = [bool(x[5]) for x in v]
        for r in range(1, world):  # an empty part's entry and exit are the previous part's exit
            if void[r]:
                entries[r] = exits[r] = exits[r - 1]
        stale = [r for r in range(1, world) if not void[r] and entries[r] != exits[r - 1]]
        if not stale:
            break
        if rounds >= world:  # a change moves one part per round: cannot happen
            raise RuntimeError("decode_indexless_split: exits did not settle")
        rounds += 1
        if rank in stale:
            count, exit_, entry = refix(exits[rank - 1])
    first = sum(counts[:rank])
    take = max(0, min(count, nsym - first))
    if not empty:
        decode(first, take)
    return first, count, rounds


def part_window(start_bit, part_begin, part_end, max_len, lead=1024):
    """Global payload words [lo, hi) a rank's part reads: the part (payload bits after start_bit), the
    lead-in before it (HZ_INDEXLESS_LEAD_BITS, or the stream from its start) and max_len bits after it."""
    b0 = start_bit + part_begin - min(lead, part_begin)
    b1 = start_bit + part_end + max_len
    return b0 // 32, (b1 + 31) // 32


def fill_window(ext, ext_word0, own_word0, own_words, windows, shards, group=None, via_host=False):
    """Bring the words of this rank's part window that other ranks' shards hold into `ext`.

    ext: this rank's uint8 device buffer holding global payload words [ext_word0, ext_word0 + len/4), its
    own shard packed in place at words [own_word0, own_word0 + own_words) (zeros around it);
    windows[r] = (lo, hi): the global words rank r's part reads; shards[r] = (word0, words): rank r's
    shard. For every pair of ranks, the words of one's shard inside the other's window travel
    point-to-point (RCCL over xGMI; gloo through host copies when via_host) and are ORed in (adjacent
    shards share a boundary word). Every rank knows every window and shard, so the sends and receives
    match without a handshake. The window must lie inside ext (the caller sizes ext's halo)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = windows[rank]
    assert ext_word0 <= lo and hi <= ext_word0 + ext.numel() // 4, "part window outside the buffer"

    def inter(win, shard):
        a = max(win[0], shard[0])
        b = min(win[1], shard[0] + shard[1])
        return (a, b) if a < b else None

    sends, recvs = [], []
    for g in range(world):
        if g == rank:
            continue
        s = inter(windows[g], (own_word0, own_words))
        if s:
            sends.append((g, ext[4 * (s[0] - ext_word0):4 * (s[1] - ext_word0)]))
        r = inter((lo, hi), shards[g])
        if r:
            recvs.append((g, r, torch.empty(4 * (r[1] - r[0]), dtype=torch.uint8,
                                            device="cpu" if via_host else ext.device)))
    if via_host:
        # blocking, in a global order every rank follows: (src, dst) pairs by (min, max) rank
        pairs = sorted({(min(rank, g), max(rank, g)) for g, _ in sends} | {(min(rank, g), max(rank, g)) for g, _, _ in recvs})
        sd = {g: t for g, t in sends}
        rv = {g: t for g, _, t in recvs}
        for a, b in pairs:
            g = b if a == rank else a
            first = a == rank  # the lower rank sends first
            for phase in (0, 1):
                if (phase == 0) == first:
                    if g in sd:
                        dist.send(sd[g].cpu().contiguous(), _global(group, g), group=group)
                elif g in rv:
                    dist.recv(rv[g], _global(group, g), group=group)
    else:
        ops = [dist.P2POp(dist.isend, t, _global(group, g), group=group) for g, t in sends]
        ops += [dist.P2POp(dist.irecv, t, _global(group, g), group=group) for g, _, t in recvs]
        if ops:
            for q in dist.batch_isend_irecv(ops):
                q.wait()
    for g, (a, b), t in recvs:
        ext[4 * (a - ext_word0):4 * (b - ext_word0)].bitwise_or_(t.to(ext.device))
