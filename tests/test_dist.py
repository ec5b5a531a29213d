"""Multi-process (gloo, CPU) test of the sharded path's exchange logic
(huffman_amd/dist.py): histogram all-reduce -> global codebook -> all-gather
of payload bits -> per-shard packing at global bit offsets -> gather + OR
reassembly. The reassembled file must equal the single-stream encoder's output
byte for byte. The per-shard packer here is the oracle's (this runs without a
GPU); on the GPU the same geometry feeds hz_pack (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, kind, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import huffman_amd
        from huffman_amd import dist as hd
        data = oracle_lib.generate(n_total, offset=0, kind=kind, seed=11)
        beg, end = hd.shard_range(n_total, world, rank)
        shard = data[beg:end]
        assert beg % 2 == 0
        hist_local = torch.from_numpy(oracle_lib.hist16(shard).astype(np.int64))
        h = hd.global_histogram(hist_local).numpy().astype(np.uint64)
        cb = huffman_amd.build_codebook(h)
        hb = huffman_amd.header_bits(cb, n_total)
        pbits = huffman_amd.payload_bits(cb, hist_local.numpy().astype(np.uint64))
        off, totals = hd.shard_bit_offsets(pbits, torch.device("cpu"))
        word0, start, words = hd.local_geometry(hb, off, pbits, rank == 0)
        _, ln, code = huffman_amd.codebook_arrays(cb)
        buf = oracle_lib.pack_range(shard, 0, shard.size // 2, ln, code, start, words * 4 + 8)
        # the odd trailing byte travels from the last rank (its shard) to rank 0's header
        last = hd.odd_last_byte(shard, n_total)
        if rank == 0:
            header, pend_bits, pend = huffman_amd.write_header(cb, n_total, last)
            buf[0] |= pend
        nbytes = (start + pbits + 7) // 8
        # the device-side reassembly's exchange (bench.py N > 1), through host copies here
        stream, total = hd.reassemble_on_device(torch.from_numpy(buf.copy()), nbytes, word0, dst=0, via_host=True)
        # the RCCL code path (batched isend/irecv into views of the stream), here over gloo on CPU tensors
        hd._P2P_CHUNK = 4096  # several messages per shard
        stream2, total2 = hd.reassemble_on_device(torch.from_numpy(buf.copy()), nbytes, word0, dst=0)
        if rank == 0:
            assert total2 == total and torch.equal(stream2, stream)
        shards = hd.gather_to(torch.from_numpy(buf), nbytes, dst=0)
        if rank == 0:
            # every shard's global word offset from the gathered totals
            word0s = [hd.local_geometry(hb, sum(totals[:g]), totals[g], g == 0)[0] for g in range(world)]
            payload = hd.reassemble(shards, word0s, sum(totals), hb)
            blob = header + payload.tobytes()
            ref = oracle_lib.encode(data)
            ok = blob == ref and total == len(ref) - len(header) and header + stream[:total].numpy().tobytes() == ref
            with open(result_path, "w") as f:
                f.write("ok" if ok else "mismatch")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total,kind", [(2, 1 << 20, 1), (2, (1 << 20) + 3, 0), (3, 300001, 1),
                                                (4, 4 * 4096 + 2, 1), (8, 8 * 65536 + 4097, 1),
                                                (8, 8 * 8192 + 2, 0)])
def test_sharded_stream_equals_single_stream(tmp_path, world, n_total, kind):
    result = str(tmp_path / "result.txt")
    mp.start_processes(_worker, args=(world, _free_port(), n_total, kind, result), nprocs=world, join=True,
                       start_method="spawn")
    with open(result) as f:
        assert f.read() == "ok"


def test_shard_ranges_cover_and_align():
    from huffman_amd import dist as hd
    for n, w in [(10, 3), (1 << 20, 8), (7, 2), (100001, 4)]:
        rs = [hd.shard_range(n, w, r) for r in range(w)]
        assert rs[0][0] == 0 and rs[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
        assert all(b % 2 == 0 for b, _ in rs)


def test_part_range_and_window_properties():
    """Equal bit parts of one payload over `world` ranks (dist.part_range), 2 000 seeded random
    geometries: the parts tile [0, P) in rank order on 128-bit boundaries, every non-empty part is at
    least 128 bits unless the whole payload is shorter, empty parts come last; each part's window
    (dist.part_window) covers its lead-in (1 024 bits, or the stream from its start) and max_len bits
    past its end, in whole words."""
    import random
    from huffman_amd import dist as hd
    rnd = random.Random(6)
    for _ in range(2000):
        P = rnd.choice([0, 1, 127, 128, 129, 1000, rnd.randrange(1 << 40)])
        world = rnd.randrange(1, 17)
        parts = [hd.part_range(P, world, r) for r in range(world)]
        assert parts[0][0] == 0 and parts[-1][1] == P
        assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
        nonempty = [(b, e) for b, e in parts if e > b]
        assert all(parts[i][1] > parts[i][0] for i in range(len(nonempty)))  # empty parts last
        assert all(b % 128 == 0 for b, _ in nonempty)
        if P >= 128:
            assert all(e - b >= 128 for b, e in nonempty)
        start, max_len = rnd.randrange(0, 4096), rnd.randrange(1, 57)
        for b, e in nonempty:
            lo, hi = hd.part_window(start, b, e, max_len)
            assert 32 * lo <= start + b - min(1024, b) and start + e + max_len <= 32 * hi
            assert 32 * lo > start + b - min(1024, b) - 32 and 32 * hi < start + e + max_len + 32


def _subgroup_worker(rank, world, port, n_total, result_dir):
    """Two 2-rank subgroups of a 4-rank job, {0, 2} and {1, 3}: each encodes the
    whole (odd) stream sharded over its members. The members' group ranks differ
    from their global ranks, so every src/dst/peer must be translated
    (dist._global): the odd byte comes from global rank 2 (resp. 3), the stream
    lands on global rank 0 (resp. 1)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import huffman_amd
        from huffman_amd import dist as hd
        groups = [dist.new_group([0, 2]), dist.new_group([1, 3])]
        g = groups[rank % 2]
        gr, gw = dist.get_rank(g), dist.get_world_size(g)
        data = oracle_lib.generate(n_total, offset=0, kind=1, seed=13)
        beg, end = hd.shard_range(n_total, gw, gr)
        shard = data[beg:end]
        hist_local = torch.from_numpy(oracle_lib.hist16(shard).astype(np.int64))
        h = hd.global_histogram(hist_local, group=g).numpy().astype(np.uint64)
        cb = huffman_amd.build_codebook(h)
        hb = huffman_amd.header_bits(cb, n_total)
        pbits = huffman_amd.payload_bits(cb, hist_local.numpy().astype(np.uint64))
        off, totals = hd.shard_bit_offsets(pbits, torch.device("cpu"), group=g)
        word0, start, words = hd.local_geometry(hb, off, pbits, gr == 0)
        _, ln, code = huffman_amd.codebook_arrays(cb)
        buf = oracle_lib.pack_range(shard, 0, shard.size // 2, ln, code, start, words * 4 + 8)
        last = hd.odd_last_byte(shard, n_total, group=g)
        header = None
        if gr == 0:
            header, _, pend = huffman_amd.write_header(cb, n_total, last)
            buf[0] |= pend
        nbytes = (start + pbits + 7) // 8
        stream, total = hd.reassemble_on_device(torch.from_numpy(buf.copy()), nbytes, word0, dst=0, group=g)
        shards = hd.gather_to(torch.from_numpy(buf), nbytes, dst=0, group=g)
        if gr == 0:
            word0s = [hd.local_geometry(hb, sum(totals[:k]), totals[k], k == 0)[0] for k in range(gw)]
            payload = hd.reassemble(shards, word0s, sum(totals), hb)
            ref = oracle_lib.encode(data)
            ok = header + payload.tobytes() == ref and header + stream[:total].numpy().tobytes() == ref
            with open(os.path.join(result_dir, f"g{rank % 2}.txt"), "w") as f:
                f.write("ok" if ok else "mismatch")
    finally:
        dist.destroy_process_group()


def test_subgroups_use_global_ranks(tmp_path):
    mp.start_processes(_subgroup_worker, args=(4, _free_port(), 200003, str(tmp_path)), nprocs=4, join=True,
                       start_method="spawn")
    for k in (0, 1):
        assert (tmp_path / f"g{k}.txt").read_text() == "ok"


def _split_worker(rank, world, port, n_total, kind, lead, result_path):
    """One index-less stream (the oracle's encoding: no index, reference format) decoded in parts, one
    per rank (huffman_amd/dist.py decode_indexless_split). The per-part engine here is the oracle's
    serial walk (no GPU); on the GPU the same exchange drives hz_indexless_scan/refix/decode
    (tests/test_gpu_dist.py). `lead`: lead-in bits before a part (0: every rank but 0 starts
    mid-codeword, so the refix rounds run)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from huffman_amd import dist as hd
        data = oracle_lib.generate(n_total, offset=0, kind=kind, seed=23)
        blob = oracle_lib.encode(data)
        _, ln, code, info = oracle_lib.parse_header(blob)
        nsym = info[0] // 2
        pay = np.frombuffer(blob, dtype=np.uint8)[info[1]:]
        start = info[2]
        beg, end = hd.part_range(pay.size * 8 - start, world, rank)
        st = {}

        def scan():
            e = start + beg
            if rank > 0:  # the lead-in walk lands on the first codeword start >= the part's first bit
                _, e, _ = oracle_lib.walk(pay, ln, code, start + beg - min(lead, beg), start + beg)
            n, x, _ = oracle_lib.walk(pay, ln, code, e, start + end)
            st["entry"] = e
            return n, x, e

        def refix(entry):
            n, x, _ = oracle_lib.walk(pay, ln, code, entry, start + end)
            st["entry"] = entry
            return n, x, entry

        def decode(first, take):
            _, _, syms = oracle_lib.walk(pay, ln, code, st["entry"], start + end, max_count=max(take, 0), decode=True)
            st["out"] = (first, syms[:2 * take].tobytes())

        empty = beg == end  # a payload shorter than `world` parts: the trailing ranks have none
        first, count, rounds = hd.decode_indexless_split(scan, refix, decode, nsym, torch.device("cpu"),
                                                         empty=empty)
        if empty:
            st["out"] = (first, b"")
        parts = [None] * world
        dist.all_gather_object(parts, (st["out"][0], st["out"][1], rounds))
        if rank == 0:
            got = b"".join(p[1] for p in sorted(parts, key=lambda p: p[0]))
            ok = got == data[:2 * nsym].tobytes() and all(p[2] == parts[0][2] for p in parts)
            if lead == 0 and world > 1:
                ok = ok and parts[0][2] >= 1  # the refix rounds ran
            with open(result_path, "w") as f:
                f.write("ok" if ok else f"mismatch rounds={parts[0][2]} len={len(got)}/{2 * nsym}")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total,kind,lead", [(2, 300001, 1, 1024), (3, 1 << 20, 1, 1024), (3, 200000, 1, 0),
                                                     (8, (1 << 20) + 7, 1, 1024), (8, 1 << 19, 0, 0),
                                                     (8, 400002, 1, 0), (8, 301, 1, 1024), (3, 41, 1, 1024)])
def test_indexless_split_over_ranks(tmp_path, world, n_total, kind, lead):
    """(The last two: payloads of fewer than `world` 128-bit parts -- trailing ranks get empty parts,
    join every all-gather and pass the exit on, instead of failing before it and hanging the group.)"""
    result = str(tmp_path / "result.txt")
    mp.start_processes(_split_worker, args=(world, _free_port(), n_total, kind, lead, result), nprocs=world, join=True,
                       start_method="spawn")
    assert open(result).read() == "ok"


def _window_worker(rank, world, port, result_path):
    """dist.fill_window on CPU tensors (gloo): shards of one global bit stream packed at their bit offsets
    into word-aligned buffers with a halo (adjacent shards share a boundary word); after the fill, every
    rank's part window holds the global stream's words exactly."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from huffman_amd import dist as hd
        rng = np.random.default_rng(3)
        bits = [int(b) for b in rng.integers(3000, 9000, world)]  # shard payload bits (uneven)
        S0 = 5
        total = sum(bits)
        nw = (S0 + total + 31) // 32 + 64
        stream = np.zeros(nw * 32, dtype=np.uint8)
        stream[S0:S0 + total] = rng.integers(0, 2, total)
        gwords = np.packbits(stream).view(">u4").astype(np.uint32)  # big-endian words of the global stream
        offs = [sum(bits[:g]) for g in range(world)]
        shards = []
        for g in range(world):
            w0, start, words = hd.local_geometry(S0, offs[g], bits[g], g == 0)
            shards.append((w0, words))
        w0, words = shards[rank]
        halo = 256
        ext = torch.zeros(4 * (2 * halo + words + 4), dtype=torch.uint8)
        # this rank's shard: only its own bits (zeros elsewhere in its boundary words)
        own = np.zeros(words * 32, dtype=np.uint8)
        a = S0 + offs[rank] - 32 * w0
        own[a:a + bits[rank]] = stream[S0 + offs[rank]:S0 + offs[rank] + bits[rank]]
        ext[4 * halo:4 * (halo + words)] = torch.from_numpy(np.packbits(own).copy())
        parts = [hd.part_range(total, world, r) for r in range(world)]
        windows = [hd.part_window(S0, pb, pe, 22, lead=1024) for pb, pe in parts]
        hd.fill_window(ext, w0 - halo, w0, words, windows, shards, via_host=True)
        lo, hi = windows[rank]
        got = ext[4 * (lo - (w0 - halo)):4 * (hi - (w0 - halo))].numpy().view(">u4")
        want = gwords[lo:hi]
        ok = np.array_equal(got, want)
        flags = [None] * world
        dist.all_gather_object(flags, ok)
        if rank == 0:
            with open(result_path, "w") as f:
                f.write("ok" if all(flags) else f"mismatch {flags}")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 5])
def test_fill_window_brings_neighbour_words(tmp_path, world):
    result = str(tmp_path / "result.txt")
    mp.start_processes(_window_worker, args=(world, _free_port(), result), nprocs=world, join=True,
                       start_method="spawn")
    assert open(result).read() == "ok"
