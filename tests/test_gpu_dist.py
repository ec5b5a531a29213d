"""The sharded path on the HIP kernels: an N-rank rehearsal on
one GPU (every rank on cuda:0, gloo collectives through host copies).

Each rank generates its shard of one global stream on the device, runs the
device histogram, joins the histogram all-reduce and the payload-bit
all-gather (huffman_amd/dist.py), packs its shard with hz_pack at its global
bit offset, decodes it back through the pack index, and ships its payload to
rank 0 through dist.reassemble_on_device. Rank 0's header + reassembled stream
must equal the CPU oracle's encoding of the whole stream byte for byte, and
decode whole on the device (index rebuilt from the stream alone). The 8-rank
geometry is the 128 GiB config's (8 x MI355X) at test size, with a ragged,
odd-length final shard whose raw byte travels to rank 0's header.

Tolerance: none (bit-exact)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle_lib

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, kind, result_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    status = "error"
    try:
        import huffman_amd
        from huffman_amd import dist as hd
        from huffman_amd.pipeline import StreamCodec
        codec = StreamCodec(0)
        dev = codec.device
        beg, end = hd.shard_range(n_total, world, rank)
        n = end - beg
        x = torch.empty(max(n, 16), dtype=torch.uint8, device=dev)[:n]
        codec.dev.generate(x.data_ptr(), n, offset=beg, kind=kind, alpha=1.1, seed=42)
        codec.histogram(x)
        hl = codec.hist.cpu()
        h = hl.clone()
        dist.all_reduce(h)                                         # 1. histogram all-reduce
        h_np = h.numpy().view(np.uint64)
        hl_np = hl.numpy().view(np.uint64)
        cb = huffman_amd.build_codebook(h_np)
        pbits = huffman_amd.payload_bits(cb, hl_np)
        off, totals = hd.shard_bit_offsets(pbits, torch.device("cpu"))   # 2. bit-offset all-gather
        last = hd.odd_last_byte(x.cpu().numpy(), n_total)
        plan = codec.make_plan(h_np, n_total, hist_local=hl_np, first_shard=(rank == 0), shard_bit_offset=off,
                               last_byte=last, cb=cb)
        nsym = n // 2
        payload, index = codec.alloc_payload(plan, nsym)
        codec.pack(x, plan, payload, index)                        # 3. pack at the global offset
        codec.upload_decode(plan)
        out = torch.empty(2 * nsym + 16, dtype=torch.uint8, device=dev)
        codec.decode(payload, nsym, index, out)
        codec.sync()
        local_ok = bool(torch.equal(out[:2 * nsym], x[:2 * nsym]))
        word0, start, words = hd.local_geometry(plan.header_bits, off, pbits, rank == 0)
        assert start == plan.start_bit and words == plan.words
        nbytes = (plan.start_bit + pbits + 7) // 8
        stream, total = hd.reassemble_on_device(payload, nbytes, word0, dst=0, via_host=True)
        flags = torch.tensor([0 if local_ok else 1], dtype=torch.int64)
        dist.all_reduce(flags)
        if rank == 0:
            if n_total > (64 << 20):  # the device generator (== oracle_lib.generate, test_gpu.py) is faster
                g = torch.empty(n_total, dtype=torch.uint8, device=dev)
                codec.dev.generate(g.data_ptr(), n_total, offset=0, kind=kind, alpha=1.1, seed=42)
                data = g.cpu().numpy()
                del g
            else:
                data = oracle_lib.generate(n_total, offset=0, kind=kind, seed=42)
            ref = oracle_lib.encode(data)
            blob = plan.header + stream[:total].cpu().numpy().tobytes()
            checks = {
                "per_rank_roundtrip": int(flags.item()) == 0,
                "file_equals_oracle": blob == ref,
                "whole_stream_decodes": huffman_amd.decode(blob) == data.tobytes(),
            }
            status = ",".join(k for k, v in checks.items() if not v) or "ok"
        else:
            status = "ok"
    finally:
        with open(os.path.join(result_dir, f"rank{rank}.txt"), "w") as f:
            f.write(status)
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,n_total,kind", [(8, 8 * (1 << 20) + 4097, 1), (8, 8 * (256 << 10) + 2, 0),
                                                (3, (3 << 20) + 1, 1),
                                                # real shard sizes: 4 x 256 MiB, the last shard odd (256 MiB + 3)
                                                (4, 4 * (256 << 20) + 3, 1)])
def test_sharded_rehearsal_equals_single_stream(tmp_path, world, n_total, kind):
    mp.start_processes(_worker, args=(world, _free_port(), n_total, kind, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    got = [open(tmp_path / f"rank{r}.txt").read() for r in range(world)]
    assert got == ["ok"] * world, got


def test_bench_rehearsal_three_ranks(tmp_path):
    """bench.py's own N > 1 step (pipelined: histogram all-gather, offsets from the
    gathered local histograms) under torch.distributed.run, every rank on cuda:0:
    each rank's round trip and the reassembled whole stream must be bit-exact."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "3", "--rehearse", "--size", str(96 << 20), "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 3 and line["roundtrip_bit_exact"]  # every rank's, the split drop-in's included
    assert line["reassembly_outside_step"]["whole_stream_decoded_bit_exact"]
    # the drop-in figure is ONE stream's extract split over the ranks at equal bit parts
    chk = line["dropin"]["split_check_rank0"]
    assert chk["bit_exact"] and chk["first_symbol"] == 0 and chk["symbols"] > 0
    assert line["dropin"]["decode"].startswith("index-less extract of the one global stream")


@pytest.mark.timeout(900)
@pytest.mark.parametrize("dist_kind", ["uniform", "zipf"])
def test_bench_rehearsal_eight_ranks_1gib_shards(tmp_path, dist_kind):
    """The 128 GiB config's geometry at real shard sizes: bench.py's N = 8 step with
    1 GiB + 64 B per rank (an 8 GiB stream), every rank on cuda:0. Uniform shards pack to
    just over 1 GiB of payload each, so the reassembly's messages cross
    huffman_amd/dist.py _P2P_CHUNK (1 GiB); the reassembled 8 GiB stream is then
    decoded whole on rank 0 (index rebuilt from the stream alone) and compared with
    the generator's bytes."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "8", "--rehearse", "--size", str((1 << 30) + 64), "--dist", dist_kind, "--steps", "1", "--warmup", "0",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=840)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 8 and line["roundtrip_bit_exact"]  # every rank's, the split drop-in's included
    assert line["dropin"]["split_check_rank0"]["bit_exact"]
    re = line["reassembly_outside_step"]
    assert re["whole_stream_decoded_bit_exact"]
    if dist_kind == "uniform":
        assert line["config"]["payload_bytes_rank0"] > (1 << 30) + 4  # a shard body spans two messages


def _split_worker(rank, world, port, n_total, lead, result_dir, kind="zipf"):
    """One index-less stream decoded by `world` ranks on one GPU, one part each, through
    hz_indexless_scan / hz_indexless_refix / hz_indexless_decode and the exchange of
    huffman_amd/dist.py decode_indexless_split (gloo here; RCCL on a multi-GPU node)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if lead is not None:
        os.environ["HZ_SEG_LEAD"] = str(lead)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    status = "error"
    try:
        from huffman_amd import dist as hd
        from huffman_amd.pipeline import StreamCodec
        codec = StreamCodec(0)
        dev = codec.device
        if kind == "zipf":
            x = torch.empty(n_total, dtype=torch.uint8, device=dev)
            codec.dev.generate(x.data_ptr(), n_total, offset=0, kind=1, alpha=1.1, seed=7)
        elif kind == "dense":  # every code 11-12 bits: a DEC_DENSE codebook (the LUT built beside it)
            g = torch.Generator(device=dev)
            g.manual_seed(5)
            s = torch.randint(0, 3000, (n_total // 2,), dtype=torch.int32, device=dev, generator=g)
            x = (s * 19 + 7).to(torch.int16).view(torch.uint8)
        elif kind.startswith("random:"):  # test_gpu_extract._random_stream with this seed
            import numpy as np
            from test_gpu_extract import _random_stream
            data, _ = _random_stream(np.random.default_rng(int(kind.split(":")[1])))
            x = torch.from_numpy(data).to(dev)
        elif kind == "skew90":  # 90 % one symbol (~1.1 bits per codeword against a ~1.5-bit Kraft estimate)
            import numpy as np
            rng = np.random.default_rng(5)
            s = np.where(rng.random(n_total // 2) < 0.9, 0, rng.integers(1, 301, n_total // 2)).astype("<u2")
            x = torch.from_numpy(s.view(np.uint8).copy()).to(dev)
        elif kind == "tiny3":  # three symbols, codes of 1-2 bits: a 4-entry chain LUT (padded LDS image)
            import numpy as np
            rng = np.random.default_rng(9)
            s = rng.choice(np.array([5, 300, 40000], dtype="<u2"), size=n_total // 2, p=[0.6, 0.3, 0.1])
            x = torch.from_numpy(s.view(np.uint8).copy()).to(dev)
        else:  # "deep": Fibonacci counts, codes of up to 31 bits (DEEP escapes, serial records)
            from test_gpu_extract import _fib_stream
            x = torch.from_numpy(_fib_stream(2)).to(dev)
        n_total = x.numel()
        plan, payload, _ = codec.encode(x)  # every rank holds the whole stream (as read from one file)
        codec.sync()
        nsym = n_total // 2
        pbits = payload.numel() * 8 - plan.start_bit
        beg, end = hd.part_range(pbits, world, rank)
        summ = torch.zeros(4, dtype=torch.int64, device=dev)

        def read():
            codec.sync()
            v = [int(t) & ((1 << 64) - 1) for t in summ[:3].cpu().tolist()]
            return v[0], v[1], v[2]

        def scan():
            entry = plan.start_bit if rank == 0 else hd.UNKNOWN_ENTRY
            codec.dev.indexless_scan(payload.data_ptr(), payload.numel(), plan.start_bit, beg, end, entry,
                                     summ.data_ptr())
            return read()

        def refix(entry):
            codec.dev.indexless_refix(entry, summ.data_ptr())
            return read()

        out = torch.zeros(2 * nsym + 16, dtype=torch.uint8, device=dev)
        endb = torch.zeros(2, dtype=torch.int64, device=dev)

        def decode(first, take):
            codec.dev.indexless_decode(take, out.data_ptr(), endb.data_ptr())
            codec.sync()

        first, count, rounds = hd.decode_indexless_split(scan, refix, decode, nsym, torch.device("cpu"))
        take = max(0, min(count, nsym - first))
        ok = torch.equal(out[:2 * take], x[2 * first:2 * (first + take)])
        flags = torch.tensor([0 if ok else 1, rounds, take], dtype=torch.int64)
        allf = [torch.zeros(3, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allf, flags)
        total = sum(int(f[2]) for f in allf)
        status = "ok" if all(int(f[0]) == 0 for f in allf) and total == nsym else f"bad {[f.tolist() for f in allf]}"
        if lead == 0 and world > 1 and rounds < 1:  # no lead-in: the refix exchange must have run
            status = f"bad rounds={rounds}"
    finally:
        with open(os.path.join(result_dir, f"r{rank}.txt"), "w") as f:
            f.write(status)
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,n_total,lead,kind", [(2, (8 << 20) + 2, None, "zipf"), (3, (24 << 20) + 6, None, "zipf"),
                                                     (8, (64 << 20) + 2, None, "zipf"), (4, (16 << 20) + 2, 0, "zipf"),
                                                     (3, (64 << 20) + 2, None, "dense"), (2, 0, None, "deep"),
                                                     (3, (24 << 20) + 2, None, "tiny3"), (3, (12 << 20) + 2, None, "skew90"),
                                                     (4, 0, None, "random:1"),
                                                     (3, 0, None, "random:9"), (5, 0, None, "random:11"),
                                                     (2, 0, None, "random:7")])
def test_indexless_split_over_ranks_on_device(tmp_path, world, n_total, lead, kind):
    """One index-less stream split over `world` ranks on one GPU: Zipf (LUT tables), a DEC_DENSE codebook
    (hz_indexless_scan used to refuse it), 31-bit codes (DEEP escapes, serial records) and a three-symbol
    alphabet (1-2 bit codes)."""
    mp.start_processes(_split_worker, args=(world, _free_port(), n_total, lead, str(tmp_path), kind), nprocs=world,
                       join=True, start_method="spawn")
    for r in range(world):
        assert open(tmp_path / f"r{r}.txt").read().startswith("ok"), open(tmp_path / f"r{r}.txt").read()
