"""Benchmark: encode + decode throughput of the Huffman hot path on MI355X.

Metric (BASELINE.json): encode + decode throughput GB/s and % HBM3E peak,
16 GiB Zipf(1.1) per GPU, 1/2/4/8 GPUs. One step = one full pass of the hot
path over the rank's 16 GiB shard, inputs already resident in HBM:

    hist16 (GPU) -> [all-reduce of the 512 KiB histogram when N > 1]
    -> host codebook (reference GenerateCL semantics) + header + table upload
    -> [all-gather of per-rank payload bits when N > 1: global bit offsets]
    -> pack (GPU) -> decode (GPU)

value = input bytes of all ranks / max-over-ranks step time (weak scaling).
The round trip is verified bit-exact on the device after the timed loop.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--size BYTES] [--dist zipf|uniform]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(msg):
    """Progress on stderr (the JSON line alone goes to stdout)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=16 << 30, help="input bytes per GPU")
    ap.add_argument("--dist", default="zipf", choices=["zipf", "uniform"])
    ap.add_argument("--cpu-sample-mib", type=int, default=128, help="one-process CPU baseline sample")
    ap.add_argument("--cpu-par-sample-mib", type=int, default=48, help="per-process sample, all-core CPU baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--no-reassemble", action="store_true", help="N>1: skip the (untimed-in-step) stream reassembly")
    ap.add_argument("--rehearse", action="store_true",
                    help="N>1 rehearsal on one GPU: every rank on cuda:0, gloo collectives through host copies")
    return ap.parse_args()


def _cpu_info():
    """Cores this process may use (the box's CPU share) and the host CPU model."""
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    # the CPU share of this job: the cgroup quota, else OMP_NUM_THREADS (affinity shows the whole machine)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            cores = min(cores, max(1, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        cores = min(cores, int(os.environ["OMP_NUM_THREADS"]))
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return cores, model


def _baseline_run(args):
    """One reference baseline encode + decode of `sample.bin` in its own CWD
    (the reference decoder always writes ./DECOMPRESSED_FILE); wall times."""
    enc_exe, dec_exe, td, data_bytes = args
    t0 = time.perf_counter()
    subprocess.run([enc_exe, "sample.bin"], cwd=td, check=True, capture_output=True)
    t1 = time.perf_counter()
    subprocess.run([dec_exe, "sample.bin.compressed"], cwd=td, check=True, capture_output=True)
    t2 = time.perf_counter()
    with open(os.path.join(td, "DECOMPRESSED_FILE"), "rb") as f:
        ok = f.read() == data_bytes
    return t1 - t0, t2 - t1, t2 - t0, ok


def cpu_baseline(sample_bytes, kind, par_sample_bytes):
    """Reference baseline/ encoder + decoder (built from the reference sources by
    oracle/Makefile) on bounded samples of the same stream:
    (i) one process on the first sample_bytes, (ii) one process per core this
    job may use, all at once, each on its own slice of par_sample_bytes in its
    own CWD. `value` is the all-core aggregate; the one-process rate is beside it."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    from concurrent.futures import ThreadPoolExecutor
    cores, model = _cpu_info()
    enc_exe, dec_exe = oracle_lib.ref_binary("archive_baseline"), oracle_lib.ref_binary("extract_baseline")
    if not (enc_exe and dec_exe):  # restatement in C (port): one process, same work
        data = oracle_lib.generate(sample_bytes, offset=0, kind=kind, seed=42)
        t0 = time.perf_counter()
        blob = oracle_lib.encode(data)
        ok = oracle_lib.decode(blob) == data.tobytes()
        t = time.perf_counter() - t0
        return {"value": round(sample_bytes / t / 1e9, 5), "unit": "GB/s", "cores": 1, "kind": "port",
                "sample": f"{sample_bytes >> 20} MiB prefix, oracle encode + decode, one process; round trip "
                          f"{'ok' if ok else 'FAILED'}", "cpu_model": model}
    with tempfile.TemporaryDirectory() as root:
        def stage(i, nbytes):
            d = os.path.join(root, f"p{i}")
            os.makedirs(d)
            data = oracle_lib.generate(nbytes, offset=i * nbytes, kind=kind, seed=42)
            data.tofile(os.path.join(d, "sample.bin"))
            return (enc_exe, dec_exe, d, data.tobytes())
        one = _baseline_run(stage(0, sample_bytes))
        log(f"CPU baseline: one process done ({one[2]:.1f} s); {cores} concurrent processes")
        jobs = [stage(1000 + i, par_sample_bytes) for i in range(cores)]
        t0 = time.perf_counter()
        with ThreadPoolExecutor(max_workers=cores) as ex:
            res = list(ex.map(_baseline_run, jobs))
        wall = time.perf_counter() - t0
    ok = one[3] and all(r[3] for r in res)
    agg = cores * par_sample_bytes / wall / 1e9
    return {
        "value": round(agg, 5),
        "unit": "GB/s",
        "cores": cores,
        "kind": "reference",
        "cpu_model": model,
        "sample": f"reference baseline/Compressor.cu then baseline/Decompressor.cu (g++ -O3) on the same synthetic "
                  f"stream (seed 42): {cores} concurrent processes, one per core, each its own "
                  f"{par_sample_bytes >> 20} MiB slice in its own CWD ({wall:.2f} s wall); one process on the "
                  f"first {sample_bytes >> 20} MiB: encode {one[0]:.2f} s, decode {one[1]:.2f} s; round trips "
                  f"{'ok' if ok else 'FAILED'}",
        "one_process_GBps": round(sample_bytes / one[2] / 1e9, 5),
        "one_process_encode_GBps": round(sample_bytes / one[0] / 1e9, 5),
        "one_process_decode_GBps": round(sample_bytes / one[1] / 1e9, 5),
    }


def reassemble(codec, plan, payload, rank, world, n_total, kind, args, dev):
    """SURVEY.md 8(e) step 7, outside the timed step: every rank's shard of the
    payload lands in ONE stream on rank 0 (RCCL point-to-point over xGMI).
    Timed on its own; when the stream is small enough, rank 0 decodes it whole
    (index rebuilt from the stream alone) and checks it against the input."""
    import torch
    import torch.distributed as dist
    from huffman_amd import dist as hd
    from huffman_amd import index_bytes
    offset = plan.stream_bit - plan.header_bits % 8
    word0, _, _ = hd.local_geometry(plan.header_bits, offset, plan.payload_bits, rank == 0)
    nbytes = (plan.start_bit + plan.payload_bits + 7) // 8
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stream, total = hd.reassemble_on_device(payload, nbytes, word0, dst=0, via_host=args.rehearse)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    dist.barrier()
    res = None
    if rank == 0:
        res = {"ms": round(ms, 3), "stream_bytes": int(total), "GBps_into_rank0": round(total / ms / 1e6, 1),
               "transport": "gloo via host (rehearsal)" if args.rehearse else "RCCL isend/irecv"}
        if n_total <= (9 << 30):  # the 8-rank rehearsal's 8 GiB stream (tests/test_gpu_dist.py); not 8 x 16 GiB
            nsym = n_total // 2
            idx = torch.empty((index_bytes(nsym) + 7) // 8 + 1, dtype=torch.int64, device=dev)
            codec.dev.index_build(stream.data_ptr(), stream.numel(), plan.header_bits % 8, nsym, idx.data_ptr())
            got = torch.empty(n_total + 16, dtype=torch.uint8, device=dev)
            codec.decode(stream, nsym, idx, got)
            ref = torch.empty(n_total, dtype=torch.uint8, device=dev)
            codec.dev.generate(ref.data_ptr(), n_total, offset=0, kind=kind, alpha=1.1, seed=42)
            codec.sync()
            res["whole_stream_decoded_bit_exact"] = bool(torch.equal(got[:n_total], ref))
            del idx, got, ref
        del stream
    dist.barrier()
    return res


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rehearse:
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if args.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def all_reduce(t, op=None):
        op = dist.ReduceOp.SUM if op is None else op
        if not args.rehearse:
            dist.all_reduce(t, op=op)
            return
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)

    def all_gather(out, inp):
        if not args.rehearse:
            dist.all_gather_into_tensor(out, inp)
            return
        parts = [torch.empty_like(inp, device="cpu") for _ in range(world)]
        dist.all_gather(parts, inp.cpu())
        out.copy_(torch.cat(parts))

    from huffman_amd.codec import build_codebook, payload_bits
    from huffman_amd._lib import build_id
    from huffman_amd.pipeline import StreamCodec

    codec = StreamCodec(local)
    dev = codec.device
    N = args.size
    N -= N % 2 if world > 1 else 0  # shards hold whole symbols
    kind = 1 if args.dist == "zipf" else 0
    x = torch.empty(N, dtype=torch.uint8, device=dev)
    # rank g holds bytes [g*N, (g+1)*N) of one global stream
    codec.dev.generate(x.data_ptr(), N, offset=rank * N, kind=kind, alpha=1.1, seed=42)
    n_total = N * world
    nsym = N // 2
    out = torch.empty(2 * nsym + 16, dtype=torch.uint8, device=dev)
    hist_local = torch.zeros(65536, dtype=torch.int64, device=dev)
    tbits = torch.zeros(world, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    state = {}

    def sidecar(plan, dropin, force_index=False):
        """Whether pack writes the block index and decode reads it: not on the drop-in path, and not
        for a FIXED16 codebook (every code 16 bits: its decoder places symbol i at start + 16 i and reads
        no index; hz_decode_indexless takes it directly) unless the index itself is wanted."""
        fixed16 = int(plan.cb.min_len) == 16 and int(plan.cb.max_len) == 16
        return not dropin and (force_index or not fixed16)

    def step(dropin=False, force_index=False):
        codec.histogram(x)
        if world > 1:
            hist_local.copy_(codec.hist)
            all_reduce(codec.hist)
        h = codec.hist.cpu().numpy().view(np.uint64)
        hl = hist_local.cpu().numpy().view(np.uint64) if world > 1 else h
        cb = build_codebook(h)
        offset = 0
        if world > 1:
            mine = torch.tensor([payload_bits(cb, hl)], dtype=torch.int64, device=dev)
            all_gather(tbits, mine)
            offset = int(tbits[:rank].sum().item())
        last = 0  # N is even for every shard here
        plan = codec.make_plan(h, n_total, hist_local=hl, first_shard=(rank == 0), shard_bit_offset=offset,
                               last_byte=last, cb=cb)
        if "payload" not in state or state["payload"].numel() < plan.words * 4 + 16:
            state["payload"], state["index"] = codec.alloc_payload(plan, nsym)
        side = sidecar(plan, dropin, force_index)
        codec.pack(x, plan, state["payload"], state["index"] if side else None)
        codec.upload_decode(plan)  # host builds the decode tables while pack runs
        if not side:
            codec.dev.decode_indexless(state["payload"].data_ptr(), state["payload"].numel(), plan.start_bit, nsym,
                                       out.data_ptr(), endb.data_ptr())
        else:
            codec.decode(state["payload"], nsym, state["index"], out)
        state["header"] = plan.header  # the .compressed header, written on the host while the GPU runs
        state["plan"] = plan

    # Pipelined steps: every step does hist -> codebook -> pack -> decode of one batch,
    # in one stream, and the next batch's histogram runs between this batch's pack and
    # decode, so the host builds the next codebook and encode tables while this batch
    # decodes (no work is skipped or reused: each batch's histogram, codebook, tables,
    # pack and decode are its own). N > 1: the ranks all-gather their local histograms
    # right after the histogram; every rank sums them (the global histogram) and
    # computes every rank's payload bits from them (its bit offset), so one collective
    # per step suffices and it is off the host's critical path too.
    hist_all = torch.zeros((world, 65536), dtype=torch.int64, device=dev)
    hist_host = torch.empty((world, 65536), dtype=torch.int64).pin_memory()
    ready = torch.cuda.Event()

    def hist_launch():
        codec.histogram(x)
        if world > 1:
            all_gather(hist_all.view(-1), codec.hist)
        else:
            hist_all[0].copy_(codec.hist)
        hist_host.copy_(hist_all, non_blocking=True)
        ready.record()

    def hist_plan():
        ready.synchronize()
        hs = hist_host.numpy().view(np.uint64)
        h = hs.sum(axis=0) if world > 1 else hs[0]
        cb = build_codebook(h)
        offset = 0
        bits = None
        if world > 1:
            bits = [int(payload_bits(cb, hs[r])) for r in range(world)]  # every shard's (the split decode)
            offset = int(sum(bits[:rank]))
        plan = codec.make_plan(h, n_total, hist_local=hs[rank], first_shard=(rank == 0), shard_bit_offset=offset,
                               last_byte=0, cb=cb)  # N is even for every shard here
        plan.all_bits = bits
        return plan

    # N > 1 drop-in: the `extract` of ONE reference-format stream by every rank (SURVEY.md 8e decode):
    # the global payload (every shard at its global bit offset) is split into equal bit parts
    # (dist.part_range), not at the shards' encode start bits -- a .compressed file carries none. Each
    # rank's part window (the part, its 1024-bit lead-in, max_len bits after) lies in its own shard's
    # buffer plus a halo: the neighbours' words inside it travel point-to-point (dist.fill_window), and
    # the part is decoded through hz_indexless_scan / _refix / _decode with the ranks' exchange
    # (dist.decode_indexless_split).
    from huffman_amd import dist as hd
    HALO = 1 << 22  # words on each side of the shard (16 MiB): equal bit parts lie this close to the shards
    split = {}

    def split_geometry(plan):
        S0 = plan.header_bits % 8
        offs = [int(sum(plan.all_bits[:g])) for g in range(world)]
        shards = []
        for g in range(world):
            w0, _, words = hd.local_geometry(plan.header_bits, offs[g], plan.all_bits[g], g == 0)
            shards.append((w0, words))
        P = int(sum(plan.all_bits))
        parts = [hd.part_range(P, world, r) for r in range(world)]
        windows = [hd.part_window(S0, pb, pe, int(plan.cb.max_len)) for pb, pe in parts]
        return S0, shards, parts, windows

    def split_alloc(plan):
        need = 4 * (2 * HALO + plan.words + 4)
        if "ext" not in split or split["ext"].numel() < need:
            split.pop("ext", None)
            split["ext"] = torch.zeros(need, dtype=torch.uint8, device=dev)
        ext = split["ext"]
        return ext, ext[4 * HALO:4 * (HALO + plan.words) + 16]

    def split_decode(plan, ext):
        """The part of this rank, decoded into split['out']; returns (first symbol, symbols taken)."""
        S0, shards, parts, windows = split_geometry(plan)
        w0, words = shards[rank]
        ext_word0 = w0 - HALO
        lo, hi = windows[rank]
        if not (ext_word0 <= lo and hi <= ext_word0 + ext.numel() // 4):
            raise RuntimeError(f"rank {rank}: part window {lo}..{hi} beyond the shard's halo")
        ext[:4 * HALO].zero_()
        ext[4 * (HALO + words):].zero_()
        hd.fill_window(ext, ext_word0, w0, words, windows, shards, via_host=args.rehearse)
        sl = ext[4 * (lo - ext_word0):4 * (hi - ext_word0)]
        pb, pe = parts[rank]
        summ = split["summ"]
        nsym_all = n_total // 2

        def read():
            codec.sync()
            v = [int(t) & ((1 << 64) - 1) for t in summ[:3].cpu().tolist()]
            return v[0], v[1], v[2]

        def scan():
            codec.dev.indexless_scan(sl.data_ptr(), sl.numel(), S0, pb, pe,
                                     S0 if rank == 0 else hd.UNKNOWN_ENTRY, summ.data_ptr(), nsym=nsym_all,
                                     payload_bit_base=32 * lo)
            return read()

        def refix(entry):
            codec.dev.indexless_refix(entry, summ.data_ptr())
            return read()

        def decode(first, take):
            if take > split["cap"]:
                raise RuntimeError(f"rank {rank}: part of {take} symbols over the output buffer")
            codec.dev.indexless_decode(take, split["out"].data_ptr(), endb.data_ptr())

        grp_dev = torch.device("cpu") if args.rehearse else dev
        first, count, _ = hd.decode_indexless_split(scan, refix, decode, nsym_all, grp_dev, empty=pb == pe)
        return first, max(0, min(count, nsym_all - first))

    def run(steps, dropin=False):
        """dropin=False: pack writes its block index beside the payload and decode reads it (the
        sidecar-index figure). dropin=True: what the reference's file path does, on the device --
        pack writes NO index (a .compressed payload carries none, Compressor.cu:427-601) and the
        decode is hz_decode_indexless of the bare payload (the `extract` path)."""
        hist_launch()
        plan = hist_plan()
        for i in range(steps):
            if "payload" not in state or state["payload"].numel() < plan.words * 4 + 16:
                state["payload"], state["index"] = codec.alloc_payload(plan, nsym)
            side = sidecar(plan, dropin)
            splitting = dropin and world > 1
            if splitting:  # the shard packed into its place in the part-window buffer
                ext, pay = split_alloc(plan)
                codec.pack(x, plan, pay, None)
            else:
                codec.pack(x, plan, state["payload"], state["index"] if side else None)
            if i + 1 < steps:
                hist_launch()  # the next batch's histogram, between this batch's pack and decode
            codec.upload_decode(plan)  # host builds the decode tables while pack runs
            if splitting:
                split["last"] = split_decode(plan, ext)
            elif not side:
                codec.dev.decode_indexless(state["payload"].data_ptr(), state["payload"].numel(), plan.start_bit,
                                           nsym, out.data_ptr(), endb.data_ptr())
            else:
                codec.decode(state["payload"], nsym, state["index"], out)
            state["header"] = plan.header  # the .compressed header, written on the host while the GPU runs
            state["plan"] = plan
            if i + 1 < steps:
                plan = hist_plan()  # while this batch decodes

    def timed(steps, dropin=False):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(steps, dropin)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return time.perf_counter() - t0

    endb = torch.zeros(2, dtype=torch.int64, device=dev)
    if world > 1:
        split["summ"] = torch.zeros(4, dtype=torch.int64, device=dev)
        split["cap"] = nsym + 32 * HALO  # a part's symbols: its shard's give or take the halo's bits
        split["out"] = torch.empty(2 * split["cap"] + 16, dtype=torch.uint8, device=dev)

    log(f"rank {rank}: {N} bytes generated; {args.warmup} warmup steps")
    if args.warmup:
        run(args.warmup)
    codec.sync()
    log(f"rank {rank}: {args.steps} timed steps")
    elapsed = timed(args.steps)
    codec.sync()  # surfaces device-side errors (capacity, format)
    ok = bool(torch.equal(out[:2 * nsym], x[:2 * nsym]))
    # the drop-in file path, timed the same way: pack without an index, index-less decode
    log(f"rank {rank}: drop-in path (no index): {args.warmup} warmup + {args.steps} timed steps")
    out.fill_(0)
    if args.warmup:
        run(args.warmup, dropin=True)
    codec.sync()
    elapsed_dropin = timed(args.steps, dropin=True)
    codec.sync()
    if world > 1:
        # this rank's part of the one stream: its symbols from the generator at their global offset
        first, take = split["last"]
        ref = torch.empty(2 * take + 16, dtype=torch.uint8, device=dev)
        if take:
            codec.dev.generate(ref.data_ptr(), 2 * take, offset=2 * first, kind=kind, alpha=1.1, seed=42)
        codec.sync()
        ok_dropin = bool(torch.equal(split["out"][:2 * take], ref[:2 * take]))
        split["checked"] = {"first_symbol": first, "symbols": take, "bit_exact": ok_dropin}
        del ref
    else:
        ok_dropin = bool(torch.equal(out[:2 * nsym], x[:2 * nsym]))
    ok = ok and ok_dropin
    # Kernel times (HIP events) and host stage costs: two more steps, serialised, untimed.
    kms = {"hist": [], "pack": [], "decode": []}
    host_ms = []
    host_dec_ms = []
    from huffman_amd._lib import STAGE_EXTRACT
    for _ in range(2):
        step()
        torch.cuda.synchronize()
        side = sidecar(state["plan"], False)
        for k, v in codec.kernel_ms().items():
            # (a FIXED16 step decodes through hz_decode_indexless: its time is the extract stage's)
            kms[k].append(v if k != "decode" or side else codec.dev.kernel_ms(STAGE_EXTRACT))
        host_ms.append(codec.timings.get("codebook_ms", 0) + codec.timings.get("upload_ms", 0))
        host_dec_ms.append(codec.timings.get("upload_decode_ms", 0))
    ok = ok and bool(torch.equal(out[:2 * nsym], x[:2 * nsym]))
    # the drop-in step's kernels (pack without an index; the index-less decode), serialised, untimed
    dk = {"hist": [], "pack": [], "extract": []}
    for _ in range(2):
        out.fill_(0)
        step(dropin=True)
        torch.cuda.synchronize()
        km = codec.kernel_ms()
        dk["hist"].append(km["hist"])
        dk["pack"].append(km["pack"])
        dk["extract"].append(codec.dev.kernel_ms(STAGE_EXTRACT))
    ok = ok and bool(torch.equal(out[:2 * nsym], x[:2 * nsym]))
    step(force_index=True)  # payload and index of the sidecar-index path again, for the checks below
    torch.cuda.synchronize()
    plan = state["plan"]
    log(f"rank {rank}: {elapsed * 1e3 / args.steps:.3f} ms/step; index rebuild from the payload")
    # Index-less decode path (reference-produced files): rebuild the block index
    # from the payload alone, outside the timed loop, and check it against pack's.
    from huffman_amd import index_bytes
    from huffman_amd._lib import STAGE_INDEX
    nidx = (index_bytes(nsym) + 7) // 8
    rebuilt = torch.empty_like(state["index"])
    codec.dev.index_build(state["payload"].data_ptr(), state["payload"].numel(), plan.start_bit, nsym,
                          rebuilt.data_ptr())
    codec.sync()
    index_build = {"ms": round(codec.dev.kernel_ms(STAGE_INDEX), 3),
                   "matches_pack_index": bool(torch.equal(rebuilt[:nidx], state["index"][:nidx]))}
    del rebuilt
    # `extract` of an index-less file on the device: hz_decode_indexless (no block index; chain walk,
    # fix-ups, chain-block decode), its output checked against the input, its end bit against pack's index
    xms = []
    for _ in range(2):
        out.fill_(0)
        codec.dev.decode_indexless(state["payload"].data_ptr(), state["payload"].numel(), plan.start_bit, nsym,
                                   out.data_ptr(), endb.data_ptr())
        codec.sync()
        xms.append(codec.dev.kernel_ms(STAGE_EXTRACT))
    nb_idx = (nsym + 2047) // 2048
    extract = {"ms": round(float(np.mean(xms)), 3), "ms_runs": [round(v, 3) for v in xms],
               "bit_exact": bool(torch.equal(out[:2 * nsym], x[:2 * nsym])),
               "end_bit_matches_pack_index": int(endb[0].item()) == int(state["index"][nb_idx].item())}
    ok = ok and extract["bit_exact"]
    reassembly = None
    if world > 1 and not args.no_reassemble:
        reassembly = reassemble(codec, plan, state["payload"], rank, world, n_total, kind, args, dev)
    C = plan.payload_bits // 8
    if world > 1:
        t = torch.tensor([elapsed, elapsed_dropin, 0.0 if ok else 1.0], dtype=torch.float64, device=dev)
        all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, elapsed_dropin, bad = float(t[0]), float(t[1]), float(t[2])
        ok = bad == 0.0
    ms_step = elapsed / args.steps * 1e3
    value = n_total / (ms_step / 1e3) / 1e9
    ms_dropin = elapsed_dropin / args.steps * 1e3

    if rank == 0:
        avg = {k: float(np.mean(v)) for k, v in kms.items()}
        algo = {"hist": N, "pack": N + C, "decode": C + 2 * nsym}
        dom = max(avg, key=lambda k: avg[k])
        achieved = algo[dom] / (avg[dom] / 1e3) / 1e9
        pmc = {}
        if os.path.exists(args.profile_json):
            try:
                with open(args.profile_json) as f:
                    pmc = json.load(f).get(args.dist, {})
            except Exception:
                pmc = {}

        def pmc_traffic(stage):
            # only counters of this very build (same sources) and this input size count
            ent = pmc.get(stage)
            if ent and ent.get("size") == N and ent.get("build_id") == build_id():
                return ent["hbm_bytes_per_launch"]
            return None

        traffic = pmc_traffic(dom)
        pmc_src = os.path.relpath(args.profile_json, ROOT) if traffic is not None else None
        enc_ms = avg["hist"] + avg["pack"]
        enc_algo = 2 * N + C  # hist reads N; pack reads N and writes C
        enc_traffic = [pmc_traffic("hist"), pmc_traffic("pack")]
        # payload read + block index written; a FIXED16 stream's index is arithmetic (k_idx_fixed16 reads
        # no payload), so there only the index bytes written count
        fixed16 = int(plan.cb.min_len) == 16 and int(plan.cb.max_len) == 16
        idx_algo = index_bytes(nsym) + (0 if fixed16 else C)
        idx_traffic = pmc_traffic("index")
        line = {
            "metric": "encode + decode throughput GB/s and % HBM3E peak, 16 GiB Zipf(1.1), 1/2/4/8 GPU",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic {args.dist} byte stream (splitmix64 seed 42, counter-based; rank g = bytes "
                    f"[g*N,(g+1)*N) of one stream), generated in HBM",
            "config": {
                "workload": f"{N / 2**30:g} GiB {'Zipf(1.1)' if kind else 'uniform'} bytes per GPU: "
                            "hist16 -> codebook -> pack -> decode, one global bit stream",
                "bytes_per_gpu": N,
                "total_bytes": n_total,
                "symbols_per_gpu": nsym,
                "parallelism": f"shard{world}" if world > 1 else "single",
                "payload_bytes_rank0": C,
                "compression_ratio_rank0": round(C / N, 4),
                "max_code_len": int(plan.cb.max_len),
            },
            "step_schedule": "pipelined, one stream: batch k+1's histogram runs between batch k's pack and "
                             "decode, so its host codebook and encode tables are built while batch k decodes; "
                             "kernel_ms and host_* come from two further serialised steps; pack writes the "
                             "block index and decode reads it, except for a FIXED16 codebook (every code 16 bits), "
                             "whose decoder needs no index (hz_decode_indexless: symbol i at start + 16 i)",
            "roundtrip_bit_exact": ok,
            "index_build_from_payload": index_build,
            "extract_indexless": extract,
            # the drop-in file path timed like the headline (same --steps / --warmup, same clock): pack
            # writes no block index (a .compressed payload has none) and the decode is the index-less
            # extract of the bare payload
            "dropin": {
                "schedule": "pipelined like the headline: hist16_ranges -> host codebook -> pack_ranges "
                            "(no index) -> hz_decode_indexless; the next batch's histogram between pack "
                            "and decode",
                "steps": args.steps,
                "warmup": args.warmup,
                "ms_per_step": round(ms_dropin, 3),
                "value": round(n_total / (ms_dropin / 1e3) / 1e9, 2),
                "unit": "GB/s",
                "roundtrip_bit_exact": ok_dropin,
                # N > 1: the timed decode is ONE stream's extract split over the ranks at equal bit parts
                # (not at the shards' encode start bits, which a .compressed file does not carry)
                "decode": ("index-less extract of the one global stream, split over the ranks at equal payload "
                           "bit parts: halo words point-to-point (dist.fill_window), hz_indexless_scan/refix/decode "
                           "with the ranks' exchange (dist.decode_indexless_split)") if world > 1
                          else "hz_decode_indexless of the whole payload",
                "split_check_rank0": split.get("checked") if world > 1 else None,
                "transport": ("gloo via host (one-GPU rehearsal)" if args.rehearse else "RCCL") if world > 1 else None,
                # kernel_ms: serialised per-rank steps; N > 1 they decode each rank's own shard
                "kernel_ms": {k: round(float(np.mean(v)), 4) for k, v in dk.items()},
                "roofline": {
                    "kernel": "extract",
                    "bound": "hbm",
                    "achieved": round((C + 2 * nsym) / (float(np.mean(dk["extract"])) / 1e3) / 1e9, 1),
                    "peak": HBM_PEAK_GBPS,
                    "unit": "GB/s",
                    "frac": round((C + 2 * nsym) / (float(np.mean(dk["extract"])) / 1e3) / 1e9 / HBM_PEAK_GBPS,
                                  4),
                    "traffic": pmc_traffic("extract"),
                    "algorithmic_bytes_per_launch": C + 2 * nsym,
                },
            },
            # algorithmic HBM bytes of one step per GPU: hist N + pack (N + C) + decode (C + N)
            "step_algorithmic_GBps": round((3 * N + 2 * C) / (ms_step / 1e3) / 1e9, 1),
            "step_hbm_frac": round((3 * N + 2 * C) / (ms_step / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
            "kernel_ms": {k: round(v, 4) for k, v in avg.items()},
            "kernel_GBps": {k: round(algo[k] / (avg[k] / 1e3) / 1e9, 1) for k in avg},
            "host_codebook_upload_ms": round(float(np.mean(host_ms)), 3),
            "host_decode_tables_ms_overlapped": round(float(np.mean(host_dec_ms)), 3),
            "encode_GBps_kernels": round(N / (enc_ms / 1e3) / 1e9, 1),
            "decode_GBps_kernel": round(N / (avg["decode"] / 1e3) / 1e9, 1),
            # what `extract` of a real (index-less) file costs beside the encode: hist -> pack ->
            # index-less decode of the payload alone (kernel times, data resident); the API path that
            # rebuilds the block index first (hz_index_build + hz_decode) beside it
            "file_roundtrip": {
                "ms": round(avg["hist"] + avg["pack"] + extract["ms"], 3),
                "GBps_of_input": round(N / ((avg["hist"] + avg["pack"] + extract["ms"]) / 1e3) / 1e9, 1),
                "extract_ms": extract["ms"],
                "extract_GBps_of_output": round(N / (extract["ms"] / 1e3) / 1e9, 1),
                "index_build_plus_decode_ms": round(index_build["ms"] + avg["decode"], 3),
            },
            "reassembly_outside_step": reassembly,
            "roofline": {
                "kernel": dom,
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "traffic_source": pmc_src,
                "build_id": build_id(),
                "algorithmic_bytes_per_launch": algo[dom],
            },
            # the north-star target: encode (hist + pack, the two passes over the input) against HBM peak
            "encode_roofline": {
                "kernels": ["hist", "pack"],
                "bound": "hbm",
                "ms": round(enc_ms, 4),
                "achieved": round(enc_algo / (enc_ms / 1e3) / 1e9, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(enc_algo / (enc_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                "traffic": sum(enc_traffic) if None not in enc_traffic else None,
                "algorithmic_bytes_per_launch": enc_algo,
            },
            # `extract` of an index-less file: the payload read (twice: the length walk and the decode
            # pass) and the output written; algorithmic bytes C + N (payload in, symbols out)
            "extract_roofline": {
                "kernels": ["chain_walk", "chain_fix", "scan", "chain_meta", "chain_decode", "chain_tail"],
                "bound": "hbm",
                "ms": extract["ms"],
                "achieved": round((C + 2 * nsym) / (extract["ms"] / 1e3) / 1e9, 1) if extract["ms"] else None,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round((C + 2 * nsym) / (extract["ms"] / 1e3) / 1e9 / HBM_PEAK_GBPS, 4) if extract["ms"] else None,
                "traffic": pmc_traffic("extract"),
                "algorithmic_bytes_per_launch": C + 2 * nsym,
            },
            # the block-index builder (hz_index_build, the API path for callers that keep an index)
            "index_roofline": {
                "kernels": ["index_build"],
                "bound": "hbm",
                "ms": index_build["ms"],
                "achieved": round(idx_algo / (index_build["ms"] / 1e3) / 1e9, 1) if index_build["ms"] else None,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(idx_algo / (index_build["ms"] / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)
                if index_build["ms"] else None,
                "traffic": idx_traffic,
                "algorithmic_bytes_per_launch": idx_algo,
            },
        }
        if not args.no_cpu_baseline:
            log("CPU baseline (reference baseline/ encoder + decoder)")
            line["cpu_baseline"] = cpu_baseline(args.cpu_sample_mib << 20, kind, args.cpu_par_sample_mib << 20)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
