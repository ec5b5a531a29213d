"""The `extract` path without a block index (include/huffman_amd.h
hz_decode_indexless: a length walk of long chains recording every 8th codeword,
the chain fix-ups, the count scans and the chain-block decoder, all stream-ordered)
against the inputs it must restore and against hz_pack's own index (its end bit). The reference's
decoder (Decompressor.cu:259-291) is serial; the CPU oracle pins the same
streams in test_gpu.py / test_oracle.py, and the golden reference-encoder files
go through this path via hz.decode (test_gpu.py::test_decode_golden_and_baseline_files).

Tolerance: none -- every check is bit-exact (integer/bit work)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


@pytest.fixture(scope="module")
def hz(built_lib):
    import huffman_amd
    return huffman_amd


@pytest.fixture(scope="module")
def codec(built_lib):
    from huffman_amd.pipeline import StreamCodec
    return StreamCodec(0)


def _check(codec, x, shift=0):
    """Encode x on the device, decode its payload (optionally moved `shift` bytes into a
    buffer) index-less; returns (output equal, end bit equal to pack's)."""
    import torch
    from huffman_amd import index_starts
    n = x.numel()
    nsym = n // 2
    plan, payload, index = codec.encode(x)
    codec.sync()
    end_pack = int(index_starts(index.cpu().numpy(), nsym)[-1])
    pay = payload
    if shift:
        pay = torch.zeros(payload.numel() + shift + 64, dtype=torch.uint8, device="cuda")
        pay[shift:shift + payload.numel()] = payload
    out = torch.empty(2 * nsym + 16, dtype=torch.uint8, device="cuda")
    end = torch.full((2,), -1, dtype=torch.int64, device="cuda")
    codec.dev.decode_indexless(pay.data_ptr(), pay.numel(), plan.start_bit + 8 * shift, nsym, out.data_ptr(),
                               end.data_ptr())
    codec.sync()
    return bool(torch.equal(out[:2 * nsym], x[:2 * nsym])), int(end[0].item()) == end_pack + 8 * shift


@pytest.mark.parametrize("n,shift", [(3, 0), (4099, 0), ((1 << 20) + 1, 0), ((1 << 20) + 2, 13), ((8 << 20) + 6, 0),
                                     ((64 << 20) + 3, 5000), ((256 << 20) + 2, 0)])
def test_indexless_zipf(codec, n, shift):
    import torch
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.dev.generate(x.data_ptr(), n, offset=0, kind=1, alpha=1.1, seed=n % 97)
    ok, end_ok = _check(codec, x, shift)
    assert ok and end_ok


@pytest.mark.parametrize("name", ["dense8", "short", "mid20", "long24"])
def test_indexless_table_shapes(codec, name):
    """Every table shape (DENSE, LUT with short, mid and 24-bit codes) through the chain path."""
    import torch
    from test_gpu import _shape_stream
    x = torch.from_numpy(_shape_stream(name)).cuda()
    ok, end_ok = _check(codec, x)
    assert ok and end_ok


def test_indexless_uniform_near16(codec):
    """Uniform bytes at 16 MiB: counts vary by more than 2x, so codes of 15-17 bits (the chain path)."""
    import torch
    n = (16 << 20) + 2
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.dev.generate(x.data_ptr(), n, offset=0, kind=0, alpha=1.1, seed=3)
    ok, end_ok = _check(codec, x)
    assert ok and end_ok


# (every count within 2x of every other -- all codes 16 bits -- needs about 48 MiB of uniform bytes)
@pytest.mark.parametrize("n,shift", [((64 << 20) + 2, 0), ((48 << 20) + 6, 5)])
def test_indexless_uniform_fixed16(codec, n, shift):
    """FIXED16 (every code 16 bits): hz_decode_indexless decodes symbol i from start + 16 i directly
    (no walk, no index); payload moved any number of bytes into its buffer."""
    import torch
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.dev.generate(x.data_ptr(), n, offset=0, kind=0, alpha=1.1, seed=3)
    plan, _, _ = codec.encode(x)
    codec.sync()
    assert int(plan.cb.min_len) == 16 and int(plan.cb.max_len) == 16  # the FIXED16 path is the one tested
    ok, end_ok = _check(codec, x, shift)
    assert ok and end_ok


def test_indexless_fixed16_truncated_and_captured(codec):
    """FIXED16 index-less decode: a payload short of nsym codes reports the end bit past it; the call is
    stream-ordered (captured in a HIP graph and replayed bit-exact)."""
    import torch
    n = (48 << 20) + 2
    nsym = n // 2
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.dev.generate(x.data_ptr(), n, offset=0, kind=0, alpha=1.1, seed=4)
    plan, payload, _ = codec.encode(x)
    codec.sync()
    assert int(plan.cb.min_len) == 16 and int(plan.cb.max_len) == 16
    out = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")
    end = torch.zeros(2, dtype=torch.int64, device="cuda")
    cut = payload.numel() // 2
    codec.dev.decode_indexless(payload.data_ptr(), cut, plan.start_bit, nsym, out.data_ptr(), end.data_ptr())
    codec.sync()
    assert int(end[0].item()) & ((1 << 64) - 1) > 8 * cut
    end.fill_(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=codec.stream):
        codec.dev.decode_indexless(payload.data_ptr(), payload.numel(), plan.start_bit, nsym, out.data_ptr(),
                                   end.data_ptr())
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out[:n], x)
    assert int(end[0].item()) == plan.start_bit + 16 * nsym


def test_indexless_truncated_end_past_payload(codec):
    """A payload cut short of nsym codewords: the end bit lands past the payload (the caller rejects)."""
    import torch
    n = (4 << 20) + 2
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.dev.generate(x.data_ptr(), n, offset=0, kind=1, alpha=1.1, seed=9)
    plan, payload, _ = codec.encode(x)
    cut = payload.numel() // 2
    out = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    end = torch.zeros(2, dtype=torch.int64, device="cuda")
    codec.dev.decode_indexless(payload.data_ptr(), cut, plan.start_bit, n // 2, out.data_ptr(), end.data_ptr())
    codec.sync()
    assert int(end[0].item()) & ((1 << 64) - 1) > 8 * cut  # UINT64_MAX: fewer than nsym codewords


_NO_LEAD = r"""
import sys, numpy as np
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
import oracle_lib, huffman_amd as hz
data = oracle_lib.generate({n}, offset=0, kind=1, seed=12).tobytes()
blob = oracle_lib.encode(data)
assert hz.decode(blob) == data
print("ok")
"""


@pytest.mark.parametrize("lead", ["0", "64"])
def test_indexless_fixups_without_lead_in(built_lib, lead):
    """HZ_SEG_LEAD (test hook) shortens the walk chains' lead-in, so chains start unsynchronised and
    the chain fix-ups (k_chain_fix: heads decoded by k_chain_tail) repair them: the file still decodes
    bit-exact."""
    code = _NO_LEAD.format(root=ROOT, tests=os.path.join(ROOT, "tests"), n=(24 << 20) + 1)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, HZ_SEG_LEAD=lead))
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


def test_indexless_dense_run_past_record_capacity(codec):
    """A long run of the most frequent symbol (~2 bits per codeword against ~12.5 on average) gives
    the chains inside it about 5x more records than their capacity (sized from the average code
    length): the walk stops storing records there and k_chain_tail decodes the rest of each such
    chain serially. The output and the end bit are exact, and nothing is left on the context."""
    import torch
    rng = np.random.default_rng(11)
    nsym = 8 << 20
    sym = rng.integers(1, 32769, nsym).astype("<u2")
    sym[nsym // 3: nsym // 3 + nsym // 5] = 0  # 20 % of the stream, one contiguous run
    x = torch.from_numpy(sym.view(np.uint8).copy()).cuda()
    ok, end_ok = _check(codec, x)
    assert ok and end_ok
    # and again, moved 3 bytes into a buffer
    ok2, end_ok2 = _check(codec, x, shift=3)
    assert ok2 and end_ok2


def test_indexless_skewed_rounds(codec):
    """90 % of the symbols one value (a 1-bit code): ~2 bits per codeword, so the chains are short in
    bits and long in codewords (many decode blocks per chain). The output and end bit are exact."""
    import torch
    rng = np.random.default_rng(5)
    nsym = (6 << 20) + 3
    sym = np.where(rng.random(nsym) < 0.9, 0, rng.integers(1, 301, nsym)).astype("<u2")
    x = torch.from_numpy(sym.view(np.uint8).copy()).cuda()
    ok, end_ok = _check(codec, x)
    assert ok and end_ok


def test_indexless_graph_capture(codec):
    """hz_decode_indexless is stream-ordered (no host synchronisation inside, fix-ups iterated on the
    device): captured into a HIP graph on the context's stream and replayed, it decodes bit-exact. A
    host sync inside the call would break the capture. (Every codebook takes a stream-ordered path:
    test_indexless_dense_codebook_256mib_chain_path, test_indexless_31_bit_codes_chain_path,
    test_indexless_tiny_payload_captured.)"""
    import torch
    from huffman_amd import index_starts
    n = (24 << 20) + 6
    nsym = n // 2
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.dev.generate(x.data_ptr(), n, offset=0, kind=1, alpha=1.1, seed=7)
    plan, payload, index = codec.encode(x)
    codec.sync()
    end_pack = int(index_starts(index.cpu().numpy(), nsym)[-1])
    out = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")
    end = torch.full((2,), -1, dtype=torch.int64, device="cuda")

    def call():
        codec.dev.decode_indexless(payload.data_ptr(), payload.numel(), plan.start_bit, nsym, out.data_ptr(),
                                   end.data_ptr())

    call()  # eager first: the context's scratch is sized outside the capture
    codec.sync()
    assert torch.equal(out[:n], x)
    out.zero_()
    end.fill_(-1)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=codec.stream):
        call()
    torch.cuda.synchronize()
    assert not torch.equal(out[:n], x)  # captured, not run
    for _ in range(2):
        out.zero_()
        end.fill_(-1)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out[:n], x)
        assert int(end[0].item()) == end_pack


def test_indexless_25_bit_codes_stream_ordered(codec):
    """A codebook with 25-bit codes (this 48 MiB Zipf stream) takes the chain path too (global subtables
    of up to 12 bits, a 2^25-byte escape table): captured in a HIP graph and replayed bit-exact."""
    import torch
    from huffman_amd import index_starts
    n = (48 << 20) + 2
    nsym = n // 2
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.dev.generate(x.data_ptr(), n, offset=0, kind=1, alpha=1.1, seed=21)
    plan, payload, index = codec.encode(x)
    codec.sync()
    assert int(plan.cb.max_len) == 25
    end_pack = int(index_starts(index.cpu().numpy(), nsym)[-1])
    out = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")
    end = torch.full((2,), -1, dtype=torch.int64, device="cuda")

    def call():
        codec.dev.decode_indexless(payload.data_ptr(), payload.numel(), plan.start_bit, nsym, out.data_ptr(),
                                   end.data_ptr())

    call()
    codec.sync()
    assert torch.equal(out[:n], x) and int(end[0].item()) == end_pack
    out.zero_()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=codec.stream):
        call()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out[:n], x)


def _dense_stream(nsym, seed):
    """u16 symbols uniform over 3000 values: every code 11 or 12 bits (a DEC_DENSE codebook)."""
    import torch
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    s = torch.randint(0, 3000, (nsym,), dtype=torch.int32, device="cuda", generator=g)
    return (s * 19 + 7).to(torch.int16).view(torch.uint8)


def _fib_stream(seed):
    """32 symbols with Fibonacci counts (1, 1, 2, 3, 5, ..., F(32)): the Huffman tree is a path, so the
    longest codes are 31 bits -- past the chain walker's 25-bit escape table (DEEP escapes through the
    decode LUT) and the pipelined decoder's two table levels (records decoded serially)."""
    c = [1, 1]
    while len(c) < 32:
        c.append(c[-1] + c[-2])
    sym = np.repeat((np.arange(32, dtype=np.uint32) * 2053 % 65536).astype(np.uint16), c)
    np.random.default_rng(seed).shuffle(sym)
    return sym.view(np.uint8)


def _captured_indexless(codec, x, plan, payload, nsym):
    """hz_decode_indexless eager, then captured in a HIP graph and replayed: (eager ok, replay ok, end bit)."""
    import torch
    out = torch.zeros(2 * nsym + 16, dtype=torch.uint8, device="cuda")
    end = torch.full((2,), -1, dtype=torch.int64, device="cuda")

    def call():
        codec.dev.decode_indexless(payload.data_ptr(), payload.numel(), plan.start_bit, nsym, out.data_ptr(),
                                   end.data_ptr())

    call()
    codec.sync()
    eager = bool(torch.equal(out[:2 * nsym], x[:2 * nsym]))
    end_bit = int(end[0].item())
    out.zero_()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=codec.stream):  # a host synchronisation inside would break the capture
        call()
    g.replay()
    torch.cuda.synchronize()
    return eager, bool(torch.equal(out[:2 * nsym], x[:2 * nsym])), end_bit


def test_indexless_dense_codebook_256mib_chain_path(codec):
    """A DEC_DENSE codebook (every code 11-12 bits) at 256 MiB: the chain walk + chain-block decode take
    it through the LUT built beside the DENSE tables -- stream-ordered (captured in a HIP graph and
    replayed bit-exact), end bit equal to pack's."""
    from huffman_amd import codebook_arrays, index_starts
    nsym = 128 << 20
    x = _dense_stream(nsym, 3)
    plan, payload, index = codec.encode(x)
    codec.sync()
    _, ln, _ = codebook_arrays(plan.cb)
    used = ln[ln > 0]
    assert int(used.max()) <= 16 and int(used.max()) - int(used.min()) <= 3  # DEC_DENSE
    end_pack = int(index_starts(index.cpu().numpy(), nsym)[-1])
    eager, replay, end_bit = _captured_indexless(codec, x, plan, payload, nsym)
    assert eager and replay and end_bit == end_pack


@pytest.mark.parametrize("shift", [0, 7])
def test_indexless_31_bit_codes_chain_path(codec, shift):
    """Codes of up to 31 bits (Fibonacci counts): DEEP escapes in the walk and the serial record decoder,
    stream-ordered (graph capture), bit-exact; also moved `shift` bytes into a buffer."""
    import torch
    from huffman_amd import codebook_arrays
    x = torch.from_numpy(_fib_stream(1)).cuda()
    plan, _, _ = codec.encode(x)
    codec.sync()
    _, ln, _ = codebook_arrays(plan.cb)
    assert int(ln.max()) == 31
    ok, end_ok = _check(codec, x, shift)
    assert ok and end_ok
    if shift == 0:
        nsym = x.numel() // 2
        plan, payload, _ = codec.encode(x)
        codec.sync()
        eager, replay, _ = _captured_indexless(codec, x, plan, payload, nsym)
        assert eager and replay


@pytest.mark.parametrize("n", [3, 9, 17])
def test_indexless_tiny_payload_captured(codec, n):
    """Payloads under 16 bytes (too short for the walk): one device thread decodes them serially --
    stream-ordered too (captured in a HIP graph and replayed), bit-exact, end bit equal to pack's."""
    from huffman_amd import index_starts
    import torch
    x = torch.tensor(list(range(7, 7 + n)), dtype=torch.uint8, device="cuda")
    nsym = n // 2
    plan, payload, index = codec.encode(x)
    codec.sync()
    assert payload.numel() < 16 + 16
    end_pack = int(index_starts(index.cpu().numpy(), nsym)[-1])
    pbytes = (plan.start_bit + plan.payload_bits + 7) // 8
    assert pbytes < 16
    payload = payload[:pbytes]
    eager, replay, end_bit = _captured_indexless(codec, x, plan, payload, nsym)
    assert eager and replay and end_bit == end_pack


def _random_stream(rng):
    """A seeded random symbol stream: alphabet size, distribution shape (power law, geometric,
    spiky Dirichlet or flat), symbol values and byte length (odd or even) all drawn at random."""
    U = int(rng.choice([1, 2, 3, 5, 17, 255, 4096, 40000, 65536]))
    kind = int(rng.integers(0, 4))
    r = np.arange(1, U + 1, dtype=np.float64)
    if kind == 0:
        p = r ** -rng.uniform(0.5, 2.5)
    elif kind == 1:
        p = rng.uniform(0.5, 0.999) ** r
    elif kind == 2:
        p = rng.dirichlet(np.full(U, 0.05)) + 1e-12
    else:
        p = np.ones(U)
    p /= p.sum()
    n = int(rng.integers(1, 3 << 20))
    vals = rng.permutation(65536)[:U].astype(np.uint16)
    sym = vals[rng.choice(U, size=(n + 1) // 2, p=p)]
    return sym.astype("<u2").view(np.uint8)[:n].copy(), f"U={U} kind={kind} n={n}"


def test_indexless_random_streams(hz, codec):
    """32 seeded random streams (alphabet sizes 1..65 536, power-law, geometric, spiky and flat
    counts, 1 byte to 3 MiB): the product's file equals the oracle's, the CPU oracle decodes it,
    the file decodes back through hz_decode_host (index-less), the device payload decodes index-less
    from a random byte offset with the end bit of pack's own index, and through that index (k_decode);
    hz_index_build rebuilds that index from the payload alone."""
    import torch
    rng = np.random.default_rng(20261018)
    for case in range(32):
        data, what = _random_stream(rng)
        blob = hz.encode(data.tobytes())
        assert blob == oracle_lib.encode(data), what
        assert oracle_lib.decode(blob) == data.tobytes(), what
        assert hz.decode(blob) == data.tobytes(), what
        if data.size >= 2:
            x = torch.from_numpy(data).cuda()
            ok, end_ok = _check(codec, x, int(rng.integers(0, 48)))
            assert ok and end_ok, what
            # and the headline path: pack's block index, k_decode
            nsym = data.size // 2
            plan, payload, index = codec.encode(x)
            out = torch.empty(2 * nsym + 16, dtype=torch.uint8, device="cuda")
            codec.dev.decode(payload.data_ptr(), payload.numel(), nsym, index.data_ptr(), out.data_ptr())
            codec.sync()
            assert torch.equal(out[:2 * nsym], x[:2 * nsym]), what
            # the self-synchronising index builder rebuilds pack's index from the payload alone
            from huffman_amd import index_bytes
            rebuilt = torch.full_like(index, -1)
            codec.dev.index_build(payload.data_ptr(), payload.numel(), plan.start_bit, nsym, rebuilt.data_ptr())
            codec.sync()
            nb = index_bytes(nsym)
            assert np.array_equal(index.cpu().numpy().view(np.uint8)[:nb], rebuilt.cpu().numpy().view(np.uint8)[:nb]), what


def test_random_streams_through_the_file_streams(hz, tmp_path):
    """12 more seeded random streams through the streaming CLIs' paths: hz_archive_stream in small
    chunks writes the oracle's file, and hz_extract_stream in small payload windows (each window an
    index-less part, the next window's entry from the last) restores the input."""
    rng = np.random.default_rng(7)
    for case in range(12):
        data, what = _random_stream(rng)
        chunk, window = int(rng.integers(1, 64)) * 4096, int(rng.integers(1, 17)) * 4096
        src, arc, out = tmp_path / "in", tmp_path / "in.compressed", tmp_path / "out"
        src.write_bytes(data.tobytes())
        hz.archive_stream(src, arc, chunk_bytes=chunk)
        blob = arc.read_bytes()
        assert blob == oracle_lib.encode(data), what
        hz.extract_stream(arc, out, chunk_bytes=window)
        assert out.read_bytes() == data.tobytes(), what + f" window={window}"


@pytest.mark.parametrize("seed,U,kind", [(1, 3, 0), (2, 17, 1), (3, 300, 2), (4, 65536, 1)])
def test_random_streams_range_plan(codec, seed, U, kind):
    """256 MiB + 1 random streams (the range-plan encoder: histogram snapshots, dot products, pack
    over ranges) with small and large alphabets: the file equals the oracle's, pack's index decodes
    it (k_decode) and the bare payload decodes index-less (chain path) with pack's end bit."""
    import torch
    rng = np.random.default_rng(seed)
    n = (256 << 20) + 1
    r = np.arange(1, U + 1, dtype=np.float64)
    p = [r ** -rng.uniform(0.5, 2.5), rng.uniform(0.5, 0.999) ** r, rng.dirichlet(np.full(U, 0.05)) + 1e-12][kind]
    cdf = np.cumsum(p / p.sum())
    idx = np.minimum(np.searchsorted(cdf, rng.random((n + 1) // 2)), U - 1)
    host = rng.permutation(65536)[:U].astype("<u2")[idx].view(np.uint8)[:n].copy()
    x = torch.from_numpy(host).cuda()
    plan, payload, index = codec.encode(x)
    codec.sync()
    assert codec.file_image(plan, payload) == oracle_lib.encode(host)
    nsym = n // 2
    out = torch.empty(2 * nsym + 16, dtype=torch.uint8, device="cuda")
    codec.decode(payload, nsym, index, out)
    codec.sync()
    assert torch.equal(out[:2 * nsym], x[:2 * nsym])
    ok, end_ok = _check(codec, x, 3)
    assert ok and end_ok


def test_indexless_random_streams_captured_first(codec):
    """Six seeded random streams whose first index-less decode after a table upload is captured in a
    HIP graph: the capture holds the copy of the index-less tables (staged by the upload, copied by
    their first reader), the replay decodes bit-exact, and an eager call afterwards copies them again
    and decodes bit-exact too. (An eager decode first sizes the context's scratch: growing it
    synchronises, which a capture does not allow -- include/huffman_amd.h.)"""
    import torch
    rng = np.random.default_rng(31)
    done = 0
    while done < 6:
        data, what = _random_stream(rng)
        if data.size < 64:
            continue
        nsym = data.size // 2
        x = torch.from_numpy(data).cuda()
        plan, payload, _ = codec.encode(x)
        codec.sync()
        out = torch.zeros(2 * nsym + 16, dtype=torch.uint8, device="cuda")
        end = torch.full((2,), -1, dtype=torch.int64, device="cuda")

        def call():
            codec.dev.decode_indexless(payload.data_ptr(), payload.numel(), plan.start_bit, nsym, out.data_ptr(),
                                       end.data_ptr())

        call()  # sizes the scratch
        codec.upload_decode(plan)  # the index-less tables staged again, not yet copied
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=codec.stream):
            call()
        out.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out[:2 * nsym], x[:2 * nsym]), what + " (replay)"
        out.zero_()
        torch.cuda.synchronize()
        call()
        codec.sync()
        assert torch.equal(out[:2 * nsym], x[:2 * nsym]), what + " (eager after the capture)"
        done += 1


def test_indexless_parts_from_slices(codec):
    """The split API in one context, part after part: eight seeded random streams cut at 1-4 random
    payload bits; each part is scanned from a 16-byte aligned slice holding only its lead-in, its bits
    and max_len bits after (payload_bit_base), from its true entry (the previous part's exit) or from
    its walked entry and then refixed to the true one, and decoded at the sum of the codewords before
    it. The parts together restore the stream bit-exactly."""
    import torch
    from huffman_amd.dist import UNKNOWN_ENTRY
    rng = np.random.default_rng(41)
    summ = torch.zeros(4, dtype=torch.int64, device="cuda")
    done = 0
    while done < 8:
        data, what = _random_stream(rng)
        if data.size < 4096:
            continue
        nsym = data.size // 2
        x = torch.from_numpy(data).cuda()
        plan, payload, _ = codec.encode(x)
        codec.sync()
        start, P, max_len = int(plan.start_bit), int(plan.payload_bits), int(plan.cb.max_len)
        k = int(rng.integers(2, 6))
        cuts = sorted(set(int(v) for v in rng.integers(1, P, k - 1)))
        bounds = [0] + cuts + [P]
        out = torch.zeros(2 * nsym + 16, dtype=torch.uint8, device="cuda")

        def read():
            codec.sync()
            return [int(v) & ((1 << 64) - 1) for v in summ[:3].cpu().tolist()]

        entry, first = start, 0
        for pb, pe in zip(bounds, bounds[1:]):
            lo_bit = start + pb - min(1024, pb)
            hi_bit = start + pe + max_len
            b0 = lo_bit // 8 // 16 * 16
            b1 = min(payload.numel(), ((hi_bit + 7) // 8 + 16 + 15) // 16 * 16)
            known = bool(rng.random() < 0.5) or pb == 0
            codec.dev.indexless_scan(payload.data_ptr() + b0, b1 - b0, start, pb, pe,
                                     entry if known else UNKNOWN_ENTRY, summ.data_ptr(), nsym=nsym,
                                     payload_bit_base=8 * b0)
            cnt, xit, ent = read()
            if ent != entry:
                codec.dev.indexless_refix(entry, summ.data_ptr())
                cnt, xit, ent = read()
            assert ent == entry, what
            take = min(cnt, nsym - first)
            tmp = torch.zeros(2 * take + 16, dtype=torch.uint8, device="cuda")
            codec.dev.indexless_decode(take, tmp.data_ptr())
            codec.sync()
            out[2 * first:2 * (first + take)] = tmp[:2 * take]
            first += cnt
            entry = xit
        codec.sync()
        assert first == nsym, what
        assert torch.equal(out[:2 * nsym], x[:2 * nsym]), what
        done += 1


def test_indexless_parts_from_slices_fixed16(codec):
    """The split API on a FIXED16 stream (every code 16 bits, 64 MiB of uniform bytes): parts at
    random bits, each from its own slice, entries arithmetic (start + 16 i), walked or given."""
    import torch
    from huffman_amd.dist import UNKNOWN_ENTRY
    n = (64 << 20) + 2
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.dev.generate(x.data_ptr(), n, offset=0, kind=0, alpha=1.1, seed=3)
    plan, payload, _ = codec.encode(x)
    codec.sync()
    assert int(plan.cb.min_len) == 16 and int(plan.cb.max_len) == 16
    nsym = n // 2
    start, P = int(plan.start_bit), int(plan.payload_bits)
    rng = np.random.default_rng(43)
    bounds = [0] + sorted(set(int(v) for v in rng.integers(1, P, 4))) + [P]
    summ = torch.zeros(4, dtype=torch.int64, device="cuda")
    out = torch.zeros(2 * nsym + 16, dtype=torch.uint8, device="cuda")
    entry, first = start, 0
    for i, (pb, pe) in enumerate(zip(bounds, bounds[1:])):
        b0 = (start + pb - min(1024, pb)) // 8 // 16 * 16
        b1 = min(payload.numel(), ((start + pe + 16 + 7) // 8 + 16 + 15) // 16 * 16)
        codec.dev.indexless_scan(payload.data_ptr() + b0, b1 - b0, start, pb, pe,
                                 entry if i % 2 == 0 else UNKNOWN_ENTRY, summ.data_ptr(), nsym=nsym,
                                 payload_bit_base=8 * b0)
        codec.sync()
        cnt, xit, ent = [int(v) & ((1 << 64) - 1) for v in summ[:3].cpu().tolist()]
        assert ent == entry
        take = min(cnt, nsym - first)
        tmp = torch.zeros(2 * take + 16, dtype=torch.uint8, device="cuda")
        codec.dev.indexless_decode(take, tmp.data_ptr())
        codec.sync()
        out[2 * first:2 * (first + take)] = tmp[:2 * take]
        first += cnt
        entry = xit
    assert first == nsym
    assert torch.equal(out[:2 * nsym], x[:2 * nsym])
