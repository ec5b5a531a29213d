"""GPU parity: the gfx950 path against the CPU oracle (bit-exact), the golden
fixtures, the reference decoder, and size-independent properties at scale.

Tolerance: none -- every check is bit-exact (integer/bit work)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
INPUTS = ["romeo.txt", "synth_zipf_65537.bin", "synth_unif_65536.bin", "synth_zipf_4099.bin"]
JPEG = "pexels-vlad-alexandru-popa-1402787.jpg"


def read(name):
    with open(os.path.join(GOLD, name), "rb") as f:
        return f.read()


@pytest.fixture(scope="module")
def hz(built_lib):
    import huffman_amd
    return huffman_amd


@pytest.fixture(scope="module")
def codec(built_lib):
    import torch
    from huffman_amd.pipeline import StreamCodec
    return StreamCodec(0)


# ---- whole-file parity ---------------------------------------------------------
@pytest.mark.parametrize("name", INPUTS + [JPEG])
def test_encode_matches_oracle(hz, name):
    data = read(name)
    got = hz.encode(data)
    assert got == oracle_lib.encode(data)
    if name in INPUTS:
        assert got == read(name + ".compressed")


@pytest.mark.parametrize("name", INPUTS)
def test_decode_golden_and_baseline_files(hz, name):
    data = read(name)
    assert hz.decode(read(name + ".compressed")) == data
    assert hz.decode(read(name + ".baseline.compressed")) == data   # reference baseline encoder's bytes


def test_decode_baseline_jpeg(hz, tmp_path):
    exe = oracle_lib.ref_binary("archive_baseline")
    if exe is None:
        pytest.skip("reference baseline encoder not built")
    (tmp_path / "in").write_bytes(read(JPEG))
    subprocess.run([exe, "in"], cwd=tmp_path, check=True, capture_output=True, timeout=300)
    assert hz.decode((tmp_path / "in.compressed").read_bytes()) == read(JPEG)


def _zipf_bytes(n, seed):
    return oracle_lib.generate(n, offset=seed * 1000003, kind=1, seed=seed).tobytes()


EDGE_SIZES = [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 33, 63, 64, 65, 127, 1023, 1024, 1025, 4095, 4096, 4097,
              8191, 8192, 8193, 2 * 4096 * 16 - 2, 2 * 4096 * 16, 2 * 4096 * 16 + 3, 1000001]


@pytest.mark.parametrize("n", EDGE_SIZES)
def test_edge_sizes(hz, n):
    data = _zipf_bytes(n, n)
    blob = hz.encode(data)
    assert blob == oracle_lib.encode(data)
    assert hz.decode(blob) == data


@pytest.mark.parametrize("data", [b"abab" * 100, b"ab", b"\x00\x00" * 5000 + b"\x01", b"\xff" * 3,
                                  bytes(range(256)) * 512, b"xy" * 3 + b"z"])
def test_degenerate_alphabets(hz, data):
    blob = hz.encode(data)
    assert blob == oracle_lib.encode(data)
    assert hz.decode(blob) == data


def _fib_input(depth, seed=0):
    """Symbols with Fibonacci counts: code lengths grow to ~depth bits."""
    fib = [1, 1]
    while len(fib) < depth + 1:
        fib.append(fib[-1] + fib[-2])
    sym = np.repeat(np.arange(len(fib), dtype=np.uint16) * 257 + 3, fib)
    np.random.default_rng(seed).shuffle(sym)
    return sym.astype("<u2").tobytes()


@pytest.mark.parametrize("depth,mode", [(20, "HOT"), (28, "WIDE"), (34, "WIDE>32")])
def test_long_codes_wide_tables(hz, depth, mode):
    data = _fib_input(depth)
    h = oracle_lib.hist16(data)
    _, ln, _ = oracle_lib.codebook(h)
    assert ln.max() == depth
    blob = hz.encode(data)
    assert blob == oracle_lib.encode(data)
    assert hz.decode(blob) == data


def _lut_global_entries(ln, code, k1, lvl):
    """Entries of the decoder's global LUT levels (hz_codebook.cpp fill_level) at `lvl` index bits per level."""
    syms = np.nonzero(ln)[0]

    def level(sel, depth, nb):
        # codes of `sel` with their first `depth` bits consumed; this table has nb index bits
        rem = ln[sel].astype(np.int64) - depth
        deep = sel[rem > nb]
        if deep.size == 0:
            return 0
        r = ln[deep].astype(np.int64) - depth
        q = (code[deep] >> (r - nb).astype(np.uint64)) & np.uint64((1 << nb) - 1)
        total = 0
        for qv in np.unique(q):
            grp = deep[q == qv]
            nb2 = int(min(int((ln[grp].astype(np.int64) - depth - nb).max()), lvl))
            total += (1 << nb2) + level(grp, depth + nb, nb2)
        return total
    return level(syms, 0, k1)


def test_lut_narrow_global_levels(hz):
    """a codebook whose 9-bit global LUT levels would exceed kLutMaxL2 (2^21 - 65 536
    entries) is built with narrower levels (hz_codebook.cpp build_dec_lut); pack, decode and the
    index builder stay bit-exact on it. The prefix code (not a Huffman code of the input: the tables
    take any prefix code) is 4096 caterpillars under 12-bit prefixes: lengths 13 .. 22, so every
    level-1 (13-bit) prefix ending in 0 has a 9-bit-deep subtree."""
    import ctypes
    import torch
    from huffman_amd import index_bytes
    from huffman_amd._lib import Codebook
    from huffman_amd.codec import Device
    ln = np.zeros(65536, np.uint8)
    code = np.zeros(65536, np.uint64)
    for g in range(4096):
        for j in range(11):
            s = g * 11 + j
            L = 13 + j if j < 10 else 22               # prefix g, then 0^j 1 (j < 10) or 0^10
            ln[s] = L
            code[s] = (g << (L - 12)) | (1 if j < 10 else 0)
    assert _lut_global_entries(ln, code, 13, 9) > (1 << 21) - 65536     # 9-bit levels do not fit
    assert _lut_global_entries(ln, code, 13, 8) <= (1 << 21) - 65536
    cb = Codebook()
    syms = np.nonzero(ln)[0]
    cb.nsym, cb.max_len, cb.min_len = syms.size, int(ln.max()), int(ln[syms].min())
    np.ctypeslib.as_array(cb.order)[:syms.size] = syms
    np.ctypeslib.as_array(cb.len)[:] = ln
    np.ctypeslib.as_array(cb.code)[:] = code
    rng = np.random.default_rng(8)
    sym = rng.choice(syms, size=(3 << 20) + 777).astype("<u2")
    host = sym.view(np.uint8)
    nsym = sym.size
    dev = Device()
    dev.upload(cb)
    x = torch.from_numpy(host).cuda()
    bits = int(ln[sym].astype(np.uint64).sum())
    cap = (bits + 5) // 8 + 64
    pay = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    idx = torch.full((index_bytes(nsym) // 8 + 4,), -1, dtype=torch.int64, device="cuda")
    dev.pack(x.data_ptr(), x.numel(), 5, 0, pay.data_ptr(), cap, idx.data_ptr())
    out = torch.empty(x.numel() + 16, dtype=torch.uint8, device="cuda")
    dev.decode(pay.data_ptr(), cap, nsym, idx.data_ptr(), out.data_ptr())
    rebuilt = torch.full_like(idx, -1)
    dev.index_build(pay.data_ptr(), cap, 5, nsym, rebuilt.data_ptr())
    dev.sync()
    assert torch.equal(out[:x.numel()], x)
    nb = index_bytes(nsym)
    assert np.array_equal(idx.cpu().numpy().view(np.uint8)[:nb], rebuilt.cpu().numpy().view(np.uint8)[:nb])
    ref = oracle_lib.pack_range(host, 0, nsym, ln, code, 5, cap)
    assert np.array_equal(pay.cpu().numpy()[1:(5 + bits) // 8], ref[1:(5 + bits) // 8])


def test_lut_leaf_symbols_with_high_bits(hz, codec):
    """the pipelined decoder reads every LUT entry as a link, leaves included.
    Symbols whose bits 9..5 are 30/31 (0x03C0 .. 0x03FF, the old leaf layout's widest bit-field)
    given long all-ones codes decode bit-exact (the leaf layout keeps such reads past the table)."""
    import torch
    rng = np.random.default_rng(31)
    hot = np.arange(0x03C0, 0x0400, dtype=np.uint16)                 # the rare, long-coded symbols
    common = rng.integers(0x1000, 0x1400, size=1 << 21).astype(np.uint16)
    rare = np.repeat(hot, np.arange(1, hot.size + 1))                 # ragged small counts: long codes
    sym = np.concatenate([common, rare])
    rng.shuffle(sym)
    host = sym.astype("<u2").view(np.uint8)
    x = torch.from_numpy(host).cuda()
    plan, payload, index = codec.encode(x)
    n = x.numel()
    from huffman_amd import codebook_arrays
    _, ln, _ = codebook_arrays(plan.cb)
    assert int(ln[hot].max()) >= 18
    out = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    codec.decode(payload, n // 2, index, out)
    codec.sync()
    assert torch.equal(out[:n], x)


def test_uniform_dense_tables(hz):
    data = oracle_lib.generate(1 << 22, kind=0, seed=3).tobytes()   # all 65536 symbols, 16-bit codes
    blob = hz.encode(data)
    assert blob == oracle_lib.encode(data)
    assert hz.decode(blob) == data


# ---- CLI drop-in -------------------------------------------------------------------
def test_cli_archive_extract(hz, tmp_path):
    (tmp_path / "romeo.txt").write_bytes(read("romeo.txt"))
    r = subprocess.run([os.path.join(hz.BIN_DIR, "archive"), "romeo.txt"], cwd=tmp_path, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Compression is complete" in r.stdout and "Unique symbols count: 1268" in r.stdout
    # the reference's stage timers (Compressor.cu:399, 593; gpuHuffmanConstruction.h:780-782)
    for line in ("Histograming took ", "construction time: ", "Encoding took "):
        assert line in r.stdout, r.stdout
    assert (tmp_path / "romeo.txt.compressed").read_bytes() == read("romeo.txt.compressed")
    r = subprocess.run([os.path.join(hz.BIN_DIR, "extract"), "romeo.txt.compressed"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "Decompression is complete" in r.stdout
    assert (tmp_path / "DECOMPRESSED_FILE").read_bytes() == read("romeo.txt")
    # second extract picks DECOMPRESSED_FILE(1) (Decompressor.cu:185-219)
    subprocess.run([os.path.join(hz.BIN_DIR, "extract"), "romeo.txt.compressed"], cwd=tmp_path, check=True,
                   capture_output=True, timeout=300)
    assert (tmp_path / "DECOMPRESSED_FILE(1)").read_bytes() == read("romeo.txt")
    ref = oracle_lib.ref_binary("extract")
    if ref:
        d = tmp_path / "ref"
        d.mkdir()
        (d / "x.compressed").write_bytes((tmp_path / "romeo.txt.compressed").read_bytes())
        subprocess.run([ref, "x.compressed"], cwd=d, check=True, capture_output=True, timeout=300)
        assert (d / "DECOMPRESSED_FILE").read_bytes() == read("romeo.txt")


def _skewed_bytes(n, seed):
    """One frequent symbol everywhere except a run of rare symbols (long codes):
    the stream's largest block is far above the average block (decode slots
    sized from max_bits, the two-block decoder's one-block fallback)."""
    rng = np.random.default_rng(seed)
    sym = np.zeros(n // 2, dtype=np.uint16)
    sym[4096:8192] = rng.integers(1, 65536, 4096)
    sym[8192:] = np.where(rng.random(n // 2 - 8192) < 0.02, rng.integers(1, 200, n // 2 - 8192), 0)
    return sym.astype("<u2").tobytes()


@pytest.mark.parametrize("pipe", ["0", "1", "2"])
@pytest.mark.parametrize("kind", ["zipf", "skewed"])
def test_decode_variants_cli(hz, tmp_path, pipe, kind):
    """Every LUT decoder (HZ_DEC_PIPE: 0 plain, 1 pipelined, 2 two blocks per wave) through `extract`."""
    data = _zipf_bytes((6 << 20) + 1, 11) if kind == "zipf" else _skewed_bytes(6 << 20, 5)
    blob = hz.encode(data)
    assert blob == oracle_lib.encode(data)
    (tmp_path / "x.compressed").write_bytes(blob)
    env = dict(os.environ, HZ_DEC_PIPE=pipe)
    r = subprocess.run([os.path.join(hz.BIN_DIR, "extract"), "x.compressed"], cwd=tmp_path, capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "DECOMPRESSED_FILE").read_bytes() == data


@pytest.mark.parametrize("name,chunk", [("romeo.txt", 4096), ("romeo.txt", 64), ("zipf", 1 << 20)])
def test_cli_archive_resident(hz, tmp_path, name, chunk):
    """`archive` keeps a file that fits on the device resident between its two passes
    (one read of the file, one pack launch, the payload leaving in `chunk`-byte pieces
    through parallel positional writes): the file equals the oracle's / the golden
    archive, and `extract` (double-buffered parallel writes) restores the input."""
    data = read(name) if name != "zipf" else _zipf_bytes((20 << 20) + 1, 3)
    (tmp_path / "in.bin").write_bytes(data)
    env = dict(os.environ, HZ_ARCHIVE_CHUNK=str(chunk), HZ_TIMING="1")
    r = subprocess.run([os.path.join(hz.BIN_DIR, "archive"), "in.bin"], cwd=tmp_path, capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    import json
    stage = json.loads([l for l in r.stderr.splitlines() if l.startswith("{")][-1])
    blob = (tmp_path / "in.bin.compressed").read_bytes()
    assert stage["bytes_in"] == len(data) and stage["bytes_out"] == len(blob)  # the file was read once
    assert blob == (read(name + ".compressed") if name != "zipf" else oracle_lib.encode(data))
    r = subprocess.run([os.path.join(hz.BIN_DIR, "extract"), "in.bin.compressed"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "DECOMPRESSED_FILE").read_bytes() == data


@pytest.mark.parametrize("name", ["romeo.txt", "zipf", "odd"])
@pytest.mark.parametrize("host", [False, True])
def test_cli_device_and_host_codebook_paths(hz, tmp_path, name, host):
    """`archive` builds the codebook and header on the device (k_cb_*, k_hw_*) unless
    HZ_HOST_CODEBOOK=1; `extract` parses the header on the device (k_hdr_*) unless
    HZ_HOST_HEADER=1, here with a 1 MiB payload window: both paths write the oracle's
    archive and restore the input."""
    data = {"romeo.txt": read("romeo.txt"), "zipf": _zipf_bytes((12 << 20) + 1, 21),
            "odd": _skewed_bytes(6 << 20, 2) + b"\x07"}[name]
    (tmp_path / "in.bin").write_bytes(data)
    env = dict(os.environ, HZ_EXTRACT_WINDOW=str(1 << 20))
    if host:
        env.update(HZ_HOST_CODEBOOK="1", HZ_HOST_HEADER="1")
    r = subprocess.run([os.path.join(hz.BIN_DIR, "archive"), "in.bin"], cwd=tmp_path, capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "in.bin.compressed").read_bytes() == oracle_lib.encode(data)
    r = subprocess.run([os.path.join(hz.BIN_DIR, "extract"), "in.bin.compressed"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "DECOMPRESSED_FILE").read_bytes() == data


def test_cli_exit_codes(hz, tmp_path):
    a = os.path.join(hz.BIN_DIR, "archive")
    e = os.path.join(hz.BIN_DIR, "extract")
    assert subprocess.run([a], cwd=tmp_path, capture_output=True).returncode == 0
    assert subprocess.run([a, "missing"], cwd=tmp_path, capture_output=True).returncode == 0
    assert subprocess.run([e], cwd=tmp_path, capture_output=True).returncode == 1
    assert subprocess.run([e, "missing"], cwd=tmp_path, capture_output=True).returncode == 0


# ---- device pipeline at scale --------------------------------------------------------
# ---- streaming archive (bounded memory) ---------------------------
@pytest.mark.parametrize("n,chunk", [((5 << 20) + 3, 1 << 20), (10001, 64), (4096 * 3, 4096), (4096 * 3 + 1, 4096),
                                     (0, 4096), (1, 4096), (3, 64), (1 << 20, 1 << 20), ((1 << 20) + 2, 1 << 20)])
def test_archive_stream_matches_whole_buffer(hz, tmp_path, n, chunk):
    data = _zipf_bytes(n, n + 7)
    src = tmp_path / "in.bin"
    src.write_bytes(data)
    out = hz.archive_stream(src, tmp_path / "in.bin.compressed", chunk_bytes=chunk)
    t = hz.stream_timing()
    blob = open(out, "rb").read()
    assert blob == oracle_lib.encode(data)
    assert hz.decode(blob) == data
    # stage split: two passes over the input (the second without the odd last byte), the archive written once
    assert t["bytes_in"] == n + (n - n % 2) and t["bytes_out"] == len(blob)
    assert t["total_ms"] > 0 and min(t[k] for k in ("fread_ms", "fwrite_ms", "h2d_ms", "kernel_ms", "d2h_ms")) >= 0


@pytest.mark.parametrize("kind", ["fib28", "uniform"])
def test_archive_stream_table_modes(hz, tmp_path, kind):
    if kind == "fib28":
        data = _fib_input(28)                                  # WIDE tables, codes up to 28 bits
    else:
        data = np.random.default_rng(5).integers(0, 256, 1 << 21, dtype=np.uint8).tobytes()  # FIXED16
    src = tmp_path / "in.bin"
    src.write_bytes(data)
    blob = open(hz.archive_stream(src, tmp_path / "o", chunk_bytes=4096 * 5 + 16), "rb").read()
    assert blob == oracle_lib.encode(data)


def _hetero_bytes(n, seed=3):
    """Incompressible first half, one repeated symbol after: the file's mean
    code length underestimates the first half (the window retry path)."""
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, n // 2, dtype=np.uint8)
    return (a.tobytes() + b"\x07\x01" * ((n - n // 2) // 2) + b"\x05" * (n % 2))


@pytest.mark.parametrize("kind,n,window", [("zipf", (5 << 20) + 3, 4096), ("zipf", (5 << 20) + 3, 1 << 16),
                                           ("zipf", 10001, 4096), ("zipf", 0, 4096), ("zipf", 1, 4096),
                                           ("zipf", 3, 4096), ("hetero", 3 << 20, 1 << 16),
                                           ("hetero", (1 << 20) + 1, 5000), ("fib28", 0, 4096),
                                           ("uniform", 1 << 21, 1 << 15)])
def test_extract_stream_roundtrip(hz, tmp_path, kind, n, window):
    if kind == "zipf":
        data = _zipf_bytes(n, n + 11)
    elif kind == "hetero":
        data = _hetero_bytes(n)
    elif kind == "fib28":
        data = _fib_input(28)
    else:
        data = np.random.default_rng(9).integers(0, 256, n, dtype=np.uint8).tobytes()
    blob = oracle_lib.encode(data)
    (tmp_path / "in.compressed").write_bytes(blob)
    out = hz.extract_stream(tmp_path / "in.compressed", tmp_path / "out", chunk_bytes=window)
    t = hz.stream_timing()
    assert open(out, "rb").read() == data
    assert t["bytes_out"] == len(data) and t["total_ms"] > 0
    assert min(t[k] for k in ("fread_ms", "fwrite_ms", "h2d_ms", "kernel_ms", "d2h_ms")) >= 0


@pytest.mark.parametrize("name", INPUTS)
def test_extract_stream_baseline_files(hz, tmp_path, name):
    out = hz.extract_stream(os.path.join(GOLD, name + ".baseline.compressed"), tmp_path / "out", chunk_bytes=4096)
    assert open(out, "rb").read() == read(name)


def test_generator_matches_oracle(codec):
    import torch
    n = 1 << 24
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    for kind in (0, 1):
        codec.dev.generate(x.data_ptr(), n, offset=123456789, kind=kind, alpha=1.1, seed=42)
        torch.cuda.synchronize()
        host = x.cpu().numpy()
        for off in (0, 777777, n - 4096):
            assert np.array_equal(host[off:off + 4096],
                                  oracle_lib.generate(4096, offset=123456789 + off, kind=kind, seed=42))


@pytest.mark.parametrize("kind", [1, 0])
def test_pipeline_256mib_matches_oracle(codec, kind):
    import torch
    n = (256 << 20) + 1  # odd: last byte rides in the header
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.dev.generate(x.data_ptr(), n, offset=0, kind=kind, alpha=1.1, seed=42)
    plan, payload, index = codec.encode(x)
    codec.sync()
    host = x.cpu().numpy()
    h_dev = codec.hist.cpu().numpy().view(np.uint64)
    assert np.array_equal(h_dev, oracle_lib.hist16(host))
    order, ln, code = oracle_lib.codebook(h_dev)
    # payload slices against the oracle's packer (bit-exact, block boundaries included)
    pay = payload.cpu().numpy()
    nsym = n // 2
    for sym0, cnt in [(0, 5000), (2048 * 1000 - 7, 9000), (nsym - 6000, 6000)]:
        # start bit of sym0 from the oracle's lengths
        pre = int(np.sum(ln[(host[0:2 * sym0:2].astype(np.uint32) | (host[1:2 * sym0:2].astype(np.uint32) << 8))]
                         .astype(np.uint64)))
        bit0 = plan.start_bit + pre
        nbits = int(np.sum(ln[(host[2 * sym0:2 * (sym0 + cnt):2].astype(np.uint32)
                               | (host[2 * sym0 + 1:2 * (sym0 + cnt):2].astype(np.uint32) << 8))].astype(np.uint64)))
        b0, b1 = bit0 // 8 + 1, (bit0 + nbits) // 8   # whole bytes inside the slice
        ref = oracle_lib.pack_range(host, sym0, cnt, ln, code, bit0 - 8 * (bit0 // 8), (nbits + 40) // 8 + 2)
        assert np.array_equal(pay[b0:b1], ref[b0 - bit0 // 8:b1 - bit0 // 8])
    # whole file == oracle whole-file encoder
    assert codec.file_image(plan, payload) == oracle_lib.encode(host)
    # decode on the device
    out = torch.empty(2 * nsym + 16, dtype=torch.uint8, device="cuda")
    codec.decode(payload, nsym, index, out)
    codec.sync()
    assert torch.equal(out[:2 * nsym], x[:2 * nsym])


@pytest.mark.parametrize("kind,n", [(1, (64 << 20) + 2), (0, (64 << 20) + 1), (1, 4097 * 2 + 1), (1, 3)])
def test_index_build_equals_pack_index(codec, kind, n):
    """The self-synchronising index builder (for index-less reference files)
    reproduces, from the payload alone, exactly the block index hz_pack wrote."""
    import torch
    from huffman_amd import index_bytes
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.dev.generate(x.data_ptr(), n, offset=0, kind=kind, alpha=1.1, seed=5)
    plan, payload, index = codec.encode(x)
    rebuilt = torch.full_like(index, -1)
    codec.dev.index_build(payload.data_ptr(), payload.numel(), plan.start_bit, n // 2, rebuilt.data_ptr())
    codec.sync()
    nb = index_bytes(n // 2)
    a = index.cpu().numpy().view(np.uint8)[:nb]
    b = rebuilt.cpu().numpy().view(np.uint8)[:nb]
    assert np.array_equal(a, b)


@pytest.mark.parametrize("shift", [5000, 12345, 8192 * 3 + 1])
def test_index_rebased_with_moved_payload(codec, shift):
    """Index format 2 (include/huffman_amd.h): a payload handed to hz_decode
    `shift` bytes further into its buffer decodes with the index rebased -- start[]
    and sub[] moved together by 8*shift bits (sub[] mod 2^16), max_bits kept.
    The shifts are not multiples of 8 KiB, so sub[] changes."""
    import torch
    n = (8 << 20) + 2
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.dev.generate(x.data_ptr(), n, offset=0, kind=1, alpha=1.1, seed=11)
    plan, payload, index = codec.encode(x)
    codec.sync()
    nsym = n // 2
    nb = (nsym + 2047) // 2048
    moved = torch.zeros(payload.numel() + shift + 64, dtype=torch.uint8, device="cuda")
    moved[shift:shift + payload.numel()] = payload
    idx = index.cpu().numpy().copy()
    starts = idx[:nb + 1].view(np.uint64)
    starts += np.uint64(8 * shift)
    sub = idx[nb + 2:].view(np.uint16)
    sub += np.uint16((8 * shift) & 0xffff)
    rebased = torch.from_numpy(idx).cuda()
    out = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    codec.decode(moved, nsym, rebased, out)
    codec.sync()
    assert torch.equal(out[:n], x)


def _shape_stream(name):
    """Host streams whose codebooks take the index builder's different table
    shapes: lengths <= 16 (walker, no escape table), 17..22 (walker with the
    escape table), > 22 (segment walkers), equal lengths (DENSE decode mode)."""
    rng = np.random.default_rng(17)
    if name == "dense8":   # 256 symbols, every code 8 bits
        return rng.integers(0, 16, size=(3 << 20) + 1, dtype=np.uint8)
    if name == "short":    # ~600 symbols, geometric-ish weights: max length <= 16
        sym = np.minimum(rng.geometric(0.01, size=(3 << 20) // 2), 599).astype(np.uint16)
        return sym.view(np.uint8)
    if name == "long24":   # weights 2^i: codes up to 24 bits (above the walker's 22)
        counts = [1 << i for i in range(23)] + [1]
        sym = np.repeat(np.arange(24, dtype=np.uint16) * 257, counts)
        rng.shuffle(sym)
        return sym.view(np.uint8)
    if name == "mid20":    # Zipf-like over 4096 symbols: codes into the escape range
        r = np.arange(1, 4097, dtype=np.float64)
        p = r ** -1.3
        p /= p.sum()
        sym = rng.choice(4096, size=(6 << 20) // 2, p=p).astype(np.uint16) * 13
        return sym.view(np.uint8)
    raise ValueError(name)


@pytest.mark.parametrize("name", ["dense8", "short", "mid20", "long24"])
def test_index_build_table_shapes(codec, name):
    """hz_index_build == the index hz_pack wrote, for codebooks of every table
    shape the index builder distinguishes (walker with and without escapes,
    DENSE decode tables, the segment walkers past 22-bit codes)."""
    import torch
    from huffman_amd import index_bytes, codebook_arrays
    host = _shape_stream(name)
    x = torch.from_numpy(host).cuda()
    n = x.numel()
    plan, payload, index = codec.encode(x)
    _, ln, _ = codebook_arrays(plan.cb)
    mx = int(ln.max())
    assert {"dense8": mx == 8, "short": mx <= 16, "mid20": 16 < mx <= 22, "long24": mx > 22}[name], mx
    rebuilt = torch.full_like(index, -1)
    codec.dev.index_build(payload.data_ptr(), payload.numel(), plan.start_bit, n // 2, rebuilt.data_ptr())
    codec.sync()
    nb = index_bytes(n // 2)
    assert np.array_equal(index.cpu().numpy().view(np.uint8)[:nb], rebuilt.cpu().numpy().view(np.uint8)[:nb])
    out = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    codec.decode(payload, n // 2, rebuilt, out)
    codec.sync()
    assert torch.equal(out[:n - (n & 1)], x[:n - (n & 1)])


def test_pipeline_4gib_roundtrip_properties(codec):
    """Above the reference's 4 GiB int-index limit: u64 counts, round trip,
    total bits == sum(hist * len), index monotone."""
    import torch
    n = (4 << 30) + 6
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.dev.generate(x.data_ptr(), n, offset=0, kind=1, alpha=1.1, seed=7)
    plan, payload, index = codec.encode(x)
    codec.sync()
    h = codec.hist.cpu().numpy().view(np.uint64)
    assert int(h.sum()) == n // 2
    from huffman_amd import codebook_arrays
    _, ln, _ = codebook_arrays(plan.cb)
    assert plan.payload_bits == int(np.sum(h * ln.astype(np.uint64)))
    from huffman_amd import index_starts
    idx = index_starts(index.cpu().numpy(), n // 2)
    assert idx[0] == plan.start_bit and np.all(np.diff(idx) > 0)
    assert int(idx[-1]) == plan.start_bit + plan.payload_bits
    out = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    codec.decode(payload, n // 2, index, out)
    codec.sync()
    assert torch.equal(out[:n], x[:n])
    del x, out, payload
    torch.cuda.empty_cache()


# ---- malformed input: clean errors, no hang ------------------------------------------
def _set_n(blob, n):
    """Rewrite the header's 64-bit N (8 LE bytes, each MSB-first, starting at the
    header's bit position) of an oracle file: re-encode with the same codebook."""
    import huffman_amd
    cb, info = huffman_amd.parse_header(blob)
    head, pbits, pend = huffman_amd.write_header(cb, n, info.last_byte)
    return head + bytes([(pend & (0xff << (8 - pbits))) | (blob[len(head)] & (0xff >> pbits))]) \
        + blob[len(head) + 1:] if pbits else head + blob[len(head):]


def _extract_rc(hz, tmp_path, blob):
    d = tmp_path / "x"
    d.mkdir(exist_ok=True)
    (d / "bad.compressed").write_bytes(blob)
    r = subprocess.run([os.path.join(hz.BIN_DIR, "extract"), "bad.compressed"], cwd=d, capture_output=True,
                       text=True, timeout=120)
    return r.returncode, (d / "DECOMPRESSED_FILE")


@pytest.mark.parametrize("cut", [1, 7, 1000, "half"])
def test_truncated_file_is_rejected(hz, tmp_path, cut):
    data = _zipf_bytes((1 << 20) + 1, 3)
    blob = oracle_lib.encode(data)
    bad = blob[:len(blob) // 2] if cut == "half" else blob[:-cut]
    with pytest.raises(hz.HZError):
        hz.decode(bad)
    rc, out = _extract_rc(hz, tmp_path, bad)
    assert rc == 2 and not out.exists()   # codec failure: exit 2, no partial output left behind


def test_header_n_larger_than_payload_is_rejected(hz, tmp_path):
    data = _zipf_bytes(1 << 20, 4)
    blob = oracle_lib.encode(data)
    bad = _set_n(blob, 1 << 40)
    with pytest.raises(hz.HZError):
        hz.decode(bad)
    rc, out = _extract_rc(hz, tmp_path, bad)
    assert rc == 2 and not out.exists()


def test_header_n_smaller_decodes_prefix(hz):
    data = _zipf_bytes(1 << 20, 5)
    blob = oracle_lib.encode(data)
    short = _set_n(blob, 1000)
    assert hz.decode(short) == data[:1000]


@pytest.mark.parametrize("where", ["payload", "header"])
def test_bit_flips_end_cleanly(hz, tmp_path, where):
    """A flipped bit either decodes (to some bytes) or is rejected; never a hang
    or a fault. Same outcome through the library and the CLI."""
    data = _zipf_bytes(1 << 20, 6)
    blob = bytearray(oracle_lib.encode(data))
    cb, info = hz.parse_header(bytes(blob))
    rng = np.random.default_rng(1)
    for trial in range(4):
        b = bytearray(blob)
        pos = int(rng.integers(info.payload_byte + 1, len(b))) if where == "payload" else int(rng.integers(4, 40))
        b[pos] ^= 1 << int(rng.integers(0, 8))
        try:
            out = hz.decode(bytes(b))
            ok = True
        except hz.HZError:
            ok = False
        rc, f = _extract_rc(hz, tmp_path, bytes(b))
        assert rc == (0 if ok else 2)
        if ok:
            assert f.read_bytes() == out
            f.unlink()


# ---- encoder parity at scale: literal GenerateCL codebooks, literal Compressor.cu writer ----
sys.path.insert(0, GOLD)
import make_scale_golden as msg  # noqa: E402

SCALE = msg.load_fixture()


@pytest.mark.parametrize("name,kind", [("zipf_256MiB", 1), ("uniform_256MiB", 0)])
def test_scale_codebook_on_device(hz, codec, name, kind):
    """Device histogram of the bench stream's first 256 MiB -> product codebook
    and header == the literal GenerateCL / Compressor.cu writer fixture."""
    import torch
    n = SCALE[name]["n"]
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    codec.dev.generate(x.data_ptr(), n, offset=0, kind=kind, alpha=1.1, seed=42)
    codec.histogram(x)
    h = codec.hist.cpu().numpy().view(np.uint64).copy()
    assert msg.sha(h.astype("<u8").tobytes()) == SCALE[name]["hist_sha256"]
    cb = hz.build_codebook(h)
    order, ln, code = hz.codebook_arrays(cb)
    got = msg.digest(order, ln, code, h, n, 0, header=hz.write_header(cb, n, 0))
    assert got == msg.codebook_keys(SCALE[name])
    del x
    torch.cuda.empty_cache()


@pytest.mark.parametrize("name", ["tie_dense", "tie_ragged"])
def test_scale_tie_streams(hz, name):
    """Tie-dense streams through the whole host API: codebook/header == the
    literal fixture, file == the literal Compressor.cu writer (except B1/B2)."""
    data = msg.tie_stream(name)
    blob = hz.encode(data)
    cb, info = hz.parse_header(blob)
    order, ln, code = hz.codebook_arrays(cb)
    h = oracle_lib.hist16(data)
    n = SCALE[name]["n"]
    last = int(data[-1]) if n % 2 else 0
    assert msg.digest(order, ln, code, h, n, last) == msg.codebook_keys(SCALE[name])
    diff, allowed, _ = msg.literal_divergence(data, blob, order, ln, code)
    assert set(diff) <= set(allowed)


def test_product_equals_literal_writer_except_b1_b2(hz):
    """hz.encode against the literal Compressor.cu writer: byte for byte equal
    except at the reference's B1/B2 bytes (and the sweep does hit both)."""
    hits = {"B1": 0, "B2": 0}
    for n in list(range(2, 160)) + [1001, 4097, 65537, (16 << 20) + 1]:
        for kind in (0, 1):
            data = oracle_lib.generate(n, offset=7 * n, kind=kind, seed=3)
            h = oracle_lib.hist16(data)
            if np.count_nonzero(h) < 2:
                continue
            blob = hz.encode(data)
            cb, _ = hz.parse_header(blob)
            order, ln, code = hz.codebook_arrays(cb)
            diff, allowed, undef = msg.literal_divergence(data, blob, order, ln, code)
            assert set(diff) <= set(allowed), (n, kind, diff, allowed)
            for p in diff:
                hits[allowed[p]] += 1
    assert hits["B1"] > 0 and hits["B2"] > 0, hits


@pytest.mark.parametrize("start_bit", [0, 7, 32, 45, 64, 96, 127, 145, 671])
def test_fixed16_block_kernels_any_start(hz, start_bit):
    """FIXED16 streams (every code 16 bits): every block but the last goes through the 1 KiB-coalesced
    block kernels (k_pack_fixed16_blk / k_decode_fixed16_blk) at any word and bit of the output; the
    stream equals the oracle's packer and decodes bit-exact through the index hz_pack wrote."""
    import torch
    from huffman_amd.codec import Device, build_codebook
    rng = np.random.default_rng(start_bit)
    sym = np.concatenate([rng.permutation(65536), rng.permutation(65536),
                          rng.permutation(65536)[:9000]]).astype(np.uint16)
    data = sym.view(np.uint8).copy()   # every symbol 2 or 3 times: all codes 16 bits, a partial last block
    nsym = sym.size
    h = oracle_lib.hist16(data)
    _, ln, code = oracle_lib.codebook(h)
    assert (ln == 16).all()
    dev = Device()
    dev.upload(build_codebook(h))
    d_in = torch.from_numpy(data).cuda()
    cap = (start_bit + 16 * nsym) // 8 + 64
    d_out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    idx = torch.zeros(hz.index_bytes(nsym) // 8 + 8, dtype=torch.int64, device="cuda")
    dev.pack(d_in.data_ptr(), data.size, start_bit, 0, d_out.data_ptr(), cap, idx.data_ptr())
    dec = torch.empty(data.size + 16, dtype=torch.uint8, device="cuda")
    dev.decode(d_out.data_ptr(), cap, nsym, idx.data_ptr(), dec.data_ptr())
    dev.sync()
    b0 = start_bit // 8
    ref = oracle_lib.pack_range(data, 0, nsym, ln, code, start_bit - 8 * b0, (16 * nsym + 7) // 8 + 2)
    got = d_out.cpu().numpy()[b0:b0 + ref.size]
    assert np.array_equal(got[:(start_bit % 8 + 16 * nsym) // 8], ref[:(start_bit % 8 + 16 * nsym) // 8])
    assert np.array_equal(dec[:data.size].cpu().numpy(), data)
    dev.close()


@pytest.mark.parametrize("name", ["romeo.txt", "zipf_odd"])
def test_integration_example_archives_like_the_oracle(hz, tmp_path, name):
    """INTEGRATION.md §2's C++ binding, compiled against the C ABI (tests/test_host.py), run on the
    device: the file it writes equals the oracle's (romeo.txt and a 3 MiB + 1 Zipf file)."""
    import subprocess
    from test_host import build_integration_example
    exe = build_integration_example(tmp_path)
    data = read(name) if name == "romeo.txt" else oracle_lib.generate((3 << 20) + 1, kind=1, seed=4).tobytes()
    src, dst = tmp_path / "in", tmp_path / "out"
    src.write_bytes(data)
    r = subprocess.run([str(exe), str(src), str(dst)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert dst.read_bytes() == oracle_lib.encode(data)
