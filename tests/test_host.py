"""CPU-side checks of the product library: it loads, exports every entry point
include/huffman_amd.h declares, and its host stages (codebook, header writer,
header parser) match the oracle byte for byte. No compute on a GPU here."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle_lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def read(name):
    with open(os.path.join(GOLD, name), "rb") as f:
        return f.read()


def declared_symbols():
    with open(os.path.join(ROOT, "include", "huffman_amd.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(hz_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol(built_lib):
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(built_lib, s), s
    from huffman_amd._lib import PROTOTYPES
    assert sorted(n for n, _, _ in PROTOTYPES) == syms


def test_cli_binaries_built(built_lib):
    import huffman_amd
    for name in ("archive", "extract"):
        assert os.access(os.path.join(huffman_amd.BIN_DIR, name), os.X_OK)


def test_ctx_create_fails_loudly_without_gpu(built_lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = ctypes.c_void_p()
    rc = built_lib.hz_ctx_create(0, None, ctypes.byref(h))
    assert rc == -9  # HZ_ENODEV: no silent CPU path


def _hist_random(seed, U, hi):
    rng = np.random.default_rng(seed)
    h = np.zeros(65536, dtype=np.uint64)
    h[rng.choice(65536, U, replace=False)] = rng.integers(1, hi, U)
    return h


@pytest.mark.parametrize("U,hi", [(1, 5), (2, 3), (3, 3), (257, 4), (5000, 1000), (65536, 100000)])
def test_codebook_matches_oracle(built_lib, U, hi):
    import huffman_amd
    h = _hist_random(U, U, hi)
    cb = huffman_amd.build_codebook(h)
    order, ln, code = huffman_amd.codebook_arrays(cb)
    o_order, o_ln, o_code = oracle_lib.codebook(h)
    assert np.array_equal(order, o_order)
    assert np.array_equal(ln, o_ln)
    assert np.array_equal(code, o_code)
    assert cb.max_len == ln.max() and cb.min_len == ln[ln > 0].min()


def test_codebook_matches_oracle_random_histograms(built_lib):
    """300 seeded random histograms (1..65 536 symbols; flat, power-law, geometric, tie-heavy and
    Fibonacci-like counts up to 2^40): the host builder's order, lengths and codes equal the oracle's,
    or both refuse codes past HZ_MAXLEN."""
    import huffman_amd
    rng = np.random.default_rng(17)
    for case in range(300):
        U = int(rng.choice([1, 2, 3, 7, 64, 1000, 4096, 65536]))
        kind = case % 5
        r = np.arange(1, U + 1, dtype=np.float64)
        if kind == 0:
            c = rng.integers(1, 1 << int(rng.integers(1, 40)), U)
        elif kind == 1:
            c = np.maximum(1, (1e9 * r ** -rng.uniform(0.5, 2.5)).astype(np.int64))
        elif kind == 2:
            c = np.maximum(1, (1e12 * rng.uniform(0.3, 0.95) ** r).astype(np.int64))
        elif kind == 3:
            c = rng.integers(1, 4, U)  # ties everywhere
        else:
            f = [1, 1]
            while len(f) < U:
                f.append(min(f[-1] + f[-2], 1 << 40))
            c = np.array(f[:U], dtype=np.int64)
        h = np.zeros(65536, dtype=np.uint64)
        h[rng.choice(65536, U, replace=False)] = c.astype(np.uint64)
        try:
            o_order, o_ln, o_code = oracle_lib.codebook(h)
        except RuntimeError:
            with pytest.raises(Exception):
                huffman_amd.build_codebook(h)
            continue
        cb = huffman_amd.build_codebook(h)
        order, ln, code = huffman_amd.codebook_arrays(cb)
        assert np.array_equal(order, o_order), (case, U, kind)
        assert np.array_equal(ln, o_ln), (case, U, kind)
        assert np.array_equal(code, o_code), (case, U, kind)


@pytest.mark.parametrize("name", ["romeo.txt", "synth_zipf_65537.bin", "synth_unif_65536.bin", "synth_zipf_4099.bin"])
def test_header_matches_golden(built_lib, name):
    import huffman_amd
    data = read(name)
    h = oracle_lib.hist16(data)
    cb = huffman_amd.build_codebook(h)
    hdr, pbits, pend = huffman_amd.write_header(cb, len(data), data[-1] if len(data) % 2 else 0)
    gold = read(name + ".compressed")
    hb = huffman_amd.header_bits(cb, len(data))
    assert len(hdr) == hb // 8 and pbits == hb % 8
    assert gold[:len(hdr)] == hdr
    # pending header bits are the top bits of the first payload byte
    if pbits:
        assert (gold[len(hdr)] >> (8 - pbits)) == (pend >> (8 - pbits))
    total = hb + huffman_amd.payload_bits(cb, h)
    assert (total + 7) // 8 == len(gold)


@pytest.mark.parametrize("name", ["romeo.txt.compressed", "romeo.txt.baseline.compressed",
                                  "synth_unif_65536.bin.baseline.compressed"])
def test_header_parse(built_lib, name):
    import huffman_amd
    blob = read(name)
    cb, info = huffman_amd.parse_header(blob)
    src = read(name.split(".compressed")[0].replace(".baseline", ""))
    assert info.n == len(src) and info.is_odd == len(src) % 2
    if info.is_odd:
        assert info.last_byte == src[-1]
    assert cb.nsym == np.count_nonzero(oracle_lib.hist16(src))


def test_header_parse_rejects_garbage(built_lib):
    import huffman_amd
    from huffman_amd import HZError
    with pytest.raises(HZError):
        huffman_amd.parse_header(b"\x05\x00\x00\x12")          # truncated codebook
    with pytest.raises(HZError):
        huffman_amd.parse_header(b"\x01")


def test_header_parse_empty_conventions(built_lib):
    import huffman_amd
    for data in (b"", b"x"):
        blob = oracle_lib.encode(data)
        cb, info = huffman_amd.parse_header(blob)
        assert cb.nsym == 0 and info.n == len(data)


def test_index_geometry(built_lib):
    """Block index: u64 start[nblocks + 1] + u64 max_bits + u16 sub[nblocks][256] (include/huffman_amd.h)."""
    assert built_lib.hz_index_format() == 2  # sub[] = absolute low 16 bits (include/huffman_amd.h)
    assert built_lib.hz_index_stride() == 2048
    assert built_lib.hz_index_bytes(0) == 0
    assert built_lib.hz_index_bytes(1) == 8 * 3 + 512
    assert built_lib.hz_index_bytes(2049) == 8 * 4 + 2 * 512
    assert built_lib.hz_index_bytes(1 << 33) == 8 * ((1 << 22) + 2) + 512 * (1 << 22)


def build_integration_example(tmp_path):
    """INTEGRATION.md §2's C++ binding (archive_buffer) with a main that archives argv[1] into argv[2],
    compiled with g++ against include/huffman_amd.h and linked with the library: the binding a
    maintainer would add is valid C++ against the ABI as declared."""
    import subprocess
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        code = re.findall(r"```cpp\n(.*?)```", f.read(), re.S)[0]
    main = r'''
#include <cstdio>
int main(int argc, char** argv) {
    if (argc != 3) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<uint8_t> in;
    for (int c; (c = fgetc(f)) != EOF;) in.push_back((uint8_t)c);
    fclose(f);
    std::vector<uint8_t> file;
    const int st = archive_buffer(in.data(), in.size(), file);
    if (st != HZ_OK) { fprintf(stderr, "status %d\n", st); return 1; }
    FILE* o = fopen(argv[2], "wb");
    fwrite(file.data(), 1, file.size(), o);
    fclose(o);
    return 0;
}
'''
    src = tmp_path / "archive_amd.cpp"
    src.write_text(code + main)
    exe = tmp_path / "archive_amd"
    lib_dir = os.path.join(ROOT, "huffman_amd", "lib")
    r = subprocess.run(["g++", "-std=c++17", "-w", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                        "-I" + os.path.join(ROOT, "include"), str(src), "-L" + lib_dir, "-lhuffman_amd",
                        "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath," + lib_dir, "-o", str(exe)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return exe


def test_integration_example_compiles_and_links(built_lib, tmp_path):
    exe = build_integration_example(tmp_path)
    assert os.access(exe, os.X_OK)
