"""Pin the CPU oracle (oracle/hz_oracle.c) before trusting it as the checker.

Pins:
  1. the reference decoder (Decompressor.cu, oracle/_ref/extract) accepts the
     oracle's files and reproduces the input;
  2. the oracle decodes the reference baseline encoder's files (golden);
  3. the codebook KAT of SURVEY.md 8(a4) and the literal round-by-round
     GenerateCL restatement (oracle/generatecl_literal.py).
"""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle_lib
from generatecl_literal import generate_cl, reference_codebook

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
INPUTS = ["romeo.txt", "synth_zipf_65537.bin", "synth_unif_65536.bin", "synth_zipf_4099.bin"]


def read(name):
    with open(os.path.join(GOLD, name), "rb") as f:
        return f.read()


def codes_of(order, ln, code):
    return [format(int(code[s]), "0%db" % ln[s]) for s in order]


def test_kat_codebook():
    kat = json.loads(read("kat.json"))
    assert generate_cl(kat["freqs"]) == kat["gpu_codes"]
    hist = np.zeros(65536, dtype=np.uint64)
    hist[:5] = kat["freqs"]
    order, ln, code = oracle_lib.codebook(hist)
    assert list(order) == [0, 1, 2, 3, 4]
    assert codes_of(order, ln, code) == kat["gpu_codes"]


@pytest.mark.parametrize("seed", range(12))
def test_sequential_matches_literal_generatecl(seed):
    rng = np.random.default_rng(seed)
    U = int(rng.integers(2, 400))
    hist = np.zeros(65536, dtype=np.uint64)
    syms = rng.choice(65536, U, replace=False)
    kind = seed % 4
    if kind == 0:
        vals = rng.integers(1, 4, U)          # heavy ties
    elif kind == 1:
        vals = rng.integers(1, 100000, U)
    elif kind == 2:
        vals = rng.zipf(1.2, U)
    else:
        vals = 2 ** rng.integers(0, 12, U)    # equal sums everywhere
    hist[syms] = vals
    # the product counts in u64; the reference's u32 (fbits=32) agrees whenever
    # the total stays below 2^32 (checked in the next test)
    ref_order, ref_codes = reference_codebook([int(x) for x in hist], fbits=64)
    order, ln, code = oracle_lib.codebook(hist)
    assert list(order) == ref_order
    assert codes_of(order, ln, code) == [ref_codes[s] for s in ref_order]


def test_u32_and_u64_literal_agree_below_2_32():
    rng = np.random.default_rng(7)
    hist = [0] * 65536
    for s in rng.choice(65536, 300, replace=False):
        hist[int(s)] = int(rng.integers(1, 1 << 20))
    assert sum(hist) < 2 ** 32
    assert reference_codebook(hist, fbits=32) == reference_codebook(hist, fbits=64)


def test_literal_generatecl_large_alphabet():
    data = read("romeo.txt")
    hist = oracle_lib.hist16(data)
    ref_order, ref_codes = reference_codebook([int(x) for x in hist])
    order, ln, code = oracle_lib.codebook(hist)
    assert list(order) == ref_order
    assert codes_of(order, ln, code) == [ref_codes[s] for s in ref_order]


def test_hist16_matches_numpy():
    data = read("synth_zipf_65537.bin")
    a = np.frombuffer(data, dtype=np.uint8)
    sym = a[0:len(a) // 2 * 2:2].astype(np.uint32) | (a[1:len(a) // 2 * 2:2].astype(np.uint32) << 8)
    assert np.array_equal(oracle_lib.hist16(data), np.bincount(sym, minlength=65536).astype(np.uint64))


@pytest.mark.parametrize("name", INPUTS)
def test_golden_encoder_output(name):
    assert oracle_lib.encode(read(name)) == read(name + ".compressed")


@pytest.mark.parametrize("name", INPUTS)
def test_oracle_decodes_baseline_files(name):
    assert oracle_lib.decode(read(name + ".baseline.compressed")) == read(name)


@pytest.mark.parametrize("name", INPUTS)
def test_oracle_roundtrip(name):
    assert oracle_lib.decode(oracle_lib.encode(read(name))) == read(name)


def _ref_extract(tmp_path, blob):
    exe = oracle_lib.ref_binary("extract")
    if exe is None:
        pytest.skip("reference decoder not built (oracle/Makefile ref)")
    p = tmp_path / "x.compressed"
    p.write_bytes(blob)
    subprocess.run([exe, "x.compressed"], cwd=tmp_path, check=True, capture_output=True, timeout=120)
    return (tmp_path / "DECOMPRESSED_FILE").read_bytes()


@pytest.mark.parametrize("name", INPUTS + ["pexels-vlad-alexandru-popa-1402787.jpg"])
def test_reference_decoder_accepts_oracle_output(tmp_path, name):
    data = read(name)
    assert _ref_extract(tmp_path, oracle_lib.encode(data)) == data


@pytest.mark.parametrize("data", [b"ab", b"abc", b"abab" * 7, b"\x00\x00" * 1000 + b"\x01", bytes(range(256)) * 3])
def test_edge_cases_reference_decoder(tmp_path, data):
    # U == 1 inputs (b"abab"...) use code "0": accepted by the reference decoder.
    assert _ref_extract(tmp_path, oracle_lib.encode(data)) == data


@pytest.mark.parametrize("n", [0, 1])
def test_degenerate_no_symbols(n):
    data = b"\x07" * n
    blob = oracle_lib.encode(data)
    assert blob[:2] == b"\x00\x00" and len(blob) == 3 + n + 8
    assert oracle_lib.decode(blob) == data


def test_baseline_differs_from_gpu_semantics():
    # the baseline encoder breaks ties differently: not an encoder golden
    assert read("romeo.txt.baseline.compressed") != read("romeo.txt.compressed")


def test_generator_zipf_distribution():
    a = oracle_lib.generate(1 << 20, kind=1)
    counts = np.bincount(a, minlength=256) / a.size
    r = np.arange(1, 257.0)
    p = r ** -1.1 / (r ** -1.1).sum()
    assert np.abs(counts - p).max() < 2e-3
    b = oracle_lib.generate(1 << 16, offset=12345, kind=1)
    assert np.array_equal(b[100:200], oracle_lib.generate(100, offset=12445, kind=1))


def test_oracle_header_parse_pins():
    """oracle_lib.parse_header (Decompressor.cu:65-103) on the golden files: the
    entries follow the oracle codebook of the input's histogram ((count, symbol)
    order for this encoder's files; any order for the reference baseline's), N and
    the odd byte match the input, and the payload decodes from the parsed position."""
    for name in ["romeo.txt", "synth_zipf_4099.bin", "synth_zipf_65537.bin", "synth_unif_65536.bin"]:
        data = open(os.path.join(GOLD, name), "rb").read()
        h = oracle_lib.hist16(data)
        order, ln, code = oracle_lib.codebook(h)
        for suffix in (".compressed", ".baseline.compressed"):
            blob = open(os.path.join(GOLD, name + suffix), "rb").read()
            porder, pln, pcode, info = oracle_lib.parse_header(blob)
            assert info[0] == len(data) and info[3] == len(data) % 2 and info[5] == int((h > 0).sum())
            if len(data) % 2:
                assert info[4] == data[-1]
            assert set(porder.tolist()) == set(np.nonzero(h)[0].tolist())
            if suffix == ".compressed":
                assert np.array_equal(porder, order) and np.array_equal(pln, ln)
                assert np.array_equal(pcode[ln > 0], code[ln > 0])
            bits = 8 * info[1] + info[2] + int(np.sum(h * pln.astype(np.uint64)))
            assert (bits + 7) // 8 == len(blob)
    for cut in (2, 5, 100):
        with pytest.raises(ValueError):
            oracle_lib.parse_header(open(os.path.join(GOLD, "romeo.txt.compressed"), "rb").read()[:cut])
