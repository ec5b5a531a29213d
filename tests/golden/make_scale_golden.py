"""Generate tests/golden/scale_codebooks.json: the reference's codebook and header
at the configs' alphabet size (U = 65 536), pinned by literal restatements.

For each case the histogram is built, the codebook is computed by the literal
round-by-round GenerateCL / GenerateCW / toCpu restatement
(oracle/generatecl_literal.py, u32 node sums as in gpuHuffmanConstruction.h)
over the thrust (freq, symbol) order (Compressor.cu:378-425), and the header is
written by the literal Compressor.cu writer (oracle/compressor_literal.c,
hzl_header: Compressor.cu:431-487,637-669). Hashes of the results are stored,
so the GPU box (no reference there) checks the product's codebook and header
against them without rerunning the literal code.

Cases:
  zipf_256MiB     first 256 MiB of the bench's Zipf(1.1) stream (seed 42)
  uniform_256MiB  first 256 MiB of the bench's uniform stream (seed 42)
  tie_dense       hist[s] = 1000 + (u[s] & 1), u = uniform stream (seed 7):
                  every count in {1000, 1001}, 65 536 symbols (maximal ties,
                  gpuHuffmanConstruction.h:193-206 decides them)
  tie_ragged      about 57 000 symbols (u & 7 != 0, u = uniform stream, seed 9)
                  with counts in {1000, 1001, 2000, 2001}: ties and mixed code
                  lengths (15-17 bits), an odd N whose raw last byte is 0x5a

Run: python tests/golden/make_scale_golden.py  (about a minute on one core)
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle_lib  # noqa: E402
from generatecl_literal import reference_codebook  # noqa: E402

OUT = os.path.join(HERE, "scale_codebooks.json")


def sha(b):
    return hashlib.sha256(b).hexdigest()


def case_hist(name):
    """(histogram u64[65536], n bytes, odd last byte) of a case."""
    if name == "zipf_256MiB":
        d = oracle_lib.generate(256 << 20, offset=0, kind=1, seed=42)
        return oracle_lib.hist16(d), d.size, 0
    if name == "uniform_256MiB":
        d = oracle_lib.generate(256 << 20, offset=0, kind=0, seed=42)
        return oracle_lib.hist16(d), d.size, 0
    if name == "tie_dense":
        u = oracle_lib.generate(65536, offset=0, kind=0, seed=7)
        h = 1000 + (u & 1).astype(np.uint64)
        return h, 2 * int(h.sum()), 0
    if name == "tie_ragged":
        u = oracle_lib.generate(65536, offset=0, kind=0, seed=9)
        h = np.array([1000, 1001, 2000, 2001], dtype=np.uint64)[(u >> 3) & 3]
        h[(u & 7) == 0] = 0
        return h, 2 * int(h.sum()) + 1, 0x5a
    raise KeyError(name)


def tie_stream(name):
    """A byte stream with a tie case's histogram (symbol s repeated hist[s]
    times, then the odd raw byte if any)."""
    h, n, last = case_hist(name)
    sym = np.repeat(np.arange(65536, dtype=np.uint16), h.astype(np.int64))
    b = sym.astype("<u2").view(np.uint8)
    return np.concatenate([b, np.array([last], dtype=np.uint8)]) if n % 2 else b


def digest(order, ln, code, hist, n, last, header=None):
    """Hashes of a codebook (header order, lengths and code strings in that
    order) and of its header (complete bytes + pending bits). header: the
    (bytes, pending bit count, pending byte) a writer under test produced;
    default: the literal Compressor.cu writer's."""
    order = np.asarray(order, dtype=np.uint16)
    ln = np.asarray(ln)
    lens = ln[order].astype(np.uint8)
    strings = ",".join(format(int(code[s]), "0%db" % int(ln[s])) for s in order)
    head, pbits, pend = header if header is not None else oracle_lib.reference_header(n, last, order, ln, code)
    return {
        "U": int(order.size),
        "max_len": int(lens.max()),
        "min_len": int(lens.min()),
        "payload_bits": int(np.sum(np.asarray(hist, dtype=np.uint64) * ln.astype(np.uint64))),
        "order_sha256": sha(order.astype("<u2").tobytes()),
        "len_sha256": sha(lens.tobytes()),
        "codes_sha256": sha(strings.encode()),
        "header_sha256": sha(head + bytes([pend, pbits])),
        "header_bytes": len(head),
    }


def load_fixture():
    with open(OUT) as f:
        return json.load(f)


def codebook_keys(d):
    """The fixture fields a codebook + header digest is compared on."""
    return {k: v for k, v in d.items() if k not in ("n", "hist_sha256")}


def literal_divergence(data, ours, order, ln, code):
    """Byte positions where `ours` (a complete .compressed image) differs from
    the literal Compressor.cu writer's image of the same input and codebook,
    and the positions the reference's defects account for:
      B1 (Compressor.cu:294-310): payload byte 0 takes 8 - b bits of symbol
         0's string only; wrong when L(s0) < 8 - b, b = header bits mod 8;
      B2 (:213-247 with :597-601): the last byte walks past the last symbol.
    Returns (diff positions, {position: "B1"|"B2"}, undefined positions)."""
    a = oracle_lib.as_u8(data)
    ref, flags, b1, b2 = oracle_lib.reference_archive(a, order, ln, code)
    assert len(ref) == len(ours)
    r = np.frombuffer(ref, dtype=np.uint8)
    o = np.frombuffer(ours, dtype=np.uint8)
    diff = [int(i) for i in np.nonzero(r != o)[0]]
    b = int(np.asarray(ln)[np.asarray(order)].astype(np.int64).sum()) % 8
    s0 = int(a[0]) | (int(a[1]) << 8)
    allowed = {}
    if b1 >= 0 and b and int(ln[s0]) < 8 - b:
        allowed[b1] = "B1"
    if b2 >= 0:
        allowed[b2] = "B2"
    return diff, allowed, [int(i) for i in np.nonzero(flags)[0]]


def literal_digest(name):
    h, n, last = case_hist(name)
    order, codes = reference_codebook([int(x) for x in h], fbits=32)
    ln = np.zeros(65536, dtype=np.uint8)
    code = np.zeros(65536, dtype=np.uint64)
    for s in order:
        ln[s] = len(codes[s])
        code[s] = int(codes[s], 2)
    d = digest(order, ln, code, h, n, last)
    d.update({"n": n, "hist_sha256": sha(h.astype("<u8").tobytes())})
    return d


CASES = ["zipf_256MiB", "uniform_256MiB", "tie_dense", "tie_ragged"]

if __name__ == "__main__":
    res = {name: literal_digest(name) for name in CASES}
    with open(OUT, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))
