"""The device codebook's round structure (hz_codebook_gpu.hip, k_cb_generate),
restated in Python and held against the oracle's GenerateCL (tests/oracle_lib.codebook).

k_cb_generate never materialises GenerateCL's round lists
(gpuHuffmanConstruction.h:353-466): it keeps the unused leaves as a suffix of the
sorted keys and the unused internal nodes as a contiguous range, and relies on
(1) internal nodes being created in nondecreasing frequency and (2) the round
list being the (frequency, node id) merge of the two runs. This test replays the
kernel's steps (pivot from the two runs' counts <= f0 + f1, the tail drop when the
pivot is capped or odd, pairs from merge ranks, GenerateCW top-down) on CPU,
asserts (1) on every round, and checks the codes equal the oracle's. No GPU;
the kernel itself is checked against the host builder in test_gpu_codebook.py.

Tolerance: none (bit-exact)."""
import bisect

import numpy as np
import pytest

import oracle_lib


def implicit_generate(h):
    syms = np.nonzero(h)[0]
    order = sorted(syms, key=lambda s: (int(h[s]), int(s)))
    U = len(order)
    lf = [int(h[s]) for s in order]
    nf, par = [], {}
    lp = ip = 0
    while True:
        size = (U - lp) + (len(nf) - ip)
        if size <= 1:
            break
        heads = sorted(x for x in [(lf[lp], 0) if lp < U else None, (lf[lp + 1], 0) if lp + 1 < U else None,
                                   (nf[ip], 1) if ip < len(nf) else None,
                                   (nf[ip + 1], 1) if ip + 1 < len(nf) else None] if x is not None)
        spec = heads[0][0] + heads[1][0]
        a = bisect.bisect_right(lf, spec, lp) - lp
        b = bisect.bisect_right(nf, spec, ip) - ip
        P = min(a + b, max(size - 1, 2)) & ~1
        while a + b > P:  # drop the largest (the newer node on ties)
            if b == 0:
                a -= 1
            elif a == 0:
                b -= 1
            elif nf[ip + b - 1] >= lf[lp + a - 1]:
                b -= 1
            else:
                a -= 1
        A, B = lf[lp:lp + a], nf[ip:ip + b]
        new = [0] * (P // 2)
        node0 = U + len(nf)
        for i, f in enumerate(A):  # a leaf precedes internal nodes of its frequency
            pos = i + bisect.bisect_left(B, f)
            new[pos >> 1] += f
            par[lp + i] = (node0 + (pos >> 1), (pos & 1) ^ 1)
        for i, f in enumerate(B):
            pos = i + bisect.bisect_right(A, f)
            new[pos >> 1] += f
            par[U + ip + i] = (node0 + (pos >> 1), (pos & 1) ^ 1)
        assert all(new[i] <= new[i + 1] for i in range(len(new) - 1))
        assert not nf or new[0] >= nf[-1], "internal nodes must be created in nondecreasing frequency"
        nf += new
        lp += a
        ip += b
    code = {2 * U - 2: (0, 0)}
    for v in range(2 * U - 3, U - 1, -1):
        p, bit = par[v]
        code[v] = ((code[p][0] << 1) | bit, code[p][1] + 1)
    ln = np.zeros(65536, np.uint8)
    cw = np.zeros(65536, np.uint64)
    for i in range(U):
        p, bit = par[i]
        ln[order[i]] = code[p][1] + 1
        cw[order[i]] = (code[p][0] << 1) | bit
    return ln, cw


def _cases():
    rng = np.random.default_rng(11)
    out = {}
    for k, (U, hi) in enumerate([(2, 2), (3, 2), (5, 3), (257, 4), (1000, 2), (3000, 1000), (4096, 1 << 20),
                                 (2000, 3), (65536, 2)]):
        h = np.zeros(65536, np.uint64)
        h[rng.choice(65536, U, replace=False)] = rng.integers(1, hi, U)
        out[f"rand_U{U}_hi{hi}"] = h
    fib = [1, 1]
    while len(fib) < 41:
        fib.append(fib[-1] + fib[-2])
    h = np.zeros(65536, np.uint64)
    h[np.arange(41) * 997 + 5] = fib
    out["fibonacci_41"] = h
    h = np.zeros(65536, np.uint64)
    h[:3000] = 7
    h[3000:3003] = 21
    out["ties"] = h
    return out


CASES = _cases()


@pytest.mark.parametrize("name", sorted(CASES))
def test_implicit_rounds_equal_oracle_generatecl(name):
    h = CASES[name]
    ln, cw = implicit_generate(h)
    order, oln, ocode = oracle_lib.codebook(h)
    assert np.array_equal(ln, oln)
    assert np.array_equal(cw[ln > 0], ocode[ln > 0])
