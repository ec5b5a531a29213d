"""Escape statistics of the chain walker's 16-bit byte table (hz_codebook.cpp build_walk8) for a Zipf
sample's codebook (the CPU oracle's GenerateCL codebook): the share of codewords under a 16-bit prefix
shared by codes of different lengths (the walk parks on those), and how many distinct maps of the next
6 bits those prefixes have (the escape-class experiment).
usage: python tools/debug/escape_stats.py [bytes] [seed]"""
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import oracle_lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 42
h = oracle_lib.hist16(oracle_lib.generate(n, offset=0, kind=1, seed=seed)).astype(np.float64)
_, ln, code = oracle_lib.codebook(h.astype(np.uint64))
ln = ln.astype(np.int64)
code = [int(c) for c in code]
K, M = 16, int(ln.max())
X = M - K
sub = collections.defaultdict(lambda: np.zeros(1 << max(X, 0), dtype=np.int64))
mass = collections.defaultdict(float)
for s in np.nonzero(ln > K)[0]:
    L, c = int(ln[s]), code[s]
    p, r = c >> (L - K), c & ((1 << (L - K)) - 1)
    sub[p][r << (M - L):(r + 1) << (M - L)] = L
    mass[p] += h[s]
amb = [p for p, v in sub.items() if len(set(v[v > 0])) > 1]
tot = h.sum()
esc = sum(mass[p] for p in amb)
maps = collections.Counter(tuple(sub[p]) for p in amb)
print(f"{n} bytes seed {seed}: max_len {M}, mean code {float((h * ln).sum() / tot):.3f} bits; "
      f"{len(amb)} ambiguous 16-bit prefixes hold {esc / tot:.4f} of the codewords; "
      f"{len(maps)} distinct maps of the next {X} bits")
