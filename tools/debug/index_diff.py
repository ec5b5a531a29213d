"""Debug: rebuild the block index from the payload alone and report where it
differs from the index hz_pack wrote. usage: python tools/debug/index_diff.py [kind] sizes..."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from huffman_amd import index_bytes
from huffman_amd.pipeline import StreamCodec

kind = int(sys.argv[1]) if len(sys.argv) > 1 else 1
sizes = [int(v) for v in sys.argv[2:]] or [10001, 100001, 1 << 20, (6 << 20) + 1]
c = StreamCodec(0)
for n in sizes:
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    c.dev.generate(x.data_ptr(), n, offset=0, kind=kind, alpha=1.1, seed=11)
    plan, pay, idx = c.encode(x)
    reb = torch.full_like(idx, -1)
    c.dev.index_build(pay.data_ptr(), pay.numel(), plan.start_bit, n // 2, reb.data_ptr())
    c.sync()
    nsym = n // 2
    nb = (nsym + 2047) // 2048
    a = idx.cpu().numpy().view(np.uint64)
    b = reb.cpu().numpy().view(np.uint64)
    sa, sb = a[:nb + 2], b[:nb + 2]
    bad = np.nonzero(sa != sb)[0]
    ua = a.view(np.uint16)[4 * (nb + 2):4 * (nb + 2) + 256 * nb]
    ub = b.view(np.uint16)[4 * (nb + 2):4 * (nb + 2) + 256 * nb]
    badu = np.nonzero(ua != ub)[0]
    print(f"n={n} blocks={nb} start mismatches={bad.size} first={bad[:5]} "
          f"sub mismatches={badu.size} first={badu[:8]}", flush=True)
    if bad.size:
        i = bad[0]
        print("   pack:", sa[max(0, i - 2):i + 3], "\n   rebuilt:", sb[max(0, i - 2):i + 3], flush=True)
    if badu.size:
        i = badu[0]
        print("   pack sub:", ua[max(0, i - 4):i + 4], "\n   rebuilt:", ub[max(0, i - 4):i + 4], flush=True)
    if badu.size:
        # absolute positions of the mismatching chain starts; segment (4096-bit) and lane/chain of the walker
        for u in badu[:12]:
            b = u // 256
            P = int(sa[b]) + int(ua[u]); R = int(sa[b]) + int(ub[u])
            seg = (P - plan.start_bit) // 4096
            print(f"   chain {u}: pack {P} rebuilt {R} diff {R - P} segment {seg} lane-group {seg // 4} chain {seg % 4}",
                  flush=True)
