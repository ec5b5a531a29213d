"""k_cb_generate phase times (HZ_CB_PROF variant: HZ_LIB_VARIANT=lib_cbprof)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from huffman_amd._lib import Codebook
from huffman_amd.pipeline import StreamCodec
c = StreamCodec(0)
for kind in (1, 0):
    n = 1 << 30
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    c.dev.generate(x.data_ptr(), n, offset=0, kind=kind, alpha=1.1, seed=42)
    c.histogram(x); c.sync(); del x
    h = c.hist.cpu().numpy().view(np.uint64) * np.uint64(16)
    hd = torch.from_numpy(h.view(np.int64)).cuda()
    d_cb = torch.zeros(ctypes.sizeof(Codebook), dtype=torch.uint8, device="cuda")
    for rep in range(3):
        c.dev.codebook_build(hd.data_ptr(), d_cb.data_ptr()); c.sync()
    print("kind", kind)
    buf = (ctypes.c_uint64 * 512)()
    import huffman_amd._lib as L
    lib = L.load()
    lib.hz_debug_cb_prof.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.hz_debug_cb_prof(c.dev.h, buf)
    p = np.array(buf, dtype=np.uint64)
    t0 = int(p[0]); nr = int(p[5])
    us = lambda v: (int(v) - t0) / 100.0
    print(f"init {us(p[1]):.1f} us, CL end {us(p[2]):.1f}, CW end {us(p[3]):.1f}, end {us(p[4]):.1f}, rounds {nr}")
    prev = us(p[1])
    for r in range(min(nr, 120)):
        s_, e_ = us(p[16 + 4 * r]), us(p[17 + 4 * r])
        P, nt = int(p[18 + 4 * r]) & 0xffffffff, int(p[18 + 4 * r]) >> 32
        a, b = int(p[19 + 4 * r]) & 0xffffffff, int(p[19 + 4 * r]) >> 32
        print(f" r{r:3d} search {s_ - prev:6.2f} rest {e_ - s_:6.2f} us  P {P} tiles {nt} a {a} b {b}")
        prev = e_
