"""Time the device codebook / header kernels on the bench's 16 GiB Zipf histogram."""
import ctypes
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import huffman_amd
from huffman_amd._lib import Codebook
from huffman_amd.pipeline import StreamCodec

c = StreamCodec(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16 << 30
x = torch.empty(n, dtype=torch.uint8, device="cuda")
c.dev.generate(x.data_ptr(), n, offset=0, kind=1, alpha=1.1, seed=42)
c.histogram(x)
c.sync()
d_cb = torch.zeros(ctypes.sizeof(Codebook), dtype=torch.uint8, device="cuda")
out = torch.zeros(16 + 65536 * 11, dtype=torch.uint8, device="cuda")
info = torch.zeros(6, dtype=torch.int64, device="cuda")
for rep in range(3):
    e0, e1, e2, e3 = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    e0.record()
    c.dev.codebook_build(c.hist.data_ptr(), d_cb.data_ptr())
    e1.record()
    c.dev.header_write(d_cb.data_ptr(), n, 0, out.data_ptr(), out.numel(), info.data_ptr())
    e2.record()
    nb = int(info[0].item())
    c.dev.header_parse(out.data_ptr(), nb + 16, d_cb.data_ptr(), info.data_ptr())
    e3.record()
    c.sync()
    h = c.hist.cpu().numpy().view(np.uint64)
    t0 = time.perf_counter()
    cb = huffman_amd.build_codebook(h)
    t1 = time.perf_counter()
    hdr = huffman_amd.write_header(cb, n, 0)
    t2 = time.perf_counter()
    print(f"device codebook {e0.elapsed_time(e1):.3f} ms, header write {e1.elapsed_time(e2):.3f} ms, "
          f"header parse {e2.elapsed_time(e3):.3f} ms | host codebook {(t1 - t0) * 1e3:.3f} ms, "
          f"host header {(t2 - t1) * 1e3:.3f} ms", flush=True)
