"""Host-side step costs on the box: hist D2H, codebook build, encode/decode table
builds+uploads, header write (16 GiB-like Zipf histogram from a 1 GiB device stream scaled)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from huffman_amd.codec import build_codebook, write_header
from huffman_amd.pipeline import StreamCodec
c = StreamCodec(0)
n = 1 << 30
x = torch.empty(n, dtype=torch.uint8, device='cuda')
c.dev.generate(x.data_ptr(), n, offset=0, kind=1, alpha=1.1, seed=42)
c.histogram(x); c.sync()
for r in range(4):
    t0 = time.perf_counter(); h = c.hist.cpu().numpy().view(np.uint64) * 16
    t1 = time.perf_counter(); cb = build_codebook(h)
    t2 = time.perf_counter(); c.dev.upload_encode(cb)
    t3 = time.perf_counter(); c.dev.upload_decode(cb)
    t4 = time.perf_counter(); write_header(cb, 16 << 30, 0)
    t5 = time.perf_counter(); c.sync()
    print(f"d2h {1e3*(t1-t0):.3f} codebook {1e3*(t2-t1):.3f} upload_enc {1e3*(t3-t2):.3f} "
          f"upload_dec {1e3*(t4-t3):.3f} header {1e3*(t5-t4):.3f} ms", flush=True)
