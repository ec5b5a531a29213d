"""Timing experiment: pack the 16 GiB stream as a sequence of hz_pack
calls over C-byte chunks (count -> scan -> write per chunk, so the write's re-read of the
chunk can hit the Infinity Cache) against one hz_pack over the whole stream. Output bits at
chunk seams are not merged (timing only)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from huffman_amd.codec import payload_bits, index_bytes
from huffman_amd.pipeline import StreamCodec

n = 16 << 30
c = StreamCodec(0)
x = torch.empty(n, dtype=torch.uint8, device="cuda")
c.dev.generate(x.data_ptr(), n, offset=0, kind=1, alpha=1.1, seed=42)
plan, pay, idx = c.encode(x)
c.sync()


def timed(fn, reps=3):
    ts = []
    for _ in range(reps):
        c.sync()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        c.sync()
        ts.append(e0.elapsed_time(e1))
    return min(ts), float(np.median(ts))


print("whole", timed(lambda: c.pack(x, plan, pay, idx)), flush=True)
for C in (128 << 20, 256 << 20, 512 << 20, 1 << 30):
    starts, bits = [], []
    g = plan.start_bit
    for off in range(0, n, C):
        c.histogram(x[off:off + C])
        h = c.hist.cpu().numpy().view(np.uint64).copy()
        starts.append(g)
        b = payload_bits(plan.cb, h)
        bits.append(b)
        g += b
    cidx = torch.empty((index_bytes(C // 2) + 7) // 8, dtype=torch.int64, device="cuda")

    def run():
        for k, off in enumerate(range(0, n, C)):
            gb = starts[k]
            w0 = gb // 32
            cap = pay.numel() - 4 * w0
            c.dev.pack(x.data_ptr() + off, C, gb % 32, 0, pay.data_ptr() + 4 * w0, cap, cidx.data_ptr())
    print("chunk", C >> 20, "MiB", timed(run), flush=True)
