"""Profiling harness: encode one synthetic stream on the device, then run
pack and decode R more times (rocprofv3 --pmc passes attribute counters per kernel).
usage: python tools/debug/stage_loop.py [bytes] [reps] [zipf|uniform] [stages: h p d i]"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from huffman_amd.pipeline import StreamCodec
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4 << 30
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
kind = 0 if (len(sys.argv) > 3 and sys.argv[3] == "uniform") else 1
stages = sys.argv[4] if len(sys.argv) > 4 else "hpd"
c = StreamCodec(0)
x = torch.empty(n, dtype=torch.uint8, device='cuda')
c.dev.generate(x.data_ptr(), n, offset=0, kind=kind, alpha=1.1, seed=42)
plan, pay, idx = c.encode(x)
out = torch.empty(n + 16, dtype=torch.uint8, device='cuda')
for r in range(reps):
    if "h" in stages:
        c.histogram(x)
    if "p" in stages:
        c.pack(x, plan, pay, idx)
    if "d" in stages:
        c.decode(pay, n // 2, idx, out)
    if "i" in stages:
        c.dev.index_build(pay.data_ptr(), pay.numel(), plan.start_bit, n // 2, idx.data_ptr())
    c.sync()
    from huffman_amd._lib import STAGE_INDEX
    print("rep", r, c.kernel_ms(), "index", c.dev.kernel_ms(STAGE_INDEX), flush=True)
print('ok', torch.equal(out[:n - (n & 1)], x[:n - (n & 1)]))
