"""A/B of the index build (development): encode one synthetic stream, rebuild its
block index from the payload alone R times, print the index-stage kernel time of
each rebuild and whether the rebuilt index equals the one hz_pack wrote.
usage: HZ_LIB_VARIANT=<dir> python tools/debug/index_ab.py [bytes] [reps] [zipf|uniform]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from huffman_amd.pipeline import StreamCodec
from huffman_amd._lib import STAGE_INDEX

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16 << 30
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
kind = 0 if (len(sys.argv) > 3 and sys.argv[3] == "uniform") else 1
c = StreamCodec(0)
x = torch.empty(n, dtype=torch.uint8, device="cuda")
c.dev.generate(x.data_ptr(), n, offset=0, kind=kind, alpha=1.1, seed=42)
plan, pay, idx = c.encode(x)
del x
reb = torch.empty_like(idx)
ts = []
ok = True
for r in range(reps):
    reb.fill_(-1)
    c.dev.index_build(pay.data_ptr(), pay.numel(), plan.start_bit, n // 2, reb.data_ptr())
    c.sync()
    ts.append(c.dev.kernel_ms(STAGE_INDEX))
    ok &= bool(torch.equal(reb, idx))
print(os.environ.get("HZ_LIB_VARIANT", "lib"), "index ms", " ".join(f"{t:.2f}" for t in ts), "match", ok, flush=True)
