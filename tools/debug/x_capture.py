"""Debug: capture hz_decode_indexless into a graph (HZ_CAPTURE_DEBUG=1 prints the capture status per step)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from huffman_amd.pipeline import StreamCodec  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "global"
n = (16 << 20) + 2
c = StreamCodec(0)
x = torch.empty(n, dtype=torch.uint8, device="cuda")
c.dev.generate(x.data_ptr(), n, offset=0, kind=1, alpha=1.1, seed=21)
plan, pay, idx = c.encode(x)
c.sync()
out = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")
end = torch.full((2,), -1, dtype=torch.int64, device="cuda")
call = lambda: c.dev.decode_indexless(pay.data_ptr(), pay.numel(), plan.start_bit, n // 2, out.data_ptr(), end.data_ptr())
call()
c.sync()
print("eager ok", torch.equal(out[:n], x), flush=True)
g = torch.cuda.CUDAGraph()
try:
    with torch.cuda.graph(g, stream=c.stream, capture_error_mode=mode):
        call()
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    print("graph ok", torch.equal(out[:n], x), flush=True)
except Exception as e:  # noqa: BLE001
    print("capture failed:", type(e).__name__, str(e)[:200], flush=True)
