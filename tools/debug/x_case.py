"""Debug: one index-less decode of a synthetic Zipf stream (size, seed) with HZ_DEBUG=1 diagnostics."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("HZ_DEBUG", "1")
import torch  # noqa: E402
from huffman_amd.pipeline import StreamCodec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else (48 << 20) + 2
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 21
c = StreamCodec(0)
x = torch.empty(n, dtype=torch.uint8, device="cuda")
c.dev.generate(x.data_ptr(), n, offset=0, kind=1, alpha=1.1, seed=seed)
plan, pay, idx = c.encode(x)
c.sync()
print("max_len", plan.cb.max_len, "min_len", plan.cb.min_len, flush=True)
out = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")
end = torch.full((2,), -1, dtype=torch.int64, device="cuda")
try:
    c.dev.decode_indexless(pay.data_ptr(), pay.numel(), plan.start_bit, n // 2, out.data_ptr(), end.data_ptr())
    c.sync()
    print("ok", torch.equal(out[:n], x), flush=True)
except Exception as e:  # noqa: BLE001
    print("failed:", e, flush=True)
