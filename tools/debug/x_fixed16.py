"""Debug: the index-less decode of a uniform (FIXED16) stream against the input and pack's end bit."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from huffman_amd import index_starts  # noqa: E402
from huffman_amd.pipeline import StreamCodec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else (16 << 20) + 2
kind = int(sys.argv[2]) if len(sys.argv) > 2 else 0
c = StreamCodec(0)
x = torch.empty(n, dtype=torch.uint8, device="cuda")
c.dev.generate(x.data_ptr(), n, offset=0, kind=kind, alpha=1.1, seed=3)
plan, pay, idx = c.encode(x)
c.sync()
nsym = n // 2
print("cb", plan.cb.min_len, plan.cb.max_len, plan.cb.nsym, "start", plan.start_bit, "paybits", plan.payload_bits)
end_pack = int(index_starts(idx.cpu().numpy(), nsym)[-1])
out = torch.zeros(2 * nsym + 16, dtype=torch.uint8, device="cuda")
c.decode(pay, nsym, idx, out)
c.sync()
print("decode with pack index ok", torch.equal(out[:2 * nsym], x[:2 * nsym]))
out.zero_()
end = torch.full((2,), -1, dtype=torch.int64, device="cuda")
c.dev.decode_indexless(pay.data_ptr(), pay.numel(), plan.start_bit, nsym, out.data_ptr(), end.data_ptr())
c.sync()
eq = out[:2 * nsym] == x[:2 * nsym]
bad = (~eq).nonzero()
print("indexless ok", bool(eq.all()), "bad bytes", bad.numel(), "first", bad[:5].flatten().tolist(),
      "end", int(end[0]), "pack end", end_pack)
