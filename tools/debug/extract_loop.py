"""Extract-path timing harness: encode one synthetic stream on the device, then time the index-less
decode (hz_decode_indexless) R times and, for comparison, hz_index_build + hz_decode.
usage: python tools/debug/extract_loop.py [bytes] [reps] [zipf|uniform] [--only-indexless]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from huffman_amd._lib import STAGE_DECODE, STAGE_EXTRACT, STAGE_INDEX  # noqa: E402
from huffman_amd.pipeline import StreamCodec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16 << 30
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
kind = 0 if (len(sys.argv) > 3 and sys.argv[3] == "uniform") else 1
only = "--only-indexless" in sys.argv
c = StreamCodec(0)
x = torch.empty(n, dtype=torch.uint8, device="cuda")
c.dev.generate(x.data_ptr(), n, offset=0, kind=kind, alpha=1.1, seed=42)
plan, pay, idx = c.encode(x)
c.sync()
print("pack", c.kernel_ms(), "ranges", c.dev.last_pack_ranges(), flush=True)
out = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
end = torch.zeros(2, dtype=torch.int64, device="cuda")
for r in range(reps):
    c.dev.decode_indexless(pay.data_ptr(), pay.numel(), plan.start_bit, n // 2, out.data_ptr(), end.data_ptr())
    c.sync()
    xm = c.dev.kernel_ms(STAGE_EXTRACT)
    ok = torch.equal(out[:n - (n & 1)], x[:n - (n & 1)])
    if only:
        print(f"rep {r} indexless {xm:.3f} ms ok {ok}", flush=True)
        continue
    c.dev.index_build(pay.data_ptr(), pay.numel(), plan.start_bit, n // 2, idx.data_ptr())
    c.decode(pay, n // 2, idx, out)
    c.sync()
    print(f"rep {r} indexless {xm:.3f} ms ok {ok} | index {c.dev.kernel_ms(STAGE_INDEX):.3f} + decode "
          f"{c.dev.kernel_ms(STAGE_DECODE):.3f} ms", flush=True)
