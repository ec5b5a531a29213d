"""Debug the index-less decode (hz_decode_indexless) on one stream: device segment records (entries,
counts, F) against the true ones computed on the host from the codebook, and the first wrong symbol.
Needs the HZ_SEG_DEBUG variant: python tools/build_variant.py lib_segdbg -DHZ_SEG_DEBUG
usage: HZ_LIB_VARIANT=lib_segdbg python tools/debug/seg_debug.py [bytes] [seed]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from huffman_amd import codebook_arrays  # noqa: E402
from huffman_amd._lib import load  # noqa: E402
from huffman_amd.pipeline import StreamCodec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else (1 << 20) + 1
seed = int(sys.argv[2]) if len(sys.argv) > 2 else n % 97
c = StreamCodec(0)
x = torch.empty(n, dtype=torch.uint8, device="cuda")
c.dev.generate(x.data_ptr(), n, offset=0, kind=1, alpha=1.1, seed=seed)
plan, payload, index = c.encode(x)
c.sync()
nsym = n // 2
host = x.cpu().numpy()
sym = host[0:2 * nsym:2].astype(np.uint32) | (host[1:2 * nsym:2].astype(np.uint32) << 8)
_, ln, _ = codebook_arrays(plan.cb)
L = ln[sym].astype(np.uint64)
bnd = plan.start_bit + np.concatenate([[0], np.cumsum(L)]).astype(np.uint64)  # codeword starts, then the end
out = torch.zeros(2 * nsym + 16, dtype=torch.uint8, device="cuda")
end = torch.zeros(2, dtype=torch.int64, device="cuda")
c.dev.decode_indexless(payload.data_ptr(), payload.numel(), plan.start_bit, nsym, out.data_ptr(), end.data_ptr())
c.sync()
got = out[:2 * nsym].cpu().numpy()
bad = np.nonzero(got != host[:2 * nsym])[0]
print("n", n, "nsym", nsym, "start_bit", plan.start_bit, "max_len", plan.cb.max_len, "end", int(end[0].item()),
      "true end", int(bnd[-1]), "bad bytes", bad.size, "first bad sym", (bad[0] // 2) if bad.size else None, flush=True)
pay_bytes = payload.numel()
reach = (plan.start_bit + nsym * max(int(plan.cb.max_len), 1) + 7) // 8 + 8
pay_bytes = min(pay_bytes, reach)
bits = pay_bytes * 8 - plan.start_bit
nseg = (bits + 4095) // 4096
lib = load()
# scratch layout (hz_kernels.hip launch_decode_indexless): piece records (u16) first, then ent, cnt, first
per_seg = 4096.0 / max(bits / nsym, 1.0)
recs = per_seg / 8.0
rcap = min(max(int((recs * 1.3 + 4.0 + 15.0) / 16.0) * 16, 16), 1024)
REC = (nseg * rcap + 7) // 8 + 2
words = REC + 5 * nseg + 8
buf = np.zeros(words, dtype=np.uint64)
rc = lib.hz_debug_scratch(c.dev.h, buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(words))
print("scratch rc", rc, "nseg", nseg, "rcap", rcap)
rec = buf[:REC].view(np.uint8)[:nseg * rcap].reshape(nseg, rcap)
buf = buf[REC:]
ent, cnt, first = buf[:nseg], buf[nseg:2 * nseg], buf[2 * nseg:3 * nseg]
starts = plan.start_bit + 4096 * np.arange(nseg, dtype=np.uint64)
# true: first boundary >= segment start; codewords starting in the segment (the padding's past the end excluded)
tb = bnd[:-1]
idx = np.searchsorted(tb, starts)
true_ent = np.where(idx < tb.size, tb[np.minimum(idx, tb.size - 1)], 0)
true_cnt = np.diff(np.concatenate([idx, [tb.size]]))
true_first = idx
lim = int(np.searchsorted(starts, bnd[-1]))  # segments before the stream's end
de = np.nonzero(ent[:lim] != true_ent[:lim])[0]
dc = np.nonzero(cnt[:lim - 1] != true_cnt[:lim - 1])[0]
df = np.nonzero(first[:lim] != true_first[:lim])[0]
print("segments checked", lim, "entry diffs", de.size, de[:10], "count diffs", dc.size, dc[:10], "F diffs", df.size, df[:10])
for k in list(de[:3]) + list(dc[:3]):
    print(" seg", k, "ent", int(ent[k]), "true", int(true_ent[k]), "cnt", int(cnt[k]), "true", int(true_cnt[k]),
          "F", int(first[k]), "true", int(true_first[k]))
# piece records: every 8th codeword start of a segment, as u8 distances from the previous one (the entry first)
bad_rec = 0
for k in range(min(lim, 2000)):
    e0 = np.searchsorted(tb, starts[k])
    e1 = np.searchsorted(tb, starts[k] + 4096)
    want = tb[e0 + 8:e1:8] - starts[k]
    got_r = (int(ent[k]) - int(starts[k]) + np.cumsum(rec[k, :want.size].astype(np.int64))).astype(np.uint64)
    if want.size and not np.array_equal(want, got_r):
        bad_rec += 1
        if bad_rec <= 3:
            print(" rec seg", k, "want", want[:6], "got", got_r[:6])
print("record rows checked", min(lim, 2000), "bad", bad_rec)

