import sys; sys.path.insert(0,'.')
import torch
from huffman_amd.pipeline import StreamCodec
c = StreamCodec(0)
n = 64 << 20
x = torch.empty(n, dtype=torch.uint8, device='cuda')
c.dev.generate(x.data_ptr(), n, offset=0, kind=1, alpha=1.1, seed=42)
plan, pay, idx = c.encode(x)
out = torch.empty(n + 16, dtype=torch.uint8, device='cuda')
c.decode(pay, n // 2, idx, out)
c.sync()
print('maxlen', plan.cb.max_len, 'ok', torch.equal(out[:n], x))
