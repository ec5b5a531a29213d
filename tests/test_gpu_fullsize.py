"""The bench's own configs at full size (BASELINE.json configs 3 and 4: 16 GiB
Zipf(1.1) and 16 GiB uniform bytes on one MI355X), through the same device
pipeline bench.py times (StreamCodec: range-plan histogram -> codebook -> pack
-> decode), checked by size-independent properties, since the oracle cannot
process 16 GiB in a test's time:
  - the round trip is equal on the device;
  - the histogram sums to N/2 and payload_bits == sum(hist * len);
  - the block index is strictly monotone, starts at the payload's first bit and
    ends at start + payload_bits;
  - the index rebuilt from the payload alone (hz_index_build) == pack's index;
  - the index-less decode (hz_decode_indexless, the `extract` path) restores the
    input and ends where pack's index ends.
The 256 MiB prefix of the same streams is pinned against the oracle and the
literal GenerateCL fixtures in test_gpu.py / test_gpu_codebook.py.

Tolerance: none -- every check is bit-exact (integer/bit work)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 16 << 30


@pytest.mark.parametrize("kind", [1, 0], ids=["zipf", "uniform"])
def test_16gib_pipeline_properties(built_lib, kind):
    import torch
    from huffman_amd import codebook_arrays, index_bytes, index_starts
    from huffman_amd.pipeline import StreamCodec
    c = StreamCodec(0)
    x = torch.empty(N, dtype=torch.uint8, device="cuda")
    c.dev.generate(x.data_ptr(), N, offset=0, kind=kind, alpha=1.1, seed=42)
    plan, payload, index = c.encode(x)
    c.sync()
    nsym = N // 2
    h = c.hist.cpu().numpy().view(np.uint64)
    assert int(h.sum()) == nsym
    _, ln, _ = codebook_arrays(plan.cb)
    assert plan.payload_bits == int(np.sum(h * ln.astype(np.uint64)))
    if kind == 1:
        assert c.dev.last_pack_ranges() == 1   # the two-pass encode ran
    starts = index_starts(index.cpu().numpy(), nsym).astype(np.uint64)
    assert int(starts[0]) == plan.start_bit and np.all(np.diff(starts) > 0)
    assert int(starts[-1]) == plan.start_bit + plan.payload_bits
    out = torch.empty(N + 16, dtype=torch.uint8, device="cuda")
    c.decode(payload, nsym, index, out)
    c.sync()
    assert torch.equal(out[:N], x)
    # the index from the payload alone
    nb = index_bytes(nsym)
    rebuilt = torch.full_like(index, -1)
    c.dev.index_build(payload.data_ptr(), payload.numel(), plan.start_bit, nsym, rebuilt.data_ptr())
    c.sync()
    assert torch.equal(rebuilt.view(torch.uint8)[:nb], index.view(torch.uint8)[:nb])
    del rebuilt
    # the extract path: index-less decode
    out.zero_()
    end = torch.zeros(2, dtype=torch.int64, device="cuda")
    c.dev.decode_indexless(payload.data_ptr(), payload.numel(), plan.start_bit, nsym, out.data_ptr(), end.data_ptr())
    c.sync()
    assert torch.equal(out[:N], x)
    assert int(end[0].item()) == int(starts[-1])
    del x, out, payload, index
    torch.cuda.empty_cache()
