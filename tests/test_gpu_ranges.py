"""Two-pass encode (the range plan, include/huffman_amd.h hz_hist16_ranges /
hz_pack_ranges) against the three-pass encode (hz_hist16 + hz_pack: count pass,
scan, write) on the same inputs: the same histogram, and the same payload and
block index byte for byte; the plan path is the one that ran (no silent
fallback). The three-pass path itself is pinned against the oracle in
test_gpu.py; the 256 MiB and 4 GiB pipeline tests there now run through the
plan as well.

Tolerance: none -- every check is bit-exact (integer/bit work)."""
import numpy as np
import pytest

import oracle_lib

pytestmark = pytest.mark.gpu

MIB = 1 << 20


@pytest.fixture(scope="module")
def dev(built_lib):
    from huffman_amd.codec import Device
    return Device(0)


def _zipf(n, seed):
    import torch
    from huffman_amd.codec import Device
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    d = Device(0)
    d.generate(x.data_ptr(), n, offset=0, kind=1, alpha=1.1, seed=seed)
    d.sync()
    return x


def _skewed(n, seed):
    """90 % of symbols 0x0000: the hot counter wraps (65 536) inside every range, so
    the plan's carry records are exercised; DENSE tables (few symbols, short codes)."""
    import torch
    rng = np.random.default_rng(seed)
    sym = np.where(rng.random(n // 2) < 0.9, 0, rng.integers(1, 300, n // 2)).astype("<u2")
    host = sym.view(np.uint8)
    if n % 2:
        host = np.concatenate([host, np.array([7], np.uint8)])
    return torch.from_numpy(host).cuda()


def _fib_wide(n_target, seed):
    """Fibonacci counts (scaled): codes up to 28 bits, WIDE tables."""
    import torch
    fib = [1, 1]
    while len(fib) < 29:
        fib.append(fib[-1] + fib[-2])
    base = np.repeat(np.arange(len(fib), dtype=np.uint16) * 257 + 3, fib)
    np.random.default_rng(seed).shuffle(base)
    reps = max(1, n_target // (2 * base.size))
    return torch.from_numpy(np.tile(base, reps).astype("<u2").view(np.uint8)).cuda()


def _both(dev, x, start_bit, lead):
    """(hist, payload, index) by the three-pass encode and by the range plan."""
    import torch
    from huffman_amd import build_codebook, index_bytes, payload_bits
    n = x.numel()
    nsym = n // 2
    hist = torch.zeros(65536, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # torch's fills / copies are on torch's stream, the library's calls on dev's
    dev.hist16(x.data_ptr(), n, hist.data_ptr())
    dev.sync()
    h = hist.cpu().numpy().view(np.uint64).copy()
    cb = build_codebook(h)
    dev.upload_encode(cb)
    words = (start_bit + payload_bits(cb, h) + 31) // 32 + 4
    res = []
    for plan in (False, True):
        out = torch.full((4 * words,), 0xA5, dtype=torch.uint8, device="cuda")
        idx = torch.full(((index_bytes(nsym) + 7) // 8 + 1,), -1, dtype=torch.int64, device="cuda")
        if plan:
            rb = dev.ranges_bytes(n)
            ranges = torch.empty(max(rb, 16), dtype=torch.uint8, device="cuda")
            hist2 = torch.zeros(65536, dtype=torch.int64, device="cuda")
            torch.cuda.synchronize()
            dev.hist16_ranges(x.data_ptr(), n, hist2.data_ptr(), ranges.data_ptr())
            dev.pack_ranges(x.data_ptr(), n, start_bit, lead, out.data_ptr(), out.numel(), idx.data_ptr(),
                            ranges.data_ptr())
            took = dev.last_pack_ranges()
            dev.sync()
            res.append((hist2.cpu().numpy().view(np.uint64).copy(), out.cpu().numpy(), idx.cpu().numpy(), took, rb))
        else:
            torch.cuda.synchronize()
            dev.pack(x.data_ptr(), n, start_bit, lead, out.data_ptr(), out.numel(), idx.data_ptr())
            dev.sync()
            res.append((h, out.cpu().numpy(), idx.cpu().numpy(), 0, 0))
    nb = index_bytes(nsym)
    return res, nb, cb


@pytest.mark.parametrize("kind,n,start_bit,lead", [
    ("zipf", 256 * MIB + 3, 5, 0x1b),          # HOT tables, odd n, header pending bits
    ("zipf", 768 * MIB + 4098, 32 * 7 + 13, 0),  # 3 ranges per histogram workgroup
    ("skewed", 256 * MIB + 4096 * 3 + 2, 0, 0),  # DENSE tables, counter wraps in every range
    ("wide", 300 * MIB, 3, 0x5),               # WIDE tables (codes > 25 bits)
])
def test_range_plan_equals_three_pass(dev, kind, n, start_bit, lead):
    import torch
    x = {"zipf": lambda: _zipf(n, 9), "skewed": lambda: _skewed(n, 4), "wide": lambda: _fib_wide(n, 2)}[kind]()
    n = x.numel()
    ((h3, p3, i3, _, _), (hr, pr, ir, took, rb)), nb, cb = _both(dev, x, start_bit, lead)
    assert rb > 0
    assert took == 1, "the range plan did not run"
    assert np.array_equal(h3, hr)
    assert int(h3.sum()) == n // 2
    assert np.array_equal(p3, pr)
    assert np.array_equal(i3.view(np.uint8)[:nb], ir.view(np.uint8)[:nb])
    del x
    torch.cuda.empty_cache()


def test_range_plan_small_input_is_three_pass(dev):
    """Below 256 MiB there is no plan: hz_ranges_bytes is 0 and the calls are hz_hist16 / hz_pack."""
    import torch
    x = _zipf(64 * MIB + 1, 3)
    assert dev.ranges_bytes(x.numel()) == 0
    ((h3, p3, i3, _, _), (hr, pr, ir, took, rb)), nb, _ = _both(dev, x, 0, 0)
    assert took == 0 and rb == 0
    assert np.array_equal(h3, hr) and np.array_equal(p3, pr)
    assert np.array_equal(i3.view(np.uint8)[:nb], ir.view(np.uint8)[:nb])
    del x
    torch.cuda.empty_cache()


def test_range_plan_pipeline_matches_oracle_slices(built_lib):
    """StreamCodec (the bench's flow) through the plan: the whole 256 MiB + 2 file equals the oracle's."""
    import torch
    from huffman_amd.pipeline import StreamCodec
    c = StreamCodec(0)
    n = 256 * MIB + 2
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    c.dev.generate(x.data_ptr(), n, offset=0, kind=1, alpha=1.1, seed=42)
    plan, payload, index = c.encode(x)
    assert c.dev.last_pack_ranges() == 1
    host = x.cpu().numpy()
    assert c.file_image(plan, payload) == oracle_lib.encode(host)
    del x
    torch.cuda.empty_cache()


def test_unaligned_view_of_256mib_encodes_like_an_aligned_copy(built_lib):
    """An input view that is not 16-byte aligned (no range plan: hz_hist16 + count + scan + write)
    encodes to the same payload and index as an aligned copy of the same bytes (the range plan), and
    decodes back (the range plan must not be taken for unaligned inputs)."""
    import torch
    from huffman_amd.pipeline import StreamCodec
    codec = StreamCodec(0)
    n = (256 << 20) + 2
    big = torch.empty(n + 32, dtype=torch.uint8, device="cuda")
    codec.dev.generate(big.data_ptr(), n + 32, offset=0, kind=1, alpha=1.1, seed=17)
    view = big[3:3 + n]
    assert view.data_ptr() % 16 != 0
    plan_u, pay_u, idx_u = codec.encode(view)
    codec.sync()
    copy = view.clone()
    assert copy.data_ptr() % 16 == 0
    plan_a, pay_a, idx_a = codec.encode(copy)
    codec.sync()
    assert plan_u.payload_bits == plan_a.payload_bits
    nbytes = (plan_a.payload_bits + plan_a.start_bit + 7) // 8
    assert torch.equal(pay_u[:nbytes], pay_a[:nbytes])
    assert torch.equal(idx_u, idx_a)
    out = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    codec.decode(pay_u, n // 2, idx_u, out)
    codec.sync()
    assert torch.equal(out[:n], copy)


def test_range_plan_blocks_over_the_slot_match_oracle(dev):
    """Blocks larger than a pack wave's LDS slot (runs of rare symbols, ~20-bit codes, in a Zipf
    stream) and the stream's partial last block leave k_pack_write for k_pack_cold's list: spans at
    block-aligned and unaligned offsets in several ranges, one covering the last block. The range
    plan and the three-pass encode agree byte for byte (payload and block index), the plan's file
    equals the oracle's, and the stream decodes back."""
    import torch
    from huffman_amd.pipeline import StreamCodec
    n = 256 * MIB + 2 * 777 + 1
    x = _zipf(n, 5)
    host = x.cpu().numpy()
    sym = host[: n - 1].view("<u2")
    rng = np.random.default_rng(3)
    nsym = sym.size
    for s0, ln in [(2048 * 7, 2048 * 3), (2048 * 4001 + 100, 5000), (nsym // 2 + 33, 2048 * 9 + 17),
                   (nsym - 2048 * 2 - 5, 2048 * 2 + 5)]:
        sym[s0:s0 + ln] = rng.integers(20000, 65536, ln)
    x.copy_(torch.from_numpy(host))
    torch.cuda.synchronize()
    ((h3, p3, i3, _, _), (hr, pr, ir, took, _)), nb, _ = _both(dev, x, 0, 0)
    assert took == 1, "the range plan did not run"
    assert np.array_equal(p3, pr)
    assert np.array_equal(i3.view(np.uint8)[:nb], ir.view(np.uint8)[:nb])
    c = StreamCodec(0)
    plan, payload, index = c.encode(x)
    assert c.dev.last_pack_ranges() == 1
    assert c.file_image(plan, payload) == oracle_lib.encode(host)
    out = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    c.decode(payload, nsym, index, out)
    c.sync()
    assert torch.equal(out[: n - 1], x[: n - 1])
    del x, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n", [256 * MIB + 6, 8 * MIB + 3])
def test_dense_without_slots_matches_oracle(built_lib, n):
    """Symbols uniform over 40 000 values: codes of 15 and 16 bits, a DENSE table (max_len 16) whose
    mean code (~15.3 bits) leaves no room for output slots beside it, so k_pack_write keeps the
    direct path in its loop (no cold list); the range plan (256 MiB) and the three-pass encode
    (8 MiB) both equal the oracle's file and decode back."""
    import torch
    from huffman_amd.pipeline import StreamCodec
    rng = np.random.default_rng(n)
    sym = rng.integers(0, 40000, n // 2).astype("<u2")
    host = sym.view(np.uint8)
    if n % 2:
        host = np.concatenate([host, np.array([0x5a], np.uint8)])
    x = torch.from_numpy(host).cuda()
    c = StreamCodec(0)
    plan, payload, index = c.encode(x)
    assert int(plan.cb.max_len) == 16 and int(plan.cb.min_len) < 16  # DENSE, not FIXED16
    assert c.dev.last_pack_ranges() == (1 if n >= 256 * MIB else 0)
    assert c.file_image(plan, payload) == oracle_lib.encode(host)
    out = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    c.decode(payload, n // 2, index, out)
    c.sync()
    assert torch.equal(out[: n - (n & 1)], x[: n - (n & 1)])
    del x, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n,rare", [(256 * MIB + 4, 16000), (8 * MIB + 1, 8000)])
def test_dense_blocks_over_the_slot_match_oracle(built_lib, n, rare):
    """A DENSE table with output slots (90 % zeros, the rest over 8 000 / 16 000 symbols: codes of 1
    and 13-15 bits, 768-word slots sized for ~2.3 bits per symbol) and spans of rare symbols only,
    whose blocks (~900-960 words) exceed a slot: k_pack_cold packs them and the stream's last block.
    The range plan (256 MiB) and the three-pass encode (8 MiB) equal the oracle's file and decode back."""
    import torch
    from huffman_amd.pipeline import StreamCodec
    rng = np.random.default_rng(n)
    nsym = n // 2
    sym = np.where(rng.random(nsym) < 0.9, 0, rng.integers(1, rare + 1, nsym)).astype("<u2")
    for s0 in (2048 * 3 + 5, nsym // 3, nsym - 2048 * 3 - 7):
        sym[s0:s0 + 2048 * 2 + 100] = rng.integers(1, rare + 1, 2048 * 2 + 100)
    host = sym.view(np.uint8)
    if n % 2:
        host = np.concatenate([host, np.array([0x21], np.uint8)])
    x = torch.from_numpy(host).cuda()
    c = StreamCodec(0)
    plan, payload, index = c.encode(x)
    assert int(plan.cb.max_len) <= 16 and int(plan.cb.min_len) < 16  # DENSE
    assert c.dev.last_pack_ranges() == (1 if n >= 256 * MIB else 0)
    assert c.file_image(plan, payload) == oracle_lib.encode(host)
    out = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    c.decode(payload, nsym, index, out)
    c.sync()
    assert torch.equal(out[: n - (n & 1)], x[: n - (n & 1)])
    del x, out
    torch.cuda.empty_cache()
