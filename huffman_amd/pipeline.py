"""Device-resident encode/decode of a byte stream (torch tensors in HBM).

This is the flow `archive` runs, kept on the device end to end so it can be
timed with inputs already resident in HBM (bench.py) and sharded across ranks
(huffman_amd/dist.py):

    hist16 (GPU, + the range plan) -> host codebook + header (reference
    semantics) -> encode table upload -> pack (GPU, one bit stream + decode-unit
    index; range starts from the plan, one pass over the input) -> decode table
    upload (host build overlaps the pack kernel) -> decode (GPU)

PyTorch provides device memory and the stream; every compute stage is a
gfx950 kernel of libhuffman_amd.so.
"""
import time
import weakref

import numpy as np
import torch

from . import _lib
from .codec import Device, build_codebook, header_bits, index_bytes, payload_bits, write_header


class Plan:
    """Codebook and stream geometry for one encode."""

    def __init__(self, cb, n_total, hist_local, first_shard=True, shard_bit_offset=0, last_byte=0):
        self.cb = cb
        self.n_total = n_total
        self.header_bits = header_bits(cb, n_total)
        self.payload_bits = payload_bits(cb, hist_local)        # bits of this shard
        # absolute payload bit where this shard starts (header pending bits first)
        self.stream_bit = self.header_bits % 8 + shard_bit_offset
        self.start_bit = self.stream_bit % 32 if not first_shard else self.stream_bit
        self.first_shard = first_shard
        self.last_byte = last_byte
        self._header = None
        # The header's last header_bits % 8 bits open the payload's first byte.
        # They are the low bits of N's top byte, the last of the 8 N bytes the
        # header ends with (Compressor.cu:487,661-669), so pack needs no header.
        pbits = self.header_bits % 8
        self.lead = ((n_total >> 56) & ((1 << pbits) - 1)) if first_shard else 0
        self.words = (self.start_bit + self.payload_bits + 31) // 32

    @property
    def header(self):
        """Complete header bytes (first shard only); written on first use, so a
        caller can launch pack/decode before paying for it on the host."""
        if self._header is None:
            self._header = b""
            if self.first_shard:
                self._header, pbits, pend = write_header(self.cb, self.n_total, self.last_byte)
                assert ((pend >> (8 - pbits)) if pbits else 0) == self.lead
        return self._header


class _PlanKey:
    """Identity of a histogram's input for its range plan: the very tensor object (a weak
    reference: a freed tensor whose address the caching allocator hands out again never matches),
    its view and its in-place version counter."""

    def __init__(self, x):
        self.ref = weakref.ref(x)
        self.key = (x.data_ptr(), x.numel(), x._version)

    def __eq__(self, other):
        if not isinstance(other, _PlanKey):
            return NotImplemented
        a, b = self.ref(), other.ref()
        return a is not None and a is b and self.key == other.key


class StreamCodec:
    def __init__(self, device_index=0, use_ranges=True):
        self.device = torch.device("cuda", device_index)
        torch.cuda.set_device(self.device)
        # A real (non-null) stream shared by torch and the library, so torch
        # ops and the HIP kernels are ordered on one queue.
        self.stream = torch.cuda.Stream(device=self.device)
        torch.cuda.set_stream(self.stream)
        self.dev = Device(device_index, stream=self.stream.cuda_stream)
        self.hist = torch.zeros(_lib.HZ_NSYM, dtype=torch.int64, device=self.device)
        self.timings = {}
        # two-pass encode (hz_hist16_ranges / hz_pack_ranges): the plan of the last histogram's input
        self.use_ranges = use_ranges
        self.ranges = None
        self._ranges_of = None

    # -- stages ---------------------------------------------------------------
    def histogram(self, x, accumulate=False):
        n = x.numel()
        # the range plan needs a 16-byte aligned input (hz_hist16_ranges); offset views take hz_hist16
        aligned = x.data_ptr() % 16 == 0
        rb = self.dev.ranges_bytes(n) if self.use_ranges and not accumulate and aligned else 0
        if rb:
            if self.ranges is None or self.ranges.numel() < rb:
                self.ranges = torch.empty(rb, dtype=torch.uint8, device=self.device)
            self.dev.hist16_ranges(x.data_ptr(), n, self.hist.data_ptr(), self.ranges.data_ptr(), accumulate)
            self._ranges_of = self._ident(x)
        else:
            self.dev.hist16(x.data_ptr(), n, self.hist.data_ptr(), accumulate)
            self._ranges_of = None
        return self.hist

    @staticmethod
    def _ident(x):
        """What a range plan is valid for: the same tensor's storage, view and contents (its
        in-place version counter), so a reused address or an in-place change falls back to
        count + scan + write instead of packing with stale range starts."""
        return _PlanKey(x)

    def make_plan(self, hist_host, n_total, hist_local=None, first_shard=True, shard_bit_offset=0, last_byte=0,
                  cb=None):
        t0 = time.perf_counter()
        cb = build_codebook(hist_host) if cb is None else cb
        plan = Plan(cb, n_total, hist_host if hist_local is None else hist_local, first_shard, shard_bit_offset,
                    last_byte)
        t1 = time.perf_counter()
        self.dev.upload_encode(cb)   # decode tables follow the pack launch (upload_decode)
        t2 = time.perf_counter()
        self.timings["codebook_ms"] = (t1 - t0) * 1e3
        self.timings["upload_ms"] = (t2 - t1) * 1e3
        return plan

    def upload_decode(self, plan):
        """Decode tables; call after launching pack so the host build overlaps it."""
        t0 = time.perf_counter()
        self.dev.upload_decode(plan.cb)
        self.timings["upload_decode_ms"] = (time.perf_counter() - t0) * 1e3

    def alloc_payload(self, plan, nsym):
        out = torch.empty(max(plan.words, 1) * 4 + 16, dtype=torch.uint8, device=self.device)
        index = torch.empty(max((index_bytes(nsym) + 7) // 8, 1), dtype=torch.int64, device=self.device)
        return out, index

    def pack(self, x, plan, out, index):
        """Pack x; with the range plan of x's histogram (the last histogram() call, same tensor,
        unchanged since: stream order) in one pass over x, else count + scan + write. A plan is
        used once. index may be None: no block index is written (the drop-in file path)."""
        iptr = index.data_ptr() if index is not None else 0
        if x.data_ptr() % 16:
            # hz_pack reads 16-byte vectors (include/huffman_amd.h): an unaligned view is packed from an
            # aligned copy (its histogram took hz_hist16, so there is no range plan to match)
            x = x.clone()
        if self._ranges_of is not None and self._ranges_of == self._ident(x):
            self._ranges_of = None
            self.dev.pack_ranges(x.data_ptr(), x.numel(), plan.start_bit, plan.lead, out.data_ptr(), out.numel(),
                                 iptr, self.ranges.data_ptr())
        else:
            self.dev.pack(x.data_ptr(), x.numel(), plan.start_bit, plan.lead, out.data_ptr(), out.numel(), iptr)
        return out

    def decode(self, payload, nsym, index, out):
        self.dev.decode(payload.data_ptr(), payload.numel(), nsym, index.data_ptr(), out.data_ptr())
        return out

    def sync(self):
        self.dev.sync()

    def kernel_ms(self):
        return {
            "hist": self.dev.kernel_ms(_lib.STAGE_HIST),
            "pack": self.dev.kernel_ms(_lib.STAGE_PACK),
            "decode": self.dev.kernel_ms(_lib.STAGE_DECODE),
        }

    # -- whole stream (one device) ----------------------------------------------
    def encode(self, x):
        """Encode a device tensor. Returns (plan, payload tensor, index tensor)."""
        n = x.numel()
        self.histogram(x)
        h = self.hist.cpu().numpy().view(np.uint64)
        last = int(x[-1].item()) if n % 2 else 0
        plan = self.make_plan(h, n, last_byte=last)
        out, index = self.alloc_payload(plan, n // 2)
        if n // 2:
            self.pack(x, plan, out, index)
        self.upload_decode(plan)
        return plan, out, index

    def file_image(self, plan, payload):
        """Complete .compressed bytes (header + payload) on the host."""
        total = plan.header_bits + plan.payload_bits
        nbytes = (total + 7) // 8 - plan.header_bits // 8
        pay = payload[:nbytes].cpu().numpy().tobytes() if nbytes else b""
        if not pay and plan.header_bits % 8:
            pay = bytes([plan.lead << (8 - plan.header_bits % 8)])
        return plan.header + pay
