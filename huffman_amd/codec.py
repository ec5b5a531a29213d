"""Host-side mirror of the reference's interface for the Huffman path.

The reference exposes two executables:
  archive <file>             -> <file>.compressed          (Compressor.cu:315-632)
  extract <file.compressed>  -> ./DECOMPRESSED_FILE[(k)]   (Decompressor.cu:47-114)
`archive()` / `extract()` here are those entry points (same outputs, same
file names); `encode()` / `decode()` are their in-memory forms; `Device`
exposes the stages on device pointers (calculateFrequency -> hist16,
gpuCodebookConstruction -> build_codebook, populateCWLength + scan +
encodeFromCW -> pack, translateFile -> decode). Every call goes to the gfx950
kernels of libhuffman_amd.so.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import Codebook, HeaderInfo, check, load

HZ_NSYM = _lib.HZ_NSYM


def _buf(data):
    arr = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    return arr, arr.ctypes.data_as(ctypes.c_void_p)


def encode(data):
    """Bytes -> complete .compressed image (what `archive` writes)."""
    lib = load()
    arr, p = _buf(data)
    n = arr.size
    need = ctypes.c_uint64()
    check(lib.hz_encoded_size(p, n, ctypes.byref(need)), "hz_encoded_size")
    out = np.empty(max(need.value, 1), dtype=np.uint8)
    got = ctypes.c_uint64()
    check(lib.hz_encode_host(p, n, out.ctypes.data_as(ctypes.c_void_p), out.size, ctypes.byref(got)),
          "hz_encode_host")
    return out[:got.value].tobytes()


def decode(blob):
    """.compressed image -> original bytes (what `extract` writes)."""
    lib = load()
    arr, p = _buf(blob)
    cb, info = parse_header(arr)
    n_out = 2 * (info.n // 2) + (1 if info.is_odd else 0)
    out = np.empty(max(n_out, 1), dtype=np.uint8)
    got = ctypes.c_uint64()
    check(lib.hz_decode_host(p, arr.size, out.ctypes.data_as(ctypes.c_void_p), out.size, ctypes.byref(got)),
          "hz_decode_host")
    return out[:got.value].tobytes()


def archive(path, verbose=True):
    """`archive <path>`: writes <path>.compressed; returns its name."""
    check(load().hz_archive_file(str(path).encode(), int(verbose)), "hz_archive_file")
    return str(path) + ".compressed"


def archive_stream(path, out_path, chunk_bytes=1 << 30, verbose=False):
    """Streaming `archive` with bounded memory (chunks of chunk_bytes)."""
    check(load().hz_archive_stream(str(path).encode(), str(out_path).encode(), chunk_bytes, int(verbose)),
          "hz_archive_stream")
    return str(out_path)


def extract_stream(path, out_path, chunk_bytes=1 << 30, verbose=False):
    """Streaming `extract` with bounded memory (payload windows of chunk_bytes)."""
    check(load().hz_extract_stream(str(path).encode(), str(out_path).encode(), chunk_bytes, int(verbose)),
          "hz_extract_stream")
    return str(out_path)


def stream_timing():
    """Stage split (dict) of this thread's last archive_stream / extract_stream call."""
    from ._lib import StreamTiming
    t = StreamTiming()
    check(load().hz_stream_last_timing(ctypes.byref(t)), "hz_stream_last_timing")
    return t.as_dict()


def extract(path, verbose=True):
    """`extract <path>`: writes ./DECOMPRESSED_FILE (or (k)); returns its name."""
    name = ctypes.create_string_buffer(256)
    check(load().hz_extract_file(str(path).encode(), name, 256, int(verbose)), "hz_extract_file")
    return name.value.decode()


def build_codebook(hist):
    """65 536-entry host histogram -> Codebook with the reference's semantics."""
    h = np.ascontiguousarray(hist, dtype=np.uint64)
    assert h.size == HZ_NSYM
    cb = Codebook()
    check(load().hz_codebook_build(h.ctypes.data_as(ctypes.c_void_p), ctypes.byref(cb)), "hz_codebook_build")
    return cb


def codebook_arrays(cb):
    """(order[U], len[65536], code[65536]) numpy views of a Codebook."""
    order = np.ctypeslib.as_array(cb.order)[:cb.nsym].copy()
    return order, np.ctypeslib.as_array(cb.len).copy(), np.ctypeslib.as_array(cb.code).copy()


def header_bits(cb, n):
    v = ctypes.c_uint64()
    check(load().hz_header_bits(ctypes.byref(cb), n, ctypes.byref(v)), "hz_header_bits")
    return v.value


def payload_bits(cb, hist):
    h = np.ascontiguousarray(hist, dtype=np.uint64)
    v = ctypes.c_uint64()
    check(load().hz_payload_bits(ctypes.byref(cb), h.ctypes.data_as(ctypes.c_void_p), ctypes.byref(v)),
          "hz_payload_bits")
    return v.value


def write_header(cb, n, last_byte=0):
    """-> (complete header bytes, pending bit count, pending byte MSB-aligned)."""
    hb = header_bits(cb, n)
    out = np.zeros(hb // 8 + 8, dtype=np.uint8)
    nb, pb, pend = ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_uint8()
    check(load().hz_header_write(ctypes.byref(cb), n, last_byte, out.ctypes.data_as(ctypes.c_void_p), out.size,
                                 ctypes.byref(nb), ctypes.byref(pb), ctypes.byref(pend)), "hz_header_write")
    return out[:nb.value].tobytes(), pb.value, pend.value


def parse_header(blob):
    arr, p = _buf(blob)
    cb, info = Codebook(), HeaderInfo()
    check(load().hz_header_parse(p, arr.size, ctypes.byref(cb), ctypes.byref(info)), "hz_header_parse")
    return cb, info


def index_bytes(nsym):
    """Bytes of the block index hz_pack writes for nsym symbols (include/huffman_amd.h)."""
    return load().hz_index_bytes(nsym)


def index_starts(index, nsym):
    """The u64 start[] part of a block index (numpy or torch int64 view)."""
    nb = (nsym + load().hz_index_stride() - 1) // load().hz_index_stride()
    return index[:nb + 1]


class Device:
    """Stage API on device pointers (ints), stream-ordered on one HIP stream."""

    def __init__(self, device=0, stream=None):
        self.lib = load()
        h = ctypes.c_void_p()
        check(self.lib.hz_ctx_create(device, ctypes.c_void_p(stream) if stream else None, ctypes.byref(h)),
              "hz_ctx_create")
        self.h = h

    def close(self):
        if self.h:
            self.lib.hz_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream):
        check(self.lib.hz_ctx_set_stream(self.h, ctypes.c_void_p(stream)), "hz_ctx_set_stream")

    def sync(self):
        check(self.lib.hz_ctx_sync(self.h), "hz_ctx_sync")

    def hist16(self, d_in, n, d_hist, accumulate=False):
        check(self.lib.hz_hist16(self.h, d_in, n, d_hist, int(accumulate)), "hz_hist16")

    def codebook_build(self, d_hist, d_cb):
        """Device codebook: d_hist (u64 x 65536) -> d_cb (sizeof(Codebook) bytes)."""
        check(self.lib.hz_codebook_build_device(self.h, d_hist, d_cb), "hz_codebook_build_device")

    def header_write(self, d_cb, n, last_byte, d_out, cap, d_info):
        """Device header writer; d_info: 4 x u64 (bytes, pending bits, pending byte, bits)."""
        check(self.lib.hz_header_write_device(self.h, d_cb, n, last_byte, d_out, cap, d_info), "hz_header_write_device")

    def header_parse(self, d_file, length, d_cb, d_info):
        """Device header parser; d_info: 6 x u64 (n, payload byte, payload bit, odd, last, nsym)."""
        check(self.lib.hz_header_parse_device(self.h, d_file, length, d_cb, d_info), "hz_header_parse_device")

    def upload(self, cb):
        check(self.lib.hz_codebook_upload(self.h, ctypes.byref(cb)), "hz_codebook_upload")

    def upload_encode(self, cb):
        check(self.lib.hz_codebook_upload_encode(self.h, ctypes.byref(cb)), "hz_codebook_upload_encode")

    def upload_decode(self, cb):
        check(self.lib.hz_codebook_upload_decode(self.h, ctypes.byref(cb)), "hz_codebook_upload_decode")

    def pack(self, d_in, n, start_bit, lead, d_out, out_cap, d_index=None):
        check(self.lib.hz_pack(self.h, d_in, n, start_bit, lead, d_out, out_cap, d_index), "hz_pack")

    # -- two-pass encode (range plan): hist16_ranges then pack_ranges on the same input ----------
    def ranges_bytes(self, n):
        """Bytes of the range plan buffer for an n-byte input (0: too small, plain passes)."""
        return self.lib.hz_ranges_bytes(n)

    def hist16_ranges(self, d_in, n, d_hist, d_ranges, accumulate=False):
        check(self.lib.hz_hist16_ranges(self.h, d_in, n, d_hist, int(accumulate), d_ranges), "hz_hist16_ranges")

    def pack_ranges(self, d_in, n, start_bit, lead, d_out, out_cap, d_index, d_ranges):
        check(self.lib.hz_pack_ranges(self.h, d_in, n, start_bit, lead, d_out, out_cap, d_index, d_ranges),
              "hz_pack_ranges")

    def last_pack_ranges(self):
        """1 when the last pack_ranges took the range plan (no count pass), 0 for count + scan + write."""
        return self.lib.hz_last_pack_ranges(self.h)

    def decode(self, d_payload, payload_bytes, nsym, d_index, d_out):
        check(self.lib.hz_decode(self.h, d_payload, payload_bytes, nsym, d_index, d_out), "hz_decode")

    def index_build(self, d_payload, payload_bytes, start_bit, nsym, d_index):
        check(self.lib.hz_index_build(self.h, d_payload, payload_bytes, start_bit, nsym, d_index), "hz_index_build")

    def decode_indexless(self, d_payload, payload_bytes, start_bit, nsym, d_out, d_end_bit=None):
        """Decode an index-less stream (the `extract` path): no block index; d_end_bit (device u64) gets
        the end bit of the last codeword (past payload_bytes * 8: too few codewords)."""
        check(self.lib.hz_decode_indexless(self.h, d_payload, payload_bytes, start_bit, nsym, d_out, d_end_bit),
              "hz_decode_indexless")

    # -- one index-less stream in parts (one per rank; huffman_amd/dist.py decode_indexless_split) -----
    def indexless_scan(self, d_payload, payload_bytes, start_bit, part_begin, part_end, entry_bit, d_summary,
                       nsym=0, payload_bit_base=0):
        """Walk + fix-ups of payload bits [part_begin, part_end) after start_bit; entry_bit: the part's true
        entry or 2**64 - 1 (its walked entry). d_summary (device, 3 x u64): codewords, true exit, entry in
        use. Stream bits throughout; d_payload holds stream bits from payload_bit_base (a rank's slice:
        the part plus HZ_INDEXLESS_LEAD_BITS before it). nsym: the stream's symbols (0: unknown)."""
        check(self.lib.hz_indexless_scan(self.h, d_payload, payload_bytes, payload_bit_base, start_bit, nsym,
                                         part_begin, part_end, entry_bit, d_summary), "hz_indexless_scan")

    def indexless_refix(self, entry_bit, d_summary):
        check(self.lib.hz_indexless_refix(self.h, entry_bit, d_summary), "hz_indexless_refix")

    def indexless_decode(self, nsym, d_out, d_end_bit=None):
        check(self.lib.hz_indexless_decode(self.h, nsym, d_out, d_end_bit), "hz_indexless_decode")

    def generate(self, d_out, n, offset=0, kind=1, alpha=1.1, seed=42):
        check(self.lib.hz_generate(self.h, d_out, n, offset, kind, alpha, seed), "hz_generate")

    def kernel_ms(self, stage):
        v = ctypes.c_float()
        check(self.lib.hz_last_kernel_ms(self.h, stage, ctypes.byref(v)), "hz_last_kernel_ms")
        return v.value
