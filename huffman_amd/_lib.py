"""ctypes binding of include/huffman_amd.h (libhuffman_amd.so, built in-tree).

The library is the product: there is no Python or CPU fallback. Loading
fails loudly when the .so has not been built.
"""
import ctypes
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
# HZ_LIB_VARIANT=<dir> loads <pkg>/<dir>/libhuffman_amd.so (kernel A/B builds, tools/); never a fallback
LIB_PATH = os.path.join(_PKG, os.environ.get("HZ_LIB_VARIANT", "lib"), "libhuffman_amd.so")
BIN_DIR = os.path.join(_PKG, "bin")

HZ_NSYM = 65536
HZ_MAXLEN = 56

STATUS = {
    0: "HZ_OK", -1: "HZ_EINVAL", -2: "HZ_ENOMEM", -3: "HZ_EHIP", -4: "HZ_ETOOLONG",
    -5: "HZ_EFORMAT", -6: "HZ_ECAP", -7: "HZ_ETIMEOUT", -8: "HZ_EIO", -9: "HZ_ENODEV", -10: "HZ_ENOENT",
}
STAGE_HIST, STAGE_PACK, STAGE_DECODE, STAGE_INDEX, STAGE_EXTRACT = 0, 1, 2, 3, 4


class HZError(RuntimeError):
    def __init__(self, status, where=""):
        self.status = status
        super().__init__(f"{where}: {STATUS.get(status, status)} ({_strerror(status)})")


class Codebook(ctypes.Structure):
    _fields_ = [
        ("nsym", ctypes.c_uint32),
        ("max_len", ctypes.c_uint32),
        ("min_len", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
        ("order", ctypes.c_uint16 * HZ_NSYM),
        ("len", ctypes.c_uint8 * HZ_NSYM),
        ("code", ctypes.c_uint64 * HZ_NSYM),
    ]


class HeaderInfo(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("payload_byte", ctypes.c_uint64),
        ("payload_bit", ctypes.c_uint32),
        ("is_odd", ctypes.c_uint32),
        ("last_byte", ctypes.c_uint32),
        ("nsym", ctypes.c_uint32),
    ]


_P = ctypes.c_void_p
_U64 = ctypes.c_uint64
_U32 = ctypes.c_uint32
_I = ctypes.c_int

class StreamTiming(ctypes.Structure):
    """hz_stream_timing: stage split of the thread's last streamed archive / extract."""
    _fields_ = [("total_ms", ctypes.c_double), ("fread_ms", ctypes.c_double), ("fwrite_ms", ctypes.c_double),
                ("alloc_ms", ctypes.c_double), ("host_ms", ctypes.c_double), ("h2d_ms", ctypes.c_double), ("kernel_ms", ctypes.c_double),
                ("d2h_ms", ctypes.c_double), ("bytes_in", ctypes.c_uint64), ("bytes_out", ctypes.c_uint64)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


# (name, restype, argtypes): exactly the entry points include/huffman_amd.h declares.
PROTOTYPES = [
    ("hz_strerror", ctypes.c_char_p, [_I]),
    ("hz_version", _I, []),
    ("hz_ctx_create", _I, [_I, _P, ctypes.POINTER(_P)]),
    ("hz_ctx_destroy", _I, [_P]),
    ("hz_ctx_set_stream", _I, [_P, _P]),
    ("hz_ctx_sync", _I, [_P]),
    ("hz_hist16", _I, [_P, _P, _U64, _P, _I]),
    ("hz_codebook_build", _I, [_P, ctypes.POINTER(Codebook)]),
    ("hz_codebook_build_device", _I, [_P, _P, _P]),
    ("hz_header_write_device", _I, [_P, _P, _U64, ctypes.c_uint8, _P, _U64, _P]),
    ("hz_header_parse_device", _I, [_P, _P, _U64, _P, _P]),
    ("hz_header_bits", _I, [ctypes.POINTER(Codebook), _U64, ctypes.POINTER(_U64)]),
    ("hz_payload_bits", _I, [ctypes.POINTER(Codebook), _P, ctypes.POINTER(_U64)]),
    ("hz_header_write", _I, [ctypes.POINTER(Codebook), _U64, ctypes.c_uint8, _P, _U64, ctypes.POINTER(_U64),
                             ctypes.POINTER(_U32), ctypes.POINTER(ctypes.c_uint8)]),
    ("hz_header_parse", _I, [_P, _U64, ctypes.POINTER(Codebook), ctypes.POINTER(HeaderInfo)]),
    ("hz_codebook_upload", _I, [_P, ctypes.POINTER(Codebook)]),
    ("hz_codebook_upload_encode", _I, [_P, ctypes.POINTER(Codebook)]),
    ("hz_codebook_upload_decode", _I, [_P, ctypes.POINTER(Codebook)]),
    ("hz_index_format", _I, []),
    ("hz_index_stride", _U64, []),
    ("hz_index_bytes", _U64, [_U64]),
    ("hz_scratch_bytes", _U64, [_U64]),
    ("hz_pack", _I, [_P, _P, _U64, _U64, _U32, _P, _U64, _P]),
    ("hz_ranges_bytes", _U64, [_U64]),
    ("hz_hist16_ranges", _I, [_P, _P, _U64, _P, _I, _P]),
    ("hz_pack_ranges", _I, [_P, _P, _U64, _U64, _U32, _P, _U64, _P, _P]),
    ("hz_last_pack_ranges", _I, [_P]),
    ("hz_decode", _I, [_P, _P, _U64, _U64, _P, _P]),
    ("hz_index_build", _I, [_P, _P, _U64, _U64, _U64, _P]),
    ("hz_decode_indexless", _I, [_P, _P, _U64, _U64, _U64, _P, _P]),
    ("hz_indexless_scan", _I, [_P, _P, _U64, _U64, _U64, _U64, _U64, _U64, _U64, _P]),
    ("hz_indexless_refix", _I, [_P, _U64, _P]),
    ("hz_indexless_decode", _I, [_P, _U64, _P, _P]),
    ("hz_last_kernel_ms", _I, [_P, _I, ctypes.POINTER(ctypes.c_float)]),
    ("hz_generate", _I, [_P, _P, _U64, _U64, _I, ctypes.c_double, _U64]),
    ("hz_archive_file", _I, [ctypes.c_char_p, _I]),
    ("hz_archive_stream", _I, [ctypes.c_char_p, ctypes.c_char_p, _U64, _I]),
    ("hz_extract_stream", _I, [ctypes.c_char_p, ctypes.c_char_p, _U64, _I]),
    ("hz_extract_file", _I, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, _I]),
    ("hz_stream_last_timing", _I, [ctypes.POINTER(StreamTiming)]),
    ("hz_encode_host", _I, [_P, _U64, _P, _U64, ctypes.POINTER(_U64)]),
    ("hz_encoded_size", _I, [_P, _U64, ctypes.POINTER(_U64)]),
    ("hz_decode_host", _I, [_P, _U64, _P, _U64, ctypes.POINTER(_U64)]),
]

_lib = None


def build_id():
    """Source hash the in-tree library was built from (huffman_amd/build.py), or None."""
    path = os.path.join(os.path.dirname(LIB_PATH), "BUILD_ID")
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def load():
    """Load libhuffman_amd.so (building nothing). Raises ImportError if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python huffman_amd/build.py` "
                          "(the HIP library is required; there is no fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    variant = "HZ_LIB_VARIANT" in os.environ  # an A/B build of older sources may lack newer entry points
    for name, res, args in PROTOTYPES:
        if variant and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _strerror(status):
    try:
        return load().hz_strerror(status).decode()
    except Exception:  # pragma: no cover - only when the library is absent
        return "?"


def check(status, where):
    if status != 0:
        raise HZError(status, where)
    return status
