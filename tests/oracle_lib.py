"""ctypes wrapper of oracle/hz_oracle.c -- the CHECKER used by tests only."""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "_build", "libhzoracle.so")
REF_DIR = os.path.join(ORACLE_DIR, "_ref")

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    srcs = [os.path.join(ORACLE_DIR, f) for f in ("hz_oracle.c", "compressor_literal.c")]
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(f) for f in srcs):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    lib = ctypes.CDLL(LIB)
    P, U64 = ctypes.c_void_p, ctypes.c_uint64
    lib.hzo_hist16.argtypes = [P, U64, P]
    lib.hzo_codebook.argtypes = [P, P, P, P]
    lib.hzo_codebook.restype = ctypes.c_int
    lib.hzo_encode.argtypes = [P, U64, P, U64, ctypes.POINTER(U64)]
    lib.hzo_encode.restype = ctypes.c_int
    lib.hzo_decode.argtypes = [P, U64, P, U64, ctypes.POINTER(U64)]
    lib.hzo_decode.restype = ctypes.c_int
    lib.hzo_pack_range.argtypes = [P, U64, U64, P, P, U64, P]
    lib.hzo_parse_header.argtypes = [P, U64, P, P, P, P]
    lib.hzo_parse_header.restype = ctypes.c_int
    lib.hzo_encoded_bits.argtypes = [U64, ctypes.c_uint32, P, P, ctypes.POINTER(U64)]
    lib.hzo_encoded_bits.restype = U64
    lib.hzo_zipf_thresholds.argtypes = [ctypes.c_double, P]
    lib.hzo_walk.argtypes = [P, U64, P, P, U64, U64, U64, P, ctypes.POINTER(U64)]
    lib.hzo_walk.restype = ctypes.c_int64
    lib.hzo_gen.argtypes = [P, U64, U64, ctypes.c_int, U64, P]
    I64 = ctypes.c_int64
    lib.hzl_archive.argtypes = [P, U64, P, ctypes.c_uint32, P, P, P, U64, P, ctypes.POINTER(I64), ctypes.POINTER(I64)]
    lib.hzl_archive.restype = I64
    lib.hzl_header.argtypes = [U64, ctypes.c_uint8, P, ctypes.c_uint32, P, P, P, U64, ctypes.POINTER(ctypes.c_uint32),
                               ctypes.POINTER(ctypes.c_uint8)]
    lib.hzl_header.restype = I64
    _lib = lib
    return lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def as_u8(data):
    return np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else data,
                                dtype=np.uint8)


def hist16(data):
    a = as_u8(data)
    h = np.zeros(65536, dtype=np.uint64)
    load().hzo_hist16(_p(a), a.size, _p(h))
    return h


def codebook(hist):
    h = np.ascontiguousarray(hist, dtype=np.uint64)
    order = np.zeros(65536, dtype=np.uint16)
    ln = np.zeros(65536, dtype=np.uint8)
    code = np.zeros(65536, dtype=np.uint64)
    U = load().hzo_codebook(_p(h), _p(order), _p(ln), _p(code))
    if U < 0:
        raise RuntimeError(f"hzo_codebook {U}")
    return order[:U].copy(), ln, code


def encode(data):
    a = as_u8(data)
    cap = 2 * a.size + 400000
    out = np.zeros(cap, dtype=np.uint8)
    n = ctypes.c_uint64()
    rc = load().hzo_encode(_p(a), a.size, _p(out), cap, ctypes.byref(n))
    if rc:
        raise RuntimeError(f"hzo_encode {rc}")
    return out[:n.value].tobytes()


def decode(blob, cap=None):
    a = as_u8(blob)
    cap = cap if cap is not None else 16 * a.size + 1024
    out = np.zeros(max(cap, 1), dtype=np.uint8)
    n = ctypes.c_uint64()
    rc = load().hzo_decode(_p(a), a.size, _p(out), out.size, ctypes.byref(n))
    if rc:
        raise RuntimeError(f"hzo_decode {rc}")
    return out[:n.value].tobytes()


def reference_archive(data, order, ln, code):
    """Literal Compressor.cu file writer (oracle/compressor_literal.c), defects
    B1/B2 included: -> (file bytes, undefined-byte flags, B1 byte offset or -1,
    B2 byte offset or -1). order/ln/code: the codebook as the reference host
    holds it (header order; length and right-aligned code per symbol value)."""
    a = as_u8(data)
    order = np.ascontiguousarray(order, dtype=np.uint16)
    ln = np.ascontiguousarray(ln, dtype=np.uint8)
    code = np.ascontiguousarray(code, dtype=np.uint64)
    cap = 3 * a.size + 400000
    out = np.zeros(cap, dtype=np.uint8)
    flags = np.zeros(cap, dtype=np.uint8)
    b1, b2 = ctypes.c_int64(), ctypes.c_int64()
    n = load().hzl_archive(_p(a), a.size, _p(order), order.size, _p(ln), _p(code), _p(out), cap, _p(flags),
                           ctypes.byref(b1), ctypes.byref(b2))
    if n < 0:
        raise RuntimeError(f"hzl_archive {n}")
    return out[:n].tobytes(), flags[:n].copy(), b1.value, b2.value


def reference_header(n, last_byte, order, ln, code):
    """Literal Compressor.cu header writer (:431-487) -> (complete header bytes,
    pending bit count, pending bits MSB-aligned)."""
    order = np.ascontiguousarray(order, dtype=np.uint16)
    ln = np.ascontiguousarray(ln, dtype=np.uint8)
    code = np.ascontiguousarray(code, dtype=np.uint64)
    cap = 16 + order.size * 11
    out = np.zeros(cap, dtype=np.uint8)
    pb, pend = ctypes.c_uint32(), ctypes.c_uint8()
    k = load().hzl_header(n, last_byte, _p(order), order.size, _p(ln), _p(code), _p(out), cap, ctypes.byref(pb),
                          ctypes.byref(pend))
    if k < 0:
        raise RuntimeError(f"hzl_header {k}")
    return out[:k].tobytes(), pb.value, pend.value


def parse_header(blob):
    """Oracle header parse (Decompressor.cu:65-103): (order[:U], len, code,
    [N, payload byte, payload bit, isOdd, lastByte, U]); raises ValueError on a
    malformed or truncated header."""
    a = as_u8(blob)
    order = np.zeros(65536, dtype=np.uint16)
    ln = np.zeros(65536, dtype=np.uint8)
    code = np.zeros(65536, dtype=np.uint64)
    info = np.zeros(6, dtype=np.uint64)
    rc = load().hzo_parse_header(_p(a), a.size, _p(order), _p(ln), _p(code), _p(info))
    if rc:
        raise ValueError(f"hzo_parse_header: {rc}")
    u = int(info[5])
    return order[:u], ln, code, [int(v) for v in info]


def pack_range(data, sym0, count, ln, code, bit0, nbytes):
    a = as_u8(data)
    out = np.zeros(nbytes, dtype=np.uint8)
    load().hzo_pack_range(_p(a), sym0, count, _p(np.ascontiguousarray(ln)), _p(np.ascontiguousarray(code)), bit0,
                          _p(out))
    return out


def zipf_thresholds(alpha=1.1):
    t = np.zeros(256, dtype=np.uint64)
    load().hzo_zipf_thresholds(alpha, _p(t))
    return t


def generate(n, offset=0, kind=1, seed=42, alpha=1.1):
    t = zipf_thresholds(alpha)
    out = np.zeros(n, dtype=np.uint8)
    load().hzo_gen(_p(out), n, offset, kind, seed, _p(t))
    return out


def ref_binary(name):
    p = os.path.join(REF_DIR, name)
    return p if os.path.exists(p) else None


def walk(payload, ln, code, pos, end, max_count=(1 << 63), decode=False):
    """hzo_walk: codewords from stream bit pos (any bit) while below end; (count, exit bit, symbols or None)."""
    lib = load()
    p = as_u8(payload)
    ln = np.ascontiguousarray(ln, dtype=np.uint8)
    code = np.ascontiguousarray(code, dtype=np.uint64)
    cap = min(max_count, (max(end - pos, 0) + 1))
    out = np.zeros(2 * cap + 2, dtype=np.uint8) if decode else None
    ex = ctypes.c_uint64()
    n = lib.hzo_walk(_p(p), p.size, _p(ln), _p(code), pos, end, max_count, _p(out) if decode else None, ctypes.byref(ex))
    if n < 0:
        raise RuntimeError("hzo_walk failed")
    return n, ex.value, (out[:2 * n] if decode else None)
