"""MI355X-native Huffman codec (gfx950): drop-in for yechuan51/huffman's
`archive` / `extract` path. See DESIGN.md and include/huffman_amd.h."""
from ._lib import HZError, LIB_PATH, BIN_DIR, load  # noqa: F401
from .codec import (Device, archive, archive_stream, build_codebook, codebook_arrays, decode, encode, extract, extract_stream, stream_timing,  # noqa: F401
                    header_bits, index_bytes, index_starts, parse_header, payload_bits, write_header)

__all__ = ["Device", "HZError", "archive", "archive_stream", "extract", "extract_stream", "stream_timing", "encode", "decode", "build_codebook", "codebook_arrays",
           "header_bits", "payload_bits", "write_header", "parse_header", "index_bytes", "index_starts", "load", "LIB_PATH",
           "BIN_DIR"]
