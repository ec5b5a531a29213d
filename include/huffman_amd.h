/*
 * huffman_amd.h -- C ABI of the MI355X-native Huffman codec (gfx950 / CDNA4).
 *
 * Drop-in boundary for the reference yechuan51/huffman path: the `archive` /
 * `extract` executables and their on-disk `.compressed` format. The reference
 * has no library API; every entry point below replaces one
 * stage of Compressor.cu / Decompressor.cu, cited per function.
 *
 * Conventions
 *   - Plain pointers and sizes only. `d_*` arguments are device pointers
 *     (hipMalloc / torch CUDA tensors) and are used stream-ordered on the
 *     context's stream; host arguments are plain host memory.
 *   - The caller owns every buffer. A context owns only its scratch, its
 *     device code tables and (optionally) its stream.
 *   - Errors: negative HZ_E* status, never abort(). hz_strerror() names them.
 *   - Threading: one context per device per host thread.
 *   - Symbols are 16-bit little-endian byte pairs (Compressor.cu:45); an odd
 *     trailing byte is carried raw in the header (Compressor.cu:339-351).
 */
#ifndef HUFFMAN_AMD_H
#define HUFFMAN_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HZ_NSYM 65536  /* alphabet: every u16 value (Compressor.cu:323 kMaxSymbolSize) */
#define HZ_MAXLEN 56   /* longest supported code (needs > ~5e11 symbols to exceed) */

enum {
    HZ_OK = 0,
    HZ_EINVAL = -1,    /* bad argument / alignment */
    HZ_ENOMEM = -2,    /* host or device allocation failed */
    HZ_EHIP = -3,      /* HIP runtime error */
    HZ_ETOOLONG = -4,  /* a code longer than HZ_MAXLEN bits */
    HZ_EFORMAT = -5,   /* malformed or truncated .compressed stream */
    HZ_ECAP = -6,      /* output capacity too small */
    HZ_ETIMEOUT = -7,  /* a device-side wait exceeded its bound (reserved) */
    HZ_EIO = -8,       /* file I/O error */
    HZ_ENODEV = -9,    /* no usable gfx950 device */
    HZ_ENOENT = -10    /* input file does not exist (the reference CLIs exit 0 on it) */
};

/* Codebook in the reference's order and bit conventions. */
typedef struct hz_codebook {
    uint32_t nsym;              /* U, number of symbols with nonzero count */
    uint32_t max_len;           /* longest code */
    uint32_t min_len;           /* shortest code */
    uint32_t reserved;
    uint16_t order[HZ_NSYM];    /* header order: (count asc, symbol asc) */
    uint8_t len[HZ_NSYM];       /* code length per symbol value (0 = absent) */
    uint64_t code[HZ_NSYM];     /* code per symbol, right aligned; first bit = MSB */
} hz_codebook;

/* Parsed .compressed header (Decompressor.cu:65-103). */
typedef struct hz_header_info {
    uint64_t n;                 /* original size in bytes */
    uint64_t payload_byte;      /* file byte holding the first payload bit */
    uint32_t payload_bit;       /* bit (MSB = 0) of that byte where the payload starts */
    uint32_t is_odd;
    uint32_t last_byte;
    uint32_t nsym;
} hz_header_info;

typedef struct hz_ctx hz_ctx;

const char *hz_strerror(int status);
int hz_version(void);

/* Context: device + stream (stream may be NULL: the context creates its own). */
int hz_ctx_create(int device, void *stream, hz_ctx **out);
int hz_ctx_destroy(hz_ctx *ctx);
int hz_ctx_set_stream(hz_ctx *ctx, void *stream);
int hz_ctx_sync(hz_ctx *ctx);

/* ---- encode stages ----------------------------------------------------- */

/* 65 536-bin histogram of the u16 symbols of d_in[0..n) into d_hist (u64 x
 * 65536); accumulate != 0 adds to d_hist instead of overwriting.
 * Replaces calculateFrequency (Compressor.cu:38-48, launch :369-372). */
int hz_hist16(hz_ctx *ctx, const uint8_t *d_in, uint64_t n, uint64_t *d_hist, int accumulate);

/* Host codebook from a host histogram with the reference's semantics: thrust
 * stable sort (Compressor.cu:378-393,414,419-425) + GenerateCL / GenerateCW /
 * toCpu (gpuHuffmanConstruction.h:353-494,551-579). U == 1 gets code "0"
 * (reference defect B4). */
int hz_codebook_build(const uint64_t *hist, hz_codebook *cb);

/* The same codebook built on the device: d_hist (u64 x 65536,
 * device) -> d_cb (a device buffer of sizeof(hz_codebook), the same layout),
 * stream-ordered on the context's stream, one workgroup, GenerateCL's rounds
 * (gpuHuffmanConstruction.h:353-494) without a grid barrier. Errors surface at
 * hz_ctx_sync: HZ_EINVAL (a count >= 2^47), HZ_ETOOLONG (a code > HZ_MAXLEN). */
int hz_codebook_build_device(hz_ctx *ctx, const uint64_t *d_hist, hz_codebook *d_cb);

/* Header bit length for a codebook and input size: 8*(3 + odd) + sum(24 + L) + 64.
 * The payload starts at that bit (Compressor.cu:431-487). */
int hz_header_bits(const hz_codebook *cb, uint64_t n, uint64_t *bits);

/* Payload bits: sum over symbols of hist[s] * len[s]. */
int hz_payload_bits(const hz_codebook *cb, const uint64_t *hist, uint64_t *bits);

/* Write the header (Compressor.cu:431-487; writers :637-669). Writes
 * floor(header_bits/8) complete bytes to out; the remaining header_bits%8
 * bits are returned MSB-aligned in *pending (they begin the payload's first
 * byte, Compressor.cu:541). */
int hz_header_write(const hz_codebook *cb, uint64_t n, uint8_t last_byte, uint8_t *out,
                     uint64_t cap, uint64_t *bytes, uint32_t *pending_bits, uint8_t *pending);

/* The header written on the device from a device codebook
 * (hz_codebook_build_device): d_out (4-byte aligned, cap bytes) receives the
 * header bit stream -- floor(bits/8) complete bytes, then the pending bits
 * MSB-aligned in the next byte, zeros after. d_info (device, 4 x u64):
 * complete bytes, pending bit count, pending byte, header bits. */
int hz_header_write_device(hz_ctx *ctx, const hz_codebook *d_cb, uint64_t n, uint8_t last_byte, uint8_t *d_out,
                           uint64_t cap, uint64_t *d_info);

/* Parse a header from the first `len` bytes of a .compressed file.
 * Replaces Decompressor.cu:65-103 (U 0 => 65536 :69-71; L 0 => 65536 :94-95). */
int hz_header_parse(const uint8_t *file, uint64_t len, hz_codebook *cb, hz_header_info *info);

/* The same parse on the device: d_file (device) -> d_cb
 * (device hz_codebook) and d_info (device, 6 x u64: n, payload byte, payload
 * bit, is_odd, last byte, nsym). Malformed headers surface as HZ_EFORMAT at
 * hz_ctx_sync. */
int hz_header_parse_device(hz_ctx *ctx, const uint8_t *d_file, uint64_t len, hz_codebook *d_cb, uint64_t *d_info);

/* Upload a codebook's device tables to the context: encode tables (needed by
 * hz_pack), decode tables (needed by hz_decode / hz_index_build /
 * hz_decode_indexless / hz_indexless_*), or both. Asynchronous on the context
 * stream: the tables are built on the host (the decode half while a hz_pack
 * launched before it runs), staged in pinned memory and copied by one device
 * kernel per table set. The index-less decoder's tables (walk length and escape
 * tables, a DENSE codebook's chain LUT) are copied by the first call that reads
 * them (hz_decode_indexless, hz_indexless_scan, hz_index_build), in its stream
 * order, so a decode through a block index never copies them; under stream
 * capture that copy is part of the captured work. */
int hz_codebook_upload(hz_ctx *ctx, const hz_codebook *cb);
int hz_codebook_upload_encode(hz_ctx *ctx, const hz_codebook *cb);
int hz_codebook_upload_decode(hz_ctx *ctx, const hz_codebook *cb);

/* Block index written by hz_pack / hz_index_build and read by hz_decode
 * (hz_index_bytes(nsym) bytes, 8-byte aligned): u64 start[nblocks + 1] -- the
 * absolute start bit of every hz_index_stride() = 2048-symbol block, then the
 * stream's end bit -- then u64 max_bits, the largest block in bits (sizes the
 * decoder's LDS slots), then u16 sub[nblocks][256]: the low 16 bits of the
 * absolute start bit of every 8-symbol chain of the block (its offset from
 * start[b] is (sub - start[b]) mod 2^16). The reference
 * has no index (its decoder is serial,
 * Decompressor.cu:259-291); this is the side band that makes decode parallel.
 *
 * Bits are counted from byte 0 of the d_payload pointer the index is used
 * with. A caller that hands hz_decode a pointer D bytes before (after) the one
 * the index was built for must rebase BOTH arrays together: add (subtract)
 * 8*D to every start[] entry and 8*D mod 2^16 to every sub[] entry; max_bits
 * is unchanged. Rebasing start[] alone decodes wrong data.
 *
 * hz_index_format() identifies this layout. Format 2 (this build) stores
 * sub[] as absolute low bits; format 1 (builds before it) stored offsets
 * from start[b]. An index kept across builds must be rebuilt (hz_index_build)
 * when the formats differ. */
#define HZ_INDEX_FORMAT 2
int hz_index_format(void);
uint64_t hz_index_stride(void);
uint64_t hz_index_bytes(uint64_t nsym);
uint64_t hz_scratch_bytes(uint64_t nsym);

/* Pack the n/2 symbols of d_in (16-byte aligned: HZ_EINVAL otherwise) with the
 * uploaded codebook into d_out as one MSB-first bit stream beginning at bit
 * `start_bit` of d_out (d_out 4-byte aligned; bits of d_out's first word before start_bit are taken from `lead`,
 * right aligned, i.e. the header's pending bits). Bits after the stream's end
 * up to the next 32-bit word are zero. d_index (optional, hz_index_bytes())
 * receives the block index. Replaces
 * populateCWLength + transform_inclusive_scan + encodeFromCW
 * (Compressor.cu:50-61,541-576,182-313) and writeFileContent (:673-684,597-601). */
int hz_pack(hz_ctx *ctx, const uint8_t *d_in, uint64_t n, uint64_t start_bit, uint32_t lead,
            uint8_t *d_out, uint64_t out_cap, uint64_t *d_index);

/* ---- two-pass encode: the range plan ------------------------------------
 * The reference reads its input three times on the device: the histogram
 * (Compressor.cu:369-372), populateCWLength + the length scan (:543-553) and
 * encodeFromCW (:573-576). hz_hist16 + hz_pack do the same (count pass, scan,
 * write). The range plan removes the middle pass: hz_hist16_ranges computes the
 * same histogram and also leaves, in d_ranges (hz_ranges_bytes(n) bytes,
 * 16-byte aligned, caller-owned), the cumulative histogram of the input at the
 * end of every range of whole blocks (about 2048 ranges); hz_pack_ranges turns
 * them into every range's start bit with the codebook (a dot product with the
 * code lengths and a scan, no input read) and packs each range in one pass.
 * The output equals hz_pack's byte for byte.
 *   - hz_ranges_bytes(n) is 0 for inputs too small for a plan (< 256 MiB);
 *     both calls then behave as hz_hist16 / hz_pack and ignore d_ranges.
 *   - d_in must be 16-byte aligned and must not change between the two calls
 *     (stream order); d_ranges is overwritten by the next hz_hist16_ranges.
 *   - hz_pack_ranges falls back to count + scan + write (same output) when the
 *     codebook's packing waves cannot take the ranges evenly;
 *     hz_last_pack_ranges(ctx) says which path the last hz_pack_ranges took. */
uint64_t hz_ranges_bytes(uint64_t n);
int hz_hist16_ranges(hz_ctx *ctx, const uint8_t *d_in, uint64_t n, uint64_t *d_hist, int accumulate,
                     void *d_ranges);
int hz_pack_ranges(hz_ctx *ctx, const uint8_t *d_in, uint64_t n, uint64_t start_bit, uint32_t lead,
                   uint8_t *d_out, uint64_t out_cap, uint64_t *d_index, void *d_ranges);
int hz_last_pack_ranges(hz_ctx *ctx);

/* Decode nsym symbols from d_payload (bit stream as hz_pack writes it) into
 * d_out (2*nsym bytes, 16-byte aligned). d_index: the block index (from
 * hz_pack, or hz_index_build for an index-less stream). d_payload
 * must stay readable up to the next 4-byte boundary after payload_bytes.
 * Replaces translateFile (Decompressor.cu:259-291). */
int hz_decode(hz_ctx *ctx, const uint8_t *d_payload, uint64_t payload_bytes, uint64_t nsym,
              const uint64_t *d_index, uint8_t *d_out);

/* Build the block index of an index-less stream (a .compressed file from
 * the reference encoder) on the device. If the payload holds fewer than nsym
 * codewords, start[nblocks] (the end bit) is left at UINT64_MAX. */
int hz_index_build(hz_ctx *ctx, const uint8_t *d_payload, uint64_t payload_bytes, uint64_t start_bit,
                   uint64_t nsym, uint64_t *d_index);

/* Decode the first nsym codewords of an index-less stream (a .compressed file
 * from the reference encoder; Decompressor.cu:259-291 decodes it serially) into
 * d_out (2*nsym bytes, 16-byte aligned) with no block index: a length walk of
 * long chains over the payload (one chain per lane, recording the start of every
 * 8th codeword of the chain), device-side fix-ups of chains whose lead-in had not
 * resynchronised, then k_decode's block decoder over the chains' 2048-codeword
 * blocks placed by the scanned counts. *d_end_bit (device u64, optional)
 * receives the end bit of codeword nsym - 1, counted from byte 0 of d_payload; a
 * payload with fewer than nsym codewords leaves it at UINT64_MAX (past
 * payload_bytes * 8) with undefined output (the caller checks, as `extract`
 * does). Stream-ordered: no host synchronisation (a HIP graph can capture it)
 * unless the context's scratch grows. A FIXED16 codebook (every code 16 bits)
 * needs no walk: symbol i sits at start_bit + 16 i, decoded directly (also
 * stream-ordered). Every other codebook takes the chain path: DENSE codebooks
 * through a LUT built beside their tables, codes longer than 25 bits through
 * DEEP escapes (the walk resolves them in the decode LUT) and a serial record
 * decoder. Payloads under 16 bytes decode serially in one device thread (also
 * stream-ordered). */
int hz_decode_indexless(hz_ctx *ctx, const uint8_t *d_payload, uint64_t payload_bytes, uint64_t start_bit,
                        uint64_t nsym, uint8_t *d_out, uint64_t *d_end_bit);

/* ---- one index-less stream over several devices ------------
 * The same decode in PARTS: every device (rank) decodes the payload bits
 * [part_begin, part_end) (counted after start_bit) of one stream, found by
 * self-synchronisation; the parts then exchange three numbers (huffman_amd/
 * dist.py decode_indexless_split):
 *   hz_indexless_scan : walk and fix-ups of the part's chains. entry_bit: the
 *       part's true first codeword start if known, else UINT64_MAX (its walked
 *       entry: right for the stream's first part, and for every part whose
 *       lead-in resynchronised). d_summary (device, 3 x u64): codewords of the
 *       part, its true exit bit (the next part's true entry), the entry bit in
 *       use (entry_bit, or the walked entry for UINT64_MAX).
 *       Bits are STREAM bits: bit 0 is bit 0 of the stream's payload buffer
 *       (the one hz_decode_indexless takes), and d_payload holds stream bits
 *       [payload_bit_base, payload_bit_base + 8 * payload_bytes) -- a rank may
 *       pass only its slice (payload_bit_base a multiple of 8). The slice must
 *       hold the part and the HZ_INDEXLESS_LEAD_BITS before it (or the stream
 *       from its start), else HZ_EINVAL; the part's last codeword may run up to
 *       max_len bits past part_end (missing bits read as zeros: keep them in
 *       the slice). nsym: the stream's symbols (sizes the part's record capacity
 *       from its mean bits per codeword; 0 = unknown: the codebook's estimate).
 *   hz_indexless_refix : the part again from its true entry (the previous
 *       part's exit, when it differs from the walked entry); d_summary updated.
 *   hz_indexless_decode : the part's codewords into d_out (2 bytes each, from
 *       the part's first codeword), at most nsym of them (the stream's symbols
 *       from the part's first on); *d_end_bit as hz_decode_indexless when the
 *       stream's last codeword falls in this part (a stream bit).
 * The three calls keep their state in the context's scratch and point at its
 * decode tables: one part per context at a time, and any other call that uses
 * the scratch or the tables (hz_pack*, hz_index_build, hz_decode_indexless,
 * hz_codebook_upload_decode) ends the pending part -- hz_indexless_refix /
 * _decode then return HZ_EINVAL. The same holds for a HIP graph that captured
 * hz_decode_indexless: replay it only while no call on the context has grown
 * the scratch or replaced the decode tables since the capture.
 * Every codebook takes this path; a FIXED16 part (every code 16 bits) is
 * arithmetic: codeword i at start_bit + 16 i, no walk. */
#define HZ_INDEXLESS_LEAD_BITS 1024
int hz_indexless_scan(hz_ctx *ctx, const uint8_t *d_payload, uint64_t payload_bytes, uint64_t payload_bit_base,
                      uint64_t start_bit, uint64_t nsym, uint64_t part_begin, uint64_t part_end, uint64_t entry_bit,
                      uint64_t *d_summary);
int hz_indexless_refix(hz_ctx *ctx, uint64_t entry_bit, uint64_t *d_summary);
int hz_indexless_decode(hz_ctx *ctx, uint64_t nsym, uint8_t *d_out, uint64_t *d_end_bit);

/* Kernel timings of the last hz_hist16 / hz_pack / hz_decode / hz_index_build /
 * hz_decode_indexless call on this context, in milliseconds (HIP events on the
 * context stream). */
int hz_last_kernel_ms(hz_ctx *ctx, int stage, float *ms);
enum { HZ_STAGE_HIST = 0, HZ_STAGE_PACK = 1, HZ_STAGE_DECODE = 2, HZ_STAGE_INDEX = 3, HZ_STAGE_EXTRACT = 4 };

/* Synthetic inputs on the device (DESIGN.md "Synthetic inputs"): byte i of the
 * stream = f(splitmix64(seed ^ (offset + i))); kind 0 uniform, 1 Zipf(alpha). */
int hz_generate(hz_ctx *ctx, uint8_t *d_out, uint64_t n, uint64_t offset, int kind, double alpha,
                uint64_t seed);

/* ---- file level: the CLI contract ---------------------------------------- */

/* `archive <path>`: writes <path>.compressed (Compressor.cu:315-632). */
int hz_archive_file(const char *path, int verbose);
/* Streaming archive of in_path into out_path with bounded memory: two passes
 * over the file in chunk_bytes pieces (histogram, then pack at the running bit
 * offset with the previous chunk's partial word carried as `lead`). Output is
 * byte-identical to the whole-buffer encoder. hz_archive_file uses it with
 * 256 MiB chunks. Replaces the whole-file buffers of Compressor.cu:343-367,585-601. */
int hz_archive_stream(const char *in_path, const char *out_path, uint64_t chunk_bytes, int verbose);
/* Streaming extract of in_path into out_path through a device window of
 * chunk_bytes of payload, bounded host and device memory: each round decodes
 * the codewords the window surely holds with hz_decode_indexless (no block
 * index) and carries the unconsumed tail into the next window; the host waits
 * once per round (for the round's end bit), and the next window's file read
 * and this round's fwrite overlap the device. hz_extract_file uses it with
 * 256 MiB windows. Replaces the whole-file buffers of
 * Decompressor.cu:65-114,259-291. */
int hz_extract_stream(const char *in_path, const char *out_path, uint64_t chunk_bytes, int verbose);
/* Stage split of the calling thread's last hz_archive_stream /
 * hz_extract_stream call (hz_archive_file / hz_extract_file included). Stage
 * times are busy times: host file reads and writes overlap the device's
 * copies and kernels, so they do not add up to total_ms. */
typedef struct hz_stream_timing {
    double total_ms;   /* wall clock of the call */
    double fread_ms;   /* host: file reads */
    double fwrite_ms;  /* host: file writes */
    double alloc_ms;   /* host: device context, device buffers, pinned host buffers */
    double host_ms;    /* host: codebook build, header write / parse, table uploads */
    double h2d_ms;     /* device: host-to-device copies */
    double kernel_ms;  /* device: histogram, pack, index build, decode */
    double d2h_ms;     /* device: device-to-host copies */
    uint64_t bytes_in;   /* bytes read from in_path */
    uint64_t bytes_out;  /* bytes written to out_path */
} hz_stream_timing;
int hz_stream_last_timing(hz_stream_timing *t);
/* `extract <path>`: writes ./DECOMPRESSED_FILE or DECOMPRESSED_FILE(k)
 * (Decompressor.cu:47-114,185-219). out_name may be NULL. */
int hz_extract_file(const char *path, char *out_name, size_t out_name_cap, int verbose);

/* Whole-buffer host API (device work inside): encode host bytes to a complete
 * .compressed image / decode one. */
int hz_encode_host(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len);
int hz_encoded_size(const uint8_t *in, uint64_t n, uint64_t *out_len);
int hz_decode_host(const uint8_t *file, uint64_t len, uint8_t *out, uint64_t cap, uint64_t *out_n);

#ifdef __cplusplus
}
#endif
#endif /* HUFFMAN_AMD_H */
