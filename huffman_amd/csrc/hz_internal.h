// hz_internal.h -- shared layout constants and launch interfaces between the
// host side (hz_host.cpp) and the gfx950 kernels (hz_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "huffman_amd.h"

namespace hz {

// ---- pack: one wavefront owns a block of 64 lanes x kSPT symbols ----------
constexpr int kWave = 64;
constexpr int kSPT = 32;                       // symbols per lane (64 input bytes)
constexpr int kBlockSyms = kWave * kSPT;       // 2048 symbols = 4 KiB of input
constexpr int kChainsPerLane = 4;              // decode: independent chains per lane
constexpr int kChainSyms = kSPT / kChainsPerLane;         // 8 symbols: index granularity
constexpr int kChainsPerBlock = kBlockSyms / kChainSyms;  // 256
constexpr int kPackThreads = 1024;             // 16 waves per CU share one LDS table
constexpr uint32_t kLdsBytes = 160u * 1024u;   // LDS per CU (gfx950)

// Block index written by hz_pack / hz_index_build (DESIGN.md "Decode"):
//   u64 start[nblocks + 1]      absolute start bit of every 2048-symbol block
//                               (start[nblocks] = end of the stream)
//   u64 max_bits                largest block (bits): sizes the decoder's LDS slots
//   u16 sub[nblocks][256]       low 16 bits of the absolute start bit of every
//                               8-symbol chain (a lane's four chains are one
//                               u64); the decoder takes (sub - start[b]) mod 2^16,
//                               exact when block bits < 2^16, otherwise recovered
//                               by a prefix over deltas.
__host__ __device__ inline uint64_t index_blocks(uint64_t nsym) { return (nsym + kBlockSyms - 1) / kBlockSyms; }
__host__ __device__ inline uint64_t index_bytes(uint64_t nsym) {
    const uint64_t nb = index_blocks(nsym);
    return nsym ? 8 * (nb + 2) + 2ull * kChainsPerBlock * nb : 0;
}
__host__ __device__ inline uint64_t index_sub_offset(uint64_t nblocks) { return nblocks + 2; }  // in u64 words

// ---- range plan: the two-pass encode (DESIGN.md "Ranges") -------------------
// The input is cut into nranges RANGES of bpr whole blocks. The histogram kernel
// sweeps them with `groups` workgroups (range j by workgroup j % groups, in
// order) and snapshots its cumulative LDS histogram at the end of every range;
// with the codebook known, a dot product of each snapshot with the code
// lengths gives every range's payload bits, a scan gives its start bit, and
// one pack wave per range writes its blocks in order from there: no count
// pass over the input. Buffer (hz_ranges_bytes), in order:
//   u32 snap[nranges][32768]            LDS image at the range's end (u16 pairs, hist_word order)
//   u32 list[groups][1 + list_cap]      count, then every +-65536 carry the workgroup
//                                       made: local range << 17 | negative << 16 | bin
//   u64 dot[nranges]                    sum of len * cumulative count (k_range_dot)
//   u64 start[nranges + 1]              start bit of every range, then the stream's end
constexpr uint64_t kRangeTarget = 2048;     // ranges (= pack waves: 256 CUs x 8)
constexpr uint64_t kRangeMinBlocks = 64;    // a snapshot (128 KiB) per >= 256 KiB of input
constexpr uint64_t kRangeMinRanges = 1024;  // smaller inputs keep count + scan + write
constexpr uint32_t kRangeGroups = 256;
struct RangeGeom {
    uint64_t nsym, nblocks, bpr, nranges, per_group;
    uint32_t groups, list_cap;
    uint64_t off_list, off_dot, off_start, bytes;  // byte offsets in the range buffer
};
__host__ __device__ inline RangeGeom range_geom(uint64_t nsym) {
    RangeGeom g{};
    g.nsym = nsym;
    g.nblocks = (nsym + kBlockSyms - 1) / kBlockSyms;
    const uint64_t want = (g.nblocks + kRangeTarget - 1) / kRangeTarget;
    g.bpr = want > kRangeMinBlocks ? want : kRangeMinBlocks;
    g.nranges = (g.nblocks + g.bpr - 1) / g.bpr;
    if (g.nranges < kRangeMinRanges) return RangeGeom{};  // bytes = 0: no range plan
    g.groups = (uint32_t)(g.nranges < kRangeGroups ? g.nranges : kRangeGroups);
    g.per_group = (g.nranges + g.groups - 1) / g.groups;
    // a low-half wrap needs 65 536 adds and makes at most three records (its own, a high-half
    // wrap of its transient carry and the carry's undo); a high-half wrap one. Bound x4 + 16.
    g.list_cap = (uint32_t)(4 * (g.per_group * g.bpr * kBlockSyms / 65536) + 16);
    g.off_list = g.nranges * 32768ull * 4;
    g.off_dot = (g.off_list + 4ull * g.groups * (1 + g.list_cap) + 15) & ~15ull;
    g.off_start = g.off_dot + 8 * g.nranges;
    g.bytes = g.off_start + 8 * (g.nranges + 1);
    return g;
}

// Histogram LDS word of symbol pair s >> 1. Byte-pair symbols of skewed data
// share their low bits (the first byte), which alone would pick the LDS bank:
// the second byte times 13 (odd: distinct small bytes land on distinct, spread
// banks) is XORed into word bits 0-5; it depends only on word bits 7-14, which
// the XOR leaves alone, so the map is a bijection.
__host__ __device__ inline uint32_t hist_word(uint32_t s) { return (s >> 1) ^ (((s >> 8) * 13u) & 0x3fu); }
__host__ __device__ inline uint32_t hist_word_inv(uint32_t w) { return w ^ (((w >> 7) * 13u) & 0x3fu); }

// Encode table modes (selected on the host per codebook, DESIGN.md "Pack").
enum EncMode : int {
    ENC_DENSE = 0,  // max_len <= 16: 65536 x 17-bit sentinel entries, 139 264 B LDS
    ENC_HOT = 1,    // max_len <= 25: 32768 u32 slots (tag,len,code) + u32 escapes
    ENC_WIDE = 2,   // anything up to 56 bits: u64 table in global memory
    ENC_FIXED16 = 3 // every code 16 bits (U = 65536, min_len = max_len): u16 codes in LDS, no scan
};
constexpr uint32_t kFixed16LdsBytes = 65536u * 2u;       // 131 072
constexpr uint32_t kDenseLdsBytes = 65536u * 17u / 8u;   // 139 264
constexpr uint32_t kHotLdsBytes = 32768u * 4u;           // 131 072
constexpr uint32_t kLen8LdsBytes = 65536u;               // u8 code length per symbol (count pass)
constexpr int kHotMaxLen = 25;                           // codes in a HOT slot
constexpr int kNarrowMaxLen = 26;                        // u32 register entries

// Decode table modes.
enum DecMode : int {
    DEC_DENSE = 0,  // max-min <= 3 and the table fits beside 8 staging slots: 2^K u16 symbols + 2-bit lengths
    DEC_LUT = 1,    // 2^K1 u32 level-1 entries in LDS, deeper levels in global
    DEC_FIXED16 = 2 // every code 16 bits: u16 symbol per code in LDS, positions are arithmetic
};
constexpr int kDecLutMaxK1 = 13;  // + global levels of up to kDecLevelBits: pipelined up to 25-bit codes
constexpr int kDecLevelBits = 12; // widest global subtable (each link's is as wide as its codes need; fewer
                                  // bits when the table would exceed kLutMaxL2): codes up to 25 bits in two levels
// LUT entries (DEC_LUT; hz_codebook.cpp build_dec_lut):
//   leaf  1 << 31 | L << 24 | sym << 8   (bits 7..0 zero)
//   link  raw << 10 | nb << 5 | pos   (bit 31 clear). raw < kLutGlobal: the subtable starts at word raw of
//         the LDS image; else at l2[raw - kLutGlobal]. nb (<= 15) index bits follow the D code bits
//         already consumed; pos = 32 - D - nb (0 when D + nb > 32): the index is bits [pos, pos + nb) of
//         a 32-bit window whose bit 31 is the code's first bit, one v_bfe_u32(W, e, e >> 5) -- no depth
//         bookkeeping in the decoder's hot loop.
constexpr uint32_t kLutGlobal = 65536;                      // > any LDS word index (160 KiB / 4)
constexpr uint32_t kLutMaxL2 = (1u << 21) - kLutGlobal;     // global entries a 21-bit raw field reaches
__host__ __device__ inline uint32_t lut_link(uint32_t raw, uint32_t nb, uint32_t D) {
    return (raw << 10) | (nb << 5) | (D + nb <= 32 ? 32 - D - nb : 0u);
}
// A leaf read as a link (the pipelined decoder does so unconditionally) has pos = 0 and a width of
// (sym & 3) * 8 <= 24 bits, so its index (e >> 10) + bfe(W, 0, width) lies in [2^21, 2^21 + 2^20 + 2^24):
// past every LDS word and past the global table's num_records (2^21 entries), and its byte offset
// (index * 4 < 2^27) never wraps a 32-bit register back into a table. Symbol bits on a byte
// boundary: one v_perm packs two symbols.
__host__ __device__ inline uint32_t lut_leaf_entry(uint32_t L, uint32_t sym) {
    return (1u << 31) | (L << 24) | (sym << 8);
}
__host__ __device__ inline uint32_t lut_leaf_len(uint32_t e) { return (e >> 24) & 63u; }
__host__ __device__ inline uint32_t lut_leaf_sym(uint32_t e) { return (e >> 8) & 0xffffu; }
constexpr int kDecMaxWaves = 16;
// Smallest LDS image of a LUT (words): the pipelined decoders' staging slots follow the table, and their
// window addresses carry a bias of 128 bits per step taken (up to 7 * 128 below a lane's true bit address,
// dec_pipe_ldsn's adj): the lowest slot must start at LDS bit 1024 or more so the biased address never
// wraps below 0. (A DENSE codebook's chain LUT has 2^max_len entries: 4 words for 2-bit codes.)
constexpr uint32_t kDecMinLdsWords = 32;
// Index walker (k_idx_walk): one chain per lane, kWalkWaves waves per CU; per
// chain an LDS ring of 4 payload chunks (16 B) and kWalkMarkChunks mark chunks,
// beside a 4-bit code-length table of the top kWalkK window bits.
// Measured at 16 GiB Zipf, index build (A/B runs, round 2): 10 waves with 4 mark
// chunks 27.0 ms, 12 / 14 waves with 2 mark chunks 25.5 / 26.0 ms; 10 steps per
// round 25.3 vs 8 steps 25.5 ms. With the earlier u32 LUT walker: 2 chains per
// lane x 4 waves 53.7 vs 1 x 8 waves 38.4 ms.
constexpr int kWalkK = 17;            // walker length table: 2^17 4-bit lengths (64 KB) in LDS
constexpr int kWalkMaxLen = 25;       // escape table: 2^max_len u8 in global memory (<= 32 MiB)
constexpr int kWalkChains = 1;
constexpr int kWalkWaves = 12;
constexpr uint32_t kWalkMarkChunks = 2;
constexpr uint32_t kRingWords = 16 + 4 * kWalkMarkChunks + 1;  // odd stride: the lanes' rings start in distinct banks
constexpr uint32_t kWalkWaveBytes = 64u * kWalkChains * kRingWords * 4u;
constexpr uint32_t kWalkLdsRingBytes = kWalkWaves * kWalkWaveBytes;
static_assert((1u << kWalkK) / 2 + kWalkLdsRingBytes <= kLdsBytes, "walker LDS");
constexpr int kDecMinWaves = 8;  // DENSE only when this many staging slots fit

// Per-wave LDS slot for one block's payload (u32 words), from the largest
// block of the stream: its bits, chains past the end of a tail block (16 codes
// each), the 16-byte alignment of the first word and the words a window reads
// past the last bit.
__host__ __device__ inline uint32_t dec_slot_words(uint64_t max_bits, int max_len) {
    const uint64_t bits = max_bits + (uint64_t)kChainSyms * (uint32_t)max_len;
    const uint64_t w = (bits + 31) / 32 + 4 + 3 + 4;  // + 16-byte pad before the block
    return (uint32_t)((w + 3) & ~3ull);
}
// Worst case: every symbol of a block at max_len bits.
__host__ __device__ inline uint32_t dec_slot_words_max(int max_len) {
    return dec_slot_words((uint64_t)kBlockSyms * (uint32_t)max_len, max_len);
}

struct Tables {
    int enc_mode = -1;
    int dec_mode = -1;
    int max_len = 0;
    int min_len = 0;
    int dec_k = 0;                 // DENSE window bits / LUT level-1 bits
    int dec_level_bits = 0;        // LUT: widest global subtable (kDecLevelBits unless reduced to fit kLutMaxL2)
    int dec_max_len = 0;           // of the codebook the decode tables were built for
    int dec_min_len = 0;
    double dec_avg_bits = 0.0;     // Kraft estimate of bits per codeword of the decode codebook: sum 2^-L * L
    uint32_t enc_lds_bytes = 0;
    double enc_avg_bits = 16.0;    // Kraft estimate of bits per symbol: sum 2^-L * L
    uint32_t dec_lds_bytes = 0;
    uint32_t* d_enc_lds = nullptr; // LDS image for the pack kernel
    uint64_t* d_enc_wide = nullptr;// 65536 x u64: len << 56 | code
    uint32_t* d_enc_esc = nullptr; // 65536 x u32: len << 26 | code (HOT escapes, len <= 26)
    uint32_t* d_len8 = nullptr;    // LDS image: u8 length at len8_index(s)
    uint32_t* d_lenpair = nullptr; // range plan: u8 lengths of both symbols of every histogram word (u16 each)
    uint32_t hot_mask = 0x8000;    // HOT pairing: s and s ^ hot_mask share slot
    uint32_t* d_dec_lds = nullptr; // LDS image for the decode kernel
    uint32_t* d_dec_l2 = nullptr;  // deeper LUT levels (shared by both images)
    uint64_t dec_l2_entries = 0;
    uint32_t* d_walk_lds = nullptr; // index walker: 4-bit code length - walk_bias per walk_k-bit window (0 = longer code)
    uint32_t walk_lds_bytes = 0;    // 0 = no walker tables (the segment walkers build the index)
    uint32_t* d_walk_esc = nullptr; // index walker: u8 code length per walk_m-bit window (walk_m > walk_k)
    int walk_k = 0, walk_m = 0, walk_bias = 0;
    uint32_t* d_walk8 = nullptr;    // chain walker: u8 code length per walk8_k-bit window (0 = escape to d_walk_esc)
    uint32_t walk8_bytes = 0;
    int walk8_k = 0;
    // The index-less chain decoder's tables (hz_decode_indexless, hz_indexless_*): LUT-format decode
    // images (DEC_LUT codebooks: the decode tables themselves; DEC_DENSE: a LUT built beside them) and
    // the walker's escape table of u8 lengths per chain_esc_m-bit window (chain_esc_m = min(max_len,
    // kWalkMaxLen); 0 = a DEEP escape for codes longer than that, resolved through the LUT).
    const uint32_t* chain_lds = nullptr;  // level 1 (+ hot heads) LDS image
    const uint32_t* chain_l2 = nullptr;   // global levels
    uint32_t chain_lds_bytes = 0;         // 0: no chain tables (FIXED16: positions are arithmetic)
    int chain_k = 0, chain_level_bits = 0;
    const uint8_t* chain_esc = nullptr;
    int chain_esc_m = 0;
    uint32_t* d_chain_lds = nullptr;      // owned images behind chain_* when they are not the decode tables'
    uint32_t* d_chain_l2 = nullptr;
    uint32_t* d_chain_esc = nullptr;
};
// Walker escape table resolution (kWalkMaxLen bits at most: a 32 MiB table).
constexpr int kChainEscMaxBits = kWalkMaxLen;

// Count-pass length table layout: the high byte is XORed into the bank bits
// so skewed symbol sets (small high and low bytes) spread over LDS banks.
__host__ __device__ inline uint32_t len8_index(uint32_t s) { return s ^ (((s >> 8) & 0x3fu) << 2); }

// HOT slot of symbol s under pairing mask m (bit 15 of m set).
__host__ __device__ inline uint32_t hot_slot(uint32_t s, uint32_t m) { return (s & 0x8000u) ? (s ^ m) : s; }
// LDS word of a HOT slot: the symbol's second byte is XORed into the bank bits
// (the first byte alone would pick the bank; skewed data keeps it small).
__host__ __device__ inline uint32_t hot_word(uint32_t slot) { return slot ^ ((slot >> 8) & 0x3fu); }

// Launchers (hz_kernels.hip). All stream ordered; return hipError_t.
hipError_t launch_hist16(const uint8_t* d_in, uint64_t n, unsigned long long* d_hist, int ncu,
                         hipStream_t s);
hipError_t launch_hist16_ranges(const uint8_t* d_in, uint64_t n, unsigned long long* d_hist, void* d_ranges,
                                uint32_t* d_err, hipStream_t s);  // range plan (RangeGeom)
// d_ranges (nullable): the range plan of d_in from launch_hist16_ranges; *used_ranges = 1 when the
// pack took it (else count + scan + write)
hipError_t launch_pack(const Tables& t, const uint8_t* d_in, uint64_t nsym, uint64_t start_bit,
                       uint32_t lead, uint32_t* d_out, uint64_t out_words, unsigned long long* d_scratch,
                       unsigned long long* d_index, uint32_t* d_err, int ncu, hipStream_t s,
                       void* d_ranges = nullptr, int* used_ranges = nullptr);
uint64_t pack_scratch_words(uint64_t nsym);  // u64 words of d_scratch hz_pack needs
hipError_t launch_decode(const Tables& t, const uint8_t* d_payload, uint64_t payload_bytes,
                         uint64_t nsym, const unsigned long long* d_index, uint8_t* d_out,
                         uint32_t* d_err, int ncu, hipStream_t s,
                         uint64_t start0 = 0);  // d_index null (FIXED16 only): symbol i at start0 + 16 i
hipError_t launch_index_build(const Tables& t, const uint8_t* d_payload, uint64_t payload_bytes,
                              uint64_t start_bit, uint64_t nsym, unsigned long long* d_index,
                              unsigned long long* d_scratch, uint32_t* d_err, uint32_t* h_scratch, int ncu,
                              hipStream_t s);  // synchronises the stream (iterates to a fixed point)
uint64_t index_scratch_words(uint64_t payload_bytes, uint64_t start_bit);  // u64 words hz_index_build needs
// Index-less decode in chain blocks (hz_kernels.hip; no block index, stream-ordered: no host
// synchronisation). Phases over a PART of the payload (bits [part_begin, part_end) after start_bit; the
// whole payload for one device, a slice per rank for one stream split over ranks):
//   chain_scan   : walk, fix-ups, scans, block descriptors; summary in chain_info (device u64):
//                  [3] codewords of the part, [4] its true exit bit, [5] its entry bit in use.
//                  entry0: the part's true entry bit (~0: its walked entry, e.g. the stream's start)
//   chain_refix  : the fix-ups again from a new true entry (another rank's exit), summary updated
//   chain_decode : the part's first nsym codewords (nsym: the stream's symbols after the part's first)
//                  into d_out; d_end: end bit of its codeword nsym - 1 (all ones: not in this part)
struct ChainState;
ChainState* chain_state_create();
void chain_state_destroy(ChainState* st);
bool seg_decode_supported(const Tables& t);
uint64_t chain_scratch_words(uint64_t part_begin, uint64_t part_end, uint64_t nsym, const Tables& t, int ncu);
// base: stream bit of byte 0 of d_payload (0: the buffer starts with the stream); every bit argument
// and result is a stream bit
hipError_t chain_scan(ChainState* st, const Tables& t, const uint8_t* d_payload, uint64_t payload_bytes,
                      uint64_t base, uint64_t start_bit, uint64_t nsym, uint64_t part_begin, uint64_t part_end,
                      uint64_t entry0, unsigned long long* d_scratch, uint32_t* d_err, int ncu, hipStream_t s);
hipError_t chain_refix(ChainState* st, const Tables& t, uint64_t entry0, int ncu, hipStream_t s);
hipError_t chain_decode(ChainState* st, const Tables& t, uint64_t nsym, uint8_t* d_out, unsigned long long* d_end,
                        int ncu, hipStream_t s);
// payloads under 16 bytes: one thread, serially, stream-ordered (d_end: the end bit or UINT64_MAX)
hipError_t chain_decode_tiny(const Tables& t, const uint8_t* d_payload, uint64_t payload_bytes, uint64_t start_bit,
                             uint64_t nsym, uint8_t* d_out, unsigned long long* d_end, uint32_t* d_err, hipStream_t s);
const unsigned long long* chain_info(const ChainState* st);
void chain_invalidate(ChainState* st);  // the scratch or tables it points into changed
hipError_t chain_summary(const ChainState* st, unsigned long long* d_dst, hipStream_t s);  // 3 x u64, stream bits
hipError_t put3(unsigned long long* d_dst, uint64_t a, uint64_t b, uint64_t c, hipStream_t s);  // stream-ordered
// Table uploads: segments of a pinned host staging buffer copied to their device tables by one kernel
// (it reads the host memory over PCIe: one launch per upload instead of one copy per table).
struct StageSeg {
    void* dst;
    uint64_t off, bytes;  // off: 16-byte aligned in the staging buffer; bytes: a multiple of 4
};
constexpr int kStageMaxSegs = 16;
hipError_t stage_scatter(const uint8_t* h_src, const StageSeg* segs, int nseg, hipStream_t s);
hipError_t launch_codebook(const unsigned long long* d_hist, hz_codebook* d_cb, unsigned long long* d_ws,
                           uint32_t* d_err, hipStream_t s);  // hz_codebook_gpu.hip
uint64_t codebook_ws_words();
hipError_t launch_header_write(const hz_codebook* d_cb, uint64_t n, uint32_t last_byte, uint8_t* d_out, uint64_t cap,
                               unsigned long long* d_info, unsigned long long* d_ws, uint32_t* d_err, hipStream_t s);
hipError_t launch_header_parse(const uint8_t* d_file, uint64_t len, hz_codebook* d_cb, unsigned long long* d_info,
                               unsigned long long* d_ws, uint32_t* d_err, hipStream_t s);
hipError_t launch_generate(uint8_t* d_out, uint64_t n, uint64_t offset, int kind, uint64_t seed,
                           const unsigned long long* d_thr, hipStream_t s);

}  // namespace hz
