// hz_kernels.hip -- gfx950 (MI355X, CDNA4) kernels of the Huffman hot path.
//
//   k_hist16   65 536-bin histogram of u16 symbols      <- Compressor.cu:38-48
//   k_pack     codeword lookup + bit-length scan + pack  <- Compressor.cu:50-61,541-576,182-313
//   k_decode   block-parallel table decode              <- Decompressor.cu:259-291
//   k_sync_*   block index of an index-less stream (reference files), parallel, self-synchronising
//   k_generate synthetic Zipf / uniform byte streams (this build's generator)
//
// Layout, roofline and design notes: DESIGN.md. All integer/bit work; no MFMA.
#include <stdio.h>
#include <stdlib.h>

#include <mutex>
#include <set>
#include <type_traits>
#include <utility>

#include "hz_internal.h"

namespace hz {

#define HZ_DEV __device__ __forceinline__

// Dynamic-LDS limit of a kernel: hipFuncSetAttribute is per device, so the
// (kernel, device) pairs already raised are remembered under a lock (any
// number of contexts on any devices, from any host threads).
static hipError_t ensure_lds_limit(const void* fn, int bytes) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    static std::mutex mu;
    static std::set<std::pair<std::pair<const void*, int>, int>> done;
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair(std::make_pair(fn, dev), bytes);
    if (done.count(key)) return hipSuccess;
    if ((e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes)) != hipSuccess) return e;
    done.insert(key);
    return hipSuccess;
}

HZ_DEV uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

HZ_DEV uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

typedef short hz_i16x2 __attribute__((ext_vector_type(2)));           // packed 16-bit lanes (v_pk_*)
typedef unsigned short hz_u16x2 __attribute__((ext_vector_type(2)));

// 16 bytes at a 4-byte aligned address (global_load/store_dwordx4 need only dword alignment): the
// FIXED16 block kernels move a stream that starts at any word behind the header.
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4a2 __attribute__((ext_vector_type(4), aligned(2)));  // 16 bytes at a 2-byte aligned address

// One 16-byte non-temporal store (global_store_dwordx4 ... nt).
HZ_DEV void store_nt16(uint4* p, uint4 v) {
    uint32_t* q = reinterpret_cast<uint32_t*>(p);
    __builtin_nontemporal_store(v.x, q);
    __builtin_nontemporal_store(v.y, q + 1);
    __builtin_nontemporal_store(v.z, q + 2);
    __builtin_nontemporal_store(v.w, q + 3);
}
HZ_DEV uint32_t shfl_up_u32(uint32_t v, int d) { return (uint32_t)__shfl_up((int)v, d, 64); }
HZ_DEV uint32_t shfl_u32(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src, 64); }
HZ_DEV uint32_t shfl_xor_u32(uint32_t v, int m) { return (uint32_t)__shfl_xor((int)v, m, 64); }
// DPP lane moves (VALU, no LDS round trip). Lanes whose source lies outside
// the row (row_shr) or outside row_mask read 0.
template <int CTRL, int ROWS = 0xf>
HZ_DEV uint32_t dpp0(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, false);
}
constexpr int kDppRowShr1 = 0x111, kDppRowShr2 = 0x112, kDppRowShr4 = 0x114, kDppRowShr8 = 0x118;
constexpr int kDppRowBcast15 = 0x142, kDppRowBcast31 = 0x143, kDppWaveShr1 = 0x138, kDppWaveShl1 = 0x130;
constexpr bool kFixed16Blk = true;  // FIXED16 streams: the 1 KiB-coalesced full-block kernels

// Inclusive prefix sum over the 64 lanes.
HZ_DEV uint32_t wave_incl_sum(uint32_t v) {
    v += dpp0<kDppRowShr1>(v);
    v += dpp0<kDppRowShr2>(v);
    v += dpp0<kDppRowShr4>(v);
    v += dpp0<kDppRowShr8>(v);
    v += dpp0<kDppRowBcast15, 0xa>(v);
    v += dpp0<kDppRowBcast31, 0xc>(v);
    return v;
}

HZ_DEV uint32_t readlane(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }

// LDS word at byte address `byte` of a kernel without static LDS (its dynamic
// LDS starts at address 0): no base add per access.
typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
HZ_DEV uint32_t lds_at(uint32_t byte) { return *reinterpret_cast<lds_cu32*>(byte); }
// The wave's index in its workgroup as a wave-uniform (SGPR) value: block numbers derived from it,
// and the index / start loads they address, stay on the scalar unit.
HZ_DEV uint32_t wave_id() {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}

HZ_DEV uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        uint32_t lo = shfl_xor_u32((uint32_t)v, m), hi = shfl_xor_u32((uint32_t)(v >> 32), m);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}

// ===========================================================================
// Synthetic input generator (not a reference function).
// ===========================================================================
HZ_DEV uint8_t gen_byte(uint64_t j, int kind, uint64_t seed, const unsigned long long* t) {
    uint64_t u = splitmix64(seed ^ j);
    if (kind == 0) return (uint8_t)u;
    int lo = 0, hi = 255;
    while (lo < hi) {
        int m = (lo + hi) >> 1;
        if (u < t[m]) hi = m; else lo = m + 1;
    }
    return (uint8_t)lo;
}

__global__ __launch_bounds__(256) void k_generate(uint8_t* __restrict__ out, uint64_t n, uint64_t offset,
                                                 int kind, uint64_t seed,
                                                 const unsigned long long* __restrict__ thr) {
    __shared__ unsigned long long t[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) t[i] = thr ? thr[i] : 0ull;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const bool aligned = (((uintptr_t)out) & 7) == 0;
    const uint64_t nv = aligned ? n / 8 : 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nv; i += stride) {
        uint64_t w = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) w |= (uint64_t)gen_byte(offset + i * 8 + k, kind, seed, t) << (8 * k);
        reinterpret_cast<uint64_t*>(out)[i] = w;
    }
    for (uint64_t j = nv * 8 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += stride)
        out[j] = gen_byte(offset + j, kind, seed, t);
}

hipError_t launch_generate(uint8_t* d_out, uint64_t n, uint64_t offset, int kind, uint64_t seed,
                           const unsigned long long* d_thr, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t want = (n / 8 + 255) / 256;
    unsigned grid = (unsigned)(want < 8192 ? (want ? want : 1) : 8192);
    hipLaunchKernelGGL(k_generate, dim3(grid), dim3(256), 0, s, d_out, n, offset, kind, seed, d_thr);
    return hipGetLastError();
}

// ===========================================================================
// Histogram: 65 536 u16 counters packed two per LDS dword (128 KiB, one
// 1024-thread workgroup per CU). A counter half that wraps is corrected
// exactly through the value the LDS atomic returns (DESIGN.md "Histogram").
// ===========================================================================
constexpr int kHistThreads = 1024;

// (LDS word of a symbol pair: hist_word, hz_internal.h)

// Fix-up after `old = atomicAdd(&lds[hist_word(s)], inc)`; rare (once per 65 536 adds of a bin).
// rec(bin, negative) sees every +-65 536 the global histogram receives (range snapshots).
struct NoRec {
    HZ_DEV void operator()(uint32_t, uint32_t) const {}
};
template <typename Rec = NoRec>
HZ_DEV void hist_fix(uint32_t* lds, unsigned long long* hist, uint32_t s, uint32_t old, Rec rec = Rec()) {
    const uint32_t inc = (s & 1) ? 0x10000u : 1u;
    if (old + inc < old) {  // the dword (high half) wrapped
        atomicAdd(&hist[s | 1], 65536ull);
        rec(s | 1, 0u);
    }
    if (!(s & 1) && (old & 0xffffu) == 0xffffu) {  // low half crossed 65 536: undo its carry
        atomicAdd(&hist[s], 65536ull);
        rec(s, 0u);
        uint32_t o2 = atomicSub(&lds[hist_word(s)], 0x10000u);
        if (o2 < 0x10000u) {
            atomicAdd(&hist[s | 1], (unsigned long long)(-65536ll));
            rec(s | 1, 1u);
        }
    }
}

HZ_DEV bool hist_needs_fix(uint32_t s, uint32_t old) {
    const uint32_t inc = (s & 1) ? 0x10000u : 1u;
    return (old + inc < old) | (!(s & 1) & ((old & 0xffffu) == 0xffffu));
}

template <typename Rec = NoRec>
HZ_DEV void hist_one(uint32_t* lds, unsigned long long* hist, uint32_t s, Rec rec = Rec()) {
    uint32_t old = atomicAdd(&lds[hist_word(s)], (s & 1) ? 0x10000u : 1u);
    if (hist_needs_fix(s, old)) hist_fix(lds, hist, s, old, rec);
}

// The 8 symbols of a 16-byte vector: 8 LDS atomics; a fix-up is due exactly when the
// incremented half was 0xffff (the half a symbol counts in is its bit 0, the shift 16 * bit 0).
// hist_word of both symbols of a dword at once (packed 16-bit shifts and multiply).
template <typename Rec = NoRec>
HZ_DEV void hist_count8(uint32_t* lds, unsigned long long* hist, const uint4& v, Rec rec = Rec()) {
    const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
    uint32_t old[8], sh[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const hz_u16x2 w = __builtin_bit_cast(hz_u16x2, wd[j]);
        const hz_u16x2 hw = (w >> (hz_u16x2){1, 1}) ^ (((w >> (hz_u16x2){8, 8}) * (hz_u16x2){13, 13}) & (hz_u16x2){0x3f, 0x3f});
        const uint32_t a = __builtin_bit_cast(uint32_t, hw);  // hist_word of both symbols (< 32768 each)
        sh[2 * j] = (wd[j] << 4) & 16u;
        sh[2 * j + 1] = (wd[j] >> 12) & 16u;
        old[2 * j] = atomicAdd(&lds[a & 0x7fffu], 1u << sh[2 * j]);
        old[2 * j + 1] = atomicAdd(&lds[a >> 16], 1u << sh[2 * j + 1]);
    }
    bool any = false;
#pragma unroll
    for (int k = 0; k < 8; ++k) any |= __builtin_amdgcn_ubfe(old[k], sh[k], 16) == 0xffffu;
    if (__builtin_expect(any, 0)) {
        for (int k = 0; k < 8; ++k) {
            const uint32_t s = (wd[k >> 1] >> (16 * (k & 1))) & 0xffffu;
            if (hist_needs_fix(s, old[k])) hist_fix(lds, hist, s, old[k], rec);
        }
    }
}

// Vectors [i0, end) of in4 with stride `step` from this thread's i0: software pipelined over
// kHistDepth register buffers (no copies). One workgroup per CU leaves 16 waves to cover
// HBM latency, so each lane keeps DEPTH - 1 loads in flight while one vector's LDS atomics
// run (loads and LDS ops use separate counters). Refills past the end re-read the last
// vector (branch-free, so the waits stay vmcnt(DEPTH - 1)); the tail counts what is left.
constexpr int kHistDepth = 8;
template <typename Rec = NoRec>
HZ_DEV void hist_sweep(uint32_t* lds, unsigned long long* hist, const uint4* in4, uint64_t i, uint64_t end,
                       uint64_t step, Rec rec = Rec()) {
    constexpr int D = kHistDepth;
    if (i >= end) return;
    const uint64_t last = end - 1;
    uint4 v[D];
#pragma unroll
    for (int k = 0; k < D; ++k) v[k] = in4[i + k * step < end ? i + k * step : last];
    for (; i + (D - 1) * step < end; i += D * step) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            hist_count8(lds, hist, v[k], rec);
            const uint64_t nx = i + (k + D) * step;
            v[k] = in4[nx < end ? nx : last];
        }
    }
#pragma unroll
    for (int k = 0; k < D - 1; ++k)
        if (i + k * step < end) hist_count8(lds, hist, v[k], rec);
}

// Adds the workgroup's LDS histogram to the global one.
HZ_DEV void hist_flush(const uint32_t* lds, unsigned long long* hist) {
    for (int i = threadIdx.x; i < 32768; i += blockDim.x) {
        const uint32_t v = lds[i];
        const uint32_t s2 = hist_word_inv((uint32_t)i) << 1;  // the symbol pair this word counts
        if (v & 0xffffu) atomicAdd(&hist[s2], (unsigned long long)(v & 0xffffu));
        if (v >> 16) atomicAdd(&hist[s2 + 1], (unsigned long long)(v >> 16));
    }
}

template <bool VEC>
__global__ __launch_bounds__(kHistThreads) void k_hist16(const uint8_t* __restrict__ in, uint64_t nsym,
                                                         unsigned long long* __restrict__ hist) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    for (int i = threadIdx.x; i < 32768; i += blockDim.x) lds[i] = 0;
    __syncthreads();
    uint64_t tail_begin = 0;
    if (VEC) {
        // the whole chip sweeps the input together (neighbouring 16 KiB pieces),
        // one vector (8 symbols) per lane per step
        const uint64_t nvec = nsym / 8;
        hist_sweep(lds, hist, reinterpret_cast<const uint4*>(in), (uint64_t)blockIdx.x * blockDim.x + threadIdx.x,
                   nvec, (uint64_t)gridDim.x * blockDim.x);
        tail_begin = nvec * 8;
    }
    // Scalar symbols: the < 8-symbol tail (VEC) or everything (unaligned input).
    {
        const uint64_t nscalar = nsym - tail_begin;
        const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
        for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < nscalar; k += stride) {
            const uint64_t i = tail_begin + k;
            hist_one(lds, hist, (uint32_t)in[2 * i] | ((uint32_t)in[2 * i + 1] << 8));
        }
    }
    __syncthreads();
    hist_flush(lds, hist);
}

// ---- range plan histogram (hz_internal.h RangeGeom) -------------------------
struct RangeArgs {
    uint32_t* snap;              // [nranges][32768] LDS images
    uint32_t* list;              // [groups][1 + list_cap] carry records
    unsigned long long* dot;     // [nranges]
    unsigned long long* start;   // [nranges + 1]
    uint64_t nsym, nblocks, bpr, nranges;
    uint32_t groups, list_cap;
    uint32_t* err;
};

static RangeArgs range_args(void* buf, const RangeGeom& g, uint32_t* err) {
    RangeArgs r;
    uint8_t* b = reinterpret_cast<uint8_t*>(buf);
    r.snap = reinterpret_cast<uint32_t*>(b);
    r.list = reinterpret_cast<uint32_t*>(b + g.off_list);
    r.dot = reinterpret_cast<unsigned long long*>(b + g.off_dot);
    r.start = reinterpret_cast<unsigned long long*>(b + g.off_start);
    r.nsym = g.nsym; r.nblocks = g.nblocks; r.bpr = g.bpr; r.nranges = g.nranges;
    r.groups = g.groups; r.list_cap = g.list_cap; r.err = err;
    return r;
}

// Workgroup g sweeps ranges g, g + groups, ... (each a contiguous stretch of whole
// blocks; the last one ends at the stream's end) and stores its CUMULATIVE LDS
// image after each: range j's bits are then dot(j) - dot(j - groups), the
// difference of two snapshots weighted by the code lengths plus the carries the
// workgroup made in between (k_range_dot). The global histogram equals k_hist16's.
// Input 16-byte aligned (ranges start on block boundaries: whole vectors).
__global__ __launch_bounds__(kHistThreads) void k_hist16_rng(const uint8_t* __restrict__ in,
                                                             unsigned long long* __restrict__ hist, RangeArgs r) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    for (int i = threadIdx.x; i < 32768; i += blockDim.x) lds[i] = 0;
    if (threadIdx.x == 0) r.list[(uint64_t)blockIdx.x * (1 + r.list_cap)] = 0u;
    __syncthreads();
    const uint4* in4 = reinterpret_cast<const uint4*>(in);
    uint32_t* list = r.list + (uint64_t)blockIdx.x * (1 + r.list_cap);
    uint32_t k = 0;  // the range's index among this workgroup's (< 2^15)
    for (uint64_t j = blockIdx.x; j < r.nranges; j += r.groups, ++k) {
        const uint64_t s0 = j * r.bpr * kBlockSyms;
        const uint64_t s1 = s0 + r.bpr * kBlockSyms < r.nsym ? s0 + r.bpr * kBlockSyms : r.nsym;
        auto rec = [&](uint32_t bin, uint32_t neg) {
            const uint32_t i = atomicAdd(list, 1u);
            if (i < r.list_cap) list[1 + i] = (k << 17) | (neg << 16) | bin;
            else atomicOr(r.err, 16u);  // cannot happen (RangeGeom bound): flagged, never silent
        };
        const uint64_t v1 = s1 / 8;
        hist_sweep(lds, hist, in4, s0 / 8 + threadIdx.x, v1, blockDim.x, rec);
        for (uint64_t q = v1 * 8 + threadIdx.x; q < s1; q += blockDim.x)  // the stream's < 8-symbol tail
            hist_one(lds, hist, (uint32_t)in[2 * q] | ((uint32_t)in[2 * q + 1] << 8), rec);
        __syncthreads();
        uint4* dst = reinterpret_cast<uint4*>(r.snap) + j * 8192;
        const uint4* src = reinterpret_cast<const uint4*>(lds);
        for (int q = threadIdx.x; q < 8192; q += blockDim.x) dst[q] = src[q];
        __syncthreads();
    }
    hist_flush(lds, hist);
}

hipError_t launch_hist16(const uint8_t* d_in, uint64_t n, unsigned long long* d_hist, int ncu, hipStream_t s) {
    const uint64_t nsym = n / 2;
    if (nsym == 0) return hipSuccess;
    const bool vec = (((uintptr_t)d_in) & 15) == 0;
    const void* fn = vec ? (const void*)k_hist16<true> : (const void*)k_hist16<false>;
    hipError_t e = ensure_lds_limit(fn, 131072);
    if (e != hipSuccess) return e;
    // One workgroup per CU; fewer for small inputs (every WG zeroes + flushes 128 KiB).
    uint64_t want = (nsym + 65535) / 65536;
    unsigned grid = (unsigned)(want < (uint64_t)ncu ? (want ? want : 1) : ncu);
    if (vec)
        hipLaunchKernelGGL(k_hist16<true>, dim3(grid), dim3(kHistThreads), 131072, s, d_in, nsym, d_hist);
    else
        hipLaunchKernelGGL(k_hist16<false>, dim3(grid), dim3(kHistThreads), 131072, s, d_in, nsym, d_hist);
    return hipGetLastError();
}

hipError_t launch_hist16_ranges(const uint8_t* d_in, uint64_t n, unsigned long long* d_hist, void* d_ranges,
                                uint32_t* d_err, hipStream_t s) {
    const RangeGeom g = range_geom(n / 2);
    if (!g.bytes || (((uintptr_t)d_in) & 15) || (((uintptr_t)d_ranges) & 15)) return hipErrorInvalidValue;
    hipError_t e = ensure_lds_limit((const void*)k_hist16_rng, 131072);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_hist16_rng, dim3(g.groups), dim3(kHistThreads), 131072, s, d_in, d_hist,
                       range_args(d_ranges, g, d_err));
    return hipGetLastError();
}

// ===========================================================================
// Pack. A block is 2048 symbols (4 KiB of input): one wavefront, 64 lanes x
// 32 contiguous symbols. Three stream-ordered steps replace the reference's
// populateCWLength + transform_inclusive_scan + encodeFromCW
// (Compressor.cu:50-61,541-576,182-313):
//   k_pack_count : per block, bit count and the block's last 32 code bits
//   k_scan_*     : exclusive scan of block bit counts -> absolute start bits
//   k_pack_write : per block, codeword lookup + wave scan of (bits, tail) +
//                  each lane writes the 32-bit words whose LAST bit falls in
//                  its run (every word written exactly once, plain stores, no
//                  pre-zeroing, no atomics, no inter-workgroup waits)
// Code tables live in LDS (DENSE 17-bit sentinel entries, or HOT tagged
// slots) and are loaded once per workgroup of a grid-stride kernel.
// ===========================================================================
struct PackArgs {
    const uint8_t* in;
    uint64_t nsym;
    uint64_t nblocks;
    const uint32_t* lds_img;
    uint32_t lds_words;
    const unsigned long long* wide;
    const uint32_t* esc;         // HOT escapes: len << 26 | code
    const uint32_t* len8_img;    // count pass: u8 lengths (LDS image, 64 KiB)
    uint32_t hot_mask;
    uint32_t hw_mask;            // HOT: 0x003f003f, in an SGPR (a literal keeps the compiler from one v_bitop3)
    uint32_t* out;
    uint64_t out_words;          // stores beyond this are dropped and flagged
    uint32_t lead;               // bits before the stream's first bit (header pending bits)
    unsigned long long* blk;     // per block bit count (k_pack_count)
    const unsigned long long* blk_start;
    unsigned long long* index;   // block index start[] (optional, hz_internal.h)
    unsigned long long* index_sub;  // block index sub[] (four u16 chain start bits per lane, low 16 bits)
    uint32_t* err;
    uint32_t slot_words;         // k_pack_write: per-wave LDS output slot (0: store from the lanes)
    const unsigned long long* rstart;  // range plan: start bit of every range (k_range_scan)
    uint64_t bpr, nranges;       // range plan: blocks per range, ranges
    // blocks k_pack_write leaves to k_pack_cold (all but WIDE): [0] = count, then (block, start bit)
    // pairs -- the stream's last block and blocks larger than the wave's LDS slot
    unsigned long long* cold;
};

template <int MODE> struct PackEnt { using T = uint32_t; static constexpr int kShift = 26; };
template <> struct PackEnt<ENC_WIDE> { using T = uint64_t; static constexpr int kShift = 56; };
// Code length of a register entry. A HOT hit keeps its slot's tag in bit 31, so the u32 forms
// read the 5-bit field (every u32 entry is <= 26 bits long: kNarrowMaxLen).
template <int MODE>
HZ_DEV uint32_t ent_len(typename PackEnt<MODE>::T e) {
    if constexpr (MODE == ENC_WIDE) return (uint32_t)(e >> 56);
    else return __builtin_amdgcn_ubfe((uint32_t)e, 26, 5);
}

template <typename T, int SH>
HZ_DEV T pack_dense_one(const uint32_t* lds, uint32_t s) {
    const uint32_t bit = s * 17u;
    const uint32_t w = bit >> 5;
    const uint64_t two = ((uint64_t)lds[w + 1] << 32) | lds[w];
    const uint32_t f = (uint32_t)(two >> (bit & 31)) & 0x1ffffu;
    const uint32_t L = f ? 16u - (uint32_t)__builtin_ctz(f) : 0u;
    return f ? (T)((L << SH) | (f >> (17u - L))) : (T)0;
}

// The lane's 32 input symbols (64 bytes) of block `blk` and, for lanes 0..31,
// one of the previous block's last 32 symbols. Issued one block ahead of use
// (k_pack_write); lanes past a full run load from the buffer start and are
// re-read byte by byte in pack_lookup.
struct PackIn {
    uint32_t raw[kSPT / 2];
    uint32_t psym;
    uint64_t bstart;
};

HZ_DEV void pack_prefetch(const PackArgs& a, uint64_t blk, int lane, PackIn& x) {
    const uint64_t sym0 = blk * kBlockSyms + (uint64_t)lane * kSPT;
    const uint64_t ls = sym0 + kSPT <= a.nsym ? sym0 : 0;
    const uint4* p = reinterpret_cast<const uint4*>(a.in + 2 * ls);
#pragma unroll
    for (int q = 0; q < kSPT / 8; ++q) {
        const uint4 v = p[q];
        x.raw[4 * q] = v.x; x.raw[4 * q + 1] = v.y; x.raw[4 * q + 2] = v.z; x.raw[4 * q + 3] = v.w;
    }
    const uint64_t ps = blk ? blk * kBlockSyms - 32 + (uint64_t)(lane & 31) : 0;
    x.psym = *reinterpret_cast<const uint16_t*>(a.in + 2 * ps);
    x.bstart = a.blk_start ? a.blk_start[blk] : 0;  // range pack: a running sum instead
}

// HOT lookups of one block in two halves, for k_pack_write's pipelined loop: issue (slot
// addresses, LDS reads, hit tests, the 33 escape loads) and, a block later, finish (the blends),
// so the escape loads' latency is covered by the previous block's count and emit.
struct HotLook {
    uint32_t x[kSPT], mk[kSPT], v[kSPT];
    uint32_t xx, xmk, xv;
};
// Slot arithmetic on both symbols of a word at once (packed 16-bit shifts): slot = s ^ (mask if
// bit 15), LDS word hot_word(slot); byte addresses (the table sits at LDS byte 0 of the pack
// kernels). A slot's entry carries its owner's bit 15 as the tag in bit 31: hit <=> bit 31 of
// entry ^ (s << 16) is 0. A miss is the slot's other symbol, whose entry the escape table holds at
// the same byte offset, so the escape address is one AND. !FULL: symbols k >= nvalid read 0.
template <bool FULL>
HZ_DEV void hot_issue(const PackArgs& a, const uint32_t (&raw)[kSPT / 2], uint32_t xs, HotLook& h, int nvalid = kSPT) {
    const uint32_t m2 = a.hot_mask | (a.hot_mask << 16);
    uint32_t ad[kSPT];
#pragma unroll
    for (int j = 0; j < kSPT / 2; ++j) {
        const uint32_t r = raw[j];
        // (inline asm with an inline-constant shift would shift the high half by 0: VOP3P takes
        // a constant for the low half only; vector types let the compiler place the operands)
        const uint32_t sgn = __builtin_bit_cast(uint32_t, __builtin_bit_cast(hz_i16x2, r) >> (hz_i16x2){15, 15});
        const uint32_t sl = r ^ (sgn & m2);
        const uint32_t hi8 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(hz_u16x2, sl) >> (hz_u16x2){8, 8});
        // hw = sl ^ (hi8 & 0x003f003f) as one v_bitop3 (the mask in an SGPR: the compiler emits an
        // AND and an XOR for the literal), and each half's slot byte address as one SDWA shift
        // (pack 8.62 -> 8.50 ms, A/B)
        uint32_t hw, a0, a1;
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x6c" : "=v"(hw) : "s"(a.hw_mask), "v"(sl), "v"(hi8));
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
            : "=v"(a0) : "v"(2u), "v"(hw));
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
            : "=v"(a1) : "v"(2u), "v"(hw));
        ad[2 * j] = a0;
        ad[2 * j + 1] = a1;
    }
#pragma unroll
    for (int k = 0; k < kSPT; ++k) {
        h.x[k] = lds_at(ad[k]);
        if (!FULL) h.x[k] = k < nvalid ? h.x[k] : 0u;
    }
    uint32_t xslot = xs ^ ((uint32_t)((int32_t)(xs << 16) >> 31) & a.hot_mask);
    xslot = hot_word(xslot & 0x7fffu) << 2;
    h.xx = lds_at(xslot);
    const char* esc = reinterpret_cast<const char*>(a.esc);
#pragma unroll
    for (int k = 0; k < kSPT; ++k) {
        const uint32_t tag = (k & 1) ? raw[k >> 1] : raw[k >> 1] << 16;
        h.mk[k] = (uint32_t)((int32_t)(h.x[k] ^ tag) >> 31);
        h.v[k] = *reinterpret_cast<const uint32_t*>(esc + (ad[k] & h.mk[k]));
    }
    h.xmk = (uint32_t)((int32_t)(h.xx ^ (xs << 16)) >> 31);
    h.xv = *reinterpret_cast<const uint32_t*>(esc + (xslot & h.xmk));
}
// the blend is a v_bfi the compiler cannot turn back into a select: written as `miss ? esc[s] : e`
// the loads become 33 exec-masked branches (12.73-12.87 vs 12.61-12.67 ms at 16 GiB Zipf, round 3 A/B)
HZ_DEV void hot_finish(const HotLook& h, uint32_t (&e)[kSPT], uint32_t& xe) {
#pragma unroll
    for (int k = 0; k < kSPT; ++k) {
        uint32_t r;
        asm volatile("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(h.mk[k]), "v"(h.v[k]), "v"(h.x[k]));
        e[k] = r;
    }
    uint32_t r;
    asm volatile("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(h.xmk), "v"(h.xv), "v"(h.xx));
    xe = r;
}

// (len, code) of the lane's 32 symbols in register format (len << SH | code),
// plus the entry of one more symbol `xs` (the previous block's tail). HOT
// slots hold tag << 31 | len << 26 | code, and every occurring symbol's code
// fits a slot (HOT mode needs max_len <= 25): an entry is a hit when its tag
// (bit 31) equals bit 15 of the symbol, i.e. when bit 31 of entry ^ tag is 0.
// Misses (the slot holds the partner symbol) come from the escape table, all
// issued before one wait. FULL: all 32 symbols valid (no per-symbol masking).
// mid() runs once the lookups' global loads are in flight and before any is
// waited on (k_pack_write issues the previous block's stores there).
struct NoMid {
    HZ_DEV void operator()() const {}
};
template <int MODE, bool FULL, typename Mid = NoMid>
HZ_DEV void pack_lookup(const PackArgs& a, const uint32_t* lds, uint64_t sym0, int nvalid, uint32_t (&raw)[kSPT / 2],
                        typename PackEnt<MODE>::T (&e)[kSPT], uint32_t xs, typename PackEnt<MODE>::T& xe,
                        Mid mid = Mid()) {
    using T = typename PackEnt<MODE>::T;
    constexpr int SH = PackEnt<MODE>::kShift;
    if (!FULL) {
#pragma unroll
        for (int k = 0; k < kSPT / 2; ++k) {
            uint32_t w = 0;
            if (2 * k < nvalid) w = (uint32_t)a.in[2 * (sym0 + 2 * k)] | ((uint32_t)a.in[2 * (sym0 + 2 * k) + 1] << 8);
            if (2 * k + 1 < nvalid)
                w |= ((uint32_t)a.in[2 * (sym0 + 2 * k + 1)] | ((uint32_t)a.in[2 * (sym0 + 2 * k + 1) + 1] << 8)) << 16;
            raw[k] = w;
        }
    }
    if constexpr (MODE == ENC_DENSE) {
#pragma unroll
        for (int k = 0; k < kSPT; ++k) {
            const uint32_t s = (raw[k >> 1] >> (16 * (k & 1))) & 0xffffu;
            const uint32_t bit = s * 17u;
            const uint32_t w = bit >> 5;
            const uint64_t two = ((uint64_t)lds[w + 1] << 32) | lds[w];
            const uint32_t f = (uint32_t)(two >> (bit & 31)) & 0x1ffffu;
            const uint32_t L = f ? 16u - (uint32_t)__builtin_ctz(f) : 0u;
            e[k] = ((FULL || k < nvalid) && f) ? (T)((L << SH) | (f >> (17u - L))) : (T)0;
        }
        xe = pack_dense_one<T, SH>(lds, xs);
        mid();
    } else if constexpr (MODE == ENC_HOT) {
        HotLook h;
        hot_issue<FULL>(a, raw, xs, h, nvalid);
        mid();
        hot_finish(h, e, xe);
    } else {
#pragma unroll
        for (int k = 0; k < kSPT; ++k) {
            const uint32_t s = (raw[k >> 1] >> (16 * (k & 1))) & 0xffffu;
            e[k] = (FULL || k < nvalid) ? (T)a.wide[s] : (T)0;
        }
        xe = (T)a.wide[xs];
        mid();
    }
}

template <int MODE>
HZ_DEV void load_lds_table(uint32_t* lds, const uint32_t* img, uint32_t words) {  // all but WIDE
    if (MODE != ENC_WIDE) {
        const uint4* src = reinterpret_cast<const uint4*>(img);
        uint4* dst = reinterpret_cast<uint4*>(lds);
        for (uint32_t i = threadIdx.x; i < words / 4; i += blockDim.x) dst[i] = src[i];
        __syncthreads();
    }
}

// Bit count per block from a 64 KiB u8 length table (one LDS read per symbol).
constexpr int kCountThreads = 1024;
constexpr int kCountUnroll = 2;  // blocks in flight per wave

__global__ __launch_bounds__(kCountThreads) void k_pack_count(PackArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    {
        const uint4* src = reinterpret_cast<const uint4*>(a.len8_img);
        uint4* dst = reinterpret_cast<uint4*>(lds);
        for (uint32_t i = threadIdx.x; i < kLen8LdsBytes / 16; i += blockDim.x) dst[i] = src[i];
        __syncthreads();
    }
    const uint8_t* l8 = reinterpret_cast<const uint8_t*>(lds);
    const int lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t full = a.nsym / kBlockSyms;  // blocks without a tail
    uint64_t blk = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    for (; blk + (kCountUnroll - 1) * W < full; blk += kCountUnroll * W) {
        uint4 v[kCountUnroll][kSPT / 8];
#pragma unroll
        for (int u = 0; u < kCountUnroll; ++u) {
            // the sum is order-free: instruction q reads bytes [1024 q + 16 lane, +16) (fully coalesced)
            const uint4* p = reinterpret_cast<const uint4*>(a.in + 2 * (blk + u * W) * kBlockSyms) + lane;
#pragma unroll
            for (int q = 0; q < kSPT / 8; ++q) v[u][q] = p[q * kWave];
        }
#pragma unroll
        for (int u = 0; u < kCountUnroll; ++u) {
            uint32_t n = 0;
#pragma unroll
            for (int q = 0; q < kSPT / 8; ++q) {
                const uint32_t wd[4] = {v[u][q].x, v[u][q].y, v[u][q].z, v[u][q].w};
#pragma unroll
                for (int k = 0; k < 8; ++k) n += l8[len8_index((wd[k >> 1] >> (16 * (k & 1))) & 0xffffu)];
            }
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) n += shfl_xor_u32(n, m);
            if (lane == 0) a.blk[blk + u * W] = n;
        }
    }
    for (; blk < a.nblocks; blk += W) {
        const uint64_t sym0 = blk * kBlockSyms + (uint64_t)lane * kSPT;
        uint32_t n = 0;
        if (blk < full) {
            const uint4* p = reinterpret_cast<const uint4*>(a.in + 2 * sym0);
#pragma unroll
            for (int q = 0; q < kSPT / 8; ++q) {
                const uint4 v = p[q];
                const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int k = 0; k < 8; ++k) n += l8[len8_index((wd[k >> 1] >> (16 * (k & 1))) & 0xffffu)];
            }
        } else {
            for (int k = 0; k < kSPT; ++k) {
                const uint64_t i = sym0 + k;
                if (i < a.nsym) n += l8[len8_index((uint32_t)a.in[2 * i] | ((uint32_t)a.in[2 * i + 1] << 8))];
            }
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) n += shfl_xor_u32(n, m);
        if (lane == 0) a.blk[blk] = n;
    }
}

// Emits the lane's codes into `dst` (LDS slot or global words) starting with
// `na` bits pending in `acc`; every completed 32-bit word is stored.
template <int MODE, bool TO_LDS, typename P>
HZ_DEV void pack_emit(const typename PackEnt<MODE>::T (&e)[kSPT], uint64_t& acc, uint32_t& na, P dst, bool ok) {
    using T = typename PackEnt<MODE>::T;
    constexpr int SH = PackEnt<MODE>::kShift;
    constexpr T CMASK = (T(1) << SH) - 1;
#pragma unroll
    for (int k = 0; k < kSPT; ++k) {
        const uint32_t L = ent_len<MODE>(e[k]);
        const uint64_t c = (uint64_t)(e[k] & CMASK);
        if (MODE == ENC_WIDE && L > 32) {
            const uint32_t Lh = L - 32;
            acc = (acc << Lh) | (c >> 32);
            na += Lh;
            if (na >= 32) { na -= 32; const uint32_t w = (uint32_t)(acc >> na); if (ok) *dst = TO_LDS ? w : bswap32(w); ++dst; }
            acc = (acc << 32) | (c & 0xffffffffull);
            na += 32;
            if (na >= 32) { na -= 32; const uint32_t w = (uint32_t)(acc >> na); if (ok) *dst = TO_LDS ? w : bswap32(w); ++dst; }
        } else if (L) {
            acc = (acc << L) | c;
            na += L;
            if (na >= 32) { na -= 32; const uint32_t w = (uint32_t)(acc >> na); if (ok) *dst = TO_LDS ? w : bswap32(w); ++dst; }
        }
    }
}

// Branch-free emit into the wave's LDS slot. t = bit position in the slot;
// after each code the last completed word, (t >> 5) - 1, is (re)written, so
// no per-code branch: a word is rewritten with the same bits until the next
// one completes. Before the lane completes its first word the write goes to
// that first word (clamp; overwritten once it completes -- every lane of a
// slot-path block holds >= 32 bits, so it does). On return the low t % 32
// bits of acc are the lane's trailing partial word.
template <int MODE>
HZ_DEV void pack_emit_lds(const typename PackEnt<MODE>::T (&e)[kSPT], uint64_t& acc, uint32_t t, uint32_t* slot) {
    constexpr int SH = PackEnt<MODE>::kShift;
    const uint32_t lo = (t >> 5) + 1;
    uint32_t* base = slot - 1;
#pragma unroll
    for (int k = 0; k < kSPT; ++k) {
        const uint32_t L = ent_len<MODE>(e[k]);
        const uint32_t c = (uint32_t)e[k] & ((1u << SH) - 1u);
        acc = (acc << L) | c;
        t += L;
        const uint32_t w = __builtin_amdgcn_alignbit((uint32_t)(acc >> 32), (uint32_t)acc, t);
        const uint32_t idx = (t >> 5) > lo ? (t >> 5) : lo;
        base[idx] = w;
    }
}

// <= 8 waves: room for a block of registers in flight per lane (16 GiB Zipf, round 3: 9 / 10 waves under a
// 168-VGPR cap 11.7 / 11.0 ms vs 8 waves 9.6 ms for k_pack_write)
constexpr int kPackMaxWaves = 8;
constexpr double kPackSlotMargin = 1.12;  // LDS output slot: the Kraft-estimated block bits x this
constexpr int kPackWriteThreads = 64 * kPackMaxWaves;
constexpr int kPackCopyIters = 16;       // slot copy-out covers 16 x 64 words: a 1024-word slot

// One block of a wave between its lookup and its emit: the lane's 32 entries,
// the entry of one of the previous block's last 32 symbols, the lane's bits,
// its offset in the block, its decode-chain offsets, and the block's bits
// (wave uniform).
template <int MODE>
struct PackBlk {
    typename PackEnt<MODE>::T e[kSPT];
    typename PackEnt<MODE>::T pe;
    uint32_t n, ex_n, bits;
    uint32_t nc[kChainsPerLane];
    int nvalid;
};

// FULL_ONLY: every lane's 32 symbols are in the stream (k_pack_write's split loop: the stream's last
// block, the only partial one, is packed again by k_pack_cold; this pass only needs its lookups to be
// in bounds, which pack_prefetch's clamp gives)
template <int MODE, bool FULL_ONLY = false, typename Mid = NoMid>
HZ_DEV void pack_block_lookup(const PackArgs& a, const uint32_t* lds, uint64_t blk, int lane, PackIn& in,
                              PackBlk<MODE>& b, Mid mid = Mid()) {
    const uint64_t sym0 = blk * kBlockSyms + (uint64_t)lane * kSPT;
    if constexpr (FULL_ONLY) {
        b.nvalid = kSPT;
        pack_lookup<MODE, true>(a, lds, sym0, b.nvalid, in.raw, b.e, in.psym, b.pe, mid);
        return;
    }
    b.nvalid = sym0 >= a.nsym ? 0 : (a.nsym - sym0 >= (uint64_t)kSPT ? kSPT : (int)(a.nsym - sym0));
    // a wave-uniform choice: mid() may run wave-wide code (DPP scans of the pipelined emit), so it
    // must not run once per branch of a divergent split (the stream's last block mixes full and
    // partial lanes; the partial path handles full lanes too)
    if (__ballot(b.nvalid != kSPT) == 0)
        pack_lookup<MODE, true>(a, lds, sym0, b.nvalid, in.raw, b.e, in.psym, b.pe, mid);
    else
        pack_lookup<MODE, false>(a, lds, sym0, b.nvalid, in.raw, b.e, in.psym, b.pe, mid);
}

// A block whose words wait in the wave's LDS slot: its global stores (payload
// copy-out and index entries) are issued during the NEXT block's lookup, after
// that block's escape loads. On gfx9 stores count in vmcnt and loads wait in
// order behind them, so stores issued just before a load wait stall the wave for
// their write latency; deferred, they complete under a whole block of work.
struct PackOut {
    bool pending, fits;
    uint64_t base4, blk, bstart, sub;
    uint32_t sh4, nwords;
};

HZ_DEV void pack_copyout(const PackArgs& a, const uint32_t* slot, int lane, const PackOut& p) {
    if (!p.pending) return;
    if (p.fits) {
        // Output words [wfirst, wfirst + nwords): a partial first 16-byte chunk
        // (its words before wfirst are the previous block's), whole chunks,
        // a partial last chunk. A fixed count of stores (1 + 4 + 1; lanes with
        // nothing to write rewrite the block's first word with its own value),
        // so later load waits count them statically. nwords >= 64.
        const uint32_t sh4 = p.sh4;
        const uint32_t wend = sh4 + p.nwords;                // slot index past the block
        const uint32_t cf = sh4 ? 1u : 0u, cl = wend >> 2;  // whole chunks [cf, cl)
        const uint32_t nhead = sh4 ? 4u - sh4 : 0u, ntail = wend & 3u;
        {
            const uint32_t i = (uint32_t)lane < nhead ? sh4 + (uint32_t)lane : sh4;
            a.out[p.base4 + i] = bswap32(slot[i]);
        }
#pragma unroll
        for (int it = 0; it < kPackCopyIters / 4; ++it) {
            uint32_t c = cf + (uint32_t)lane + (uint32_t)it * kWave;
            c = c < cl ? c : cl - 1;
            const uint4 v = reinterpret_cast<const uint4*>(slot)[c];
            reinterpret_cast<uint4*>(a.out + p.base4)[c] = make_uint4(bswap32(v.x), bswap32(v.y), bswap32(v.z), bswap32(v.w));
        }
        {
            const uint32_t i = (uint32_t)lane < ntail ? 4u * cl + (uint32_t)lane : sh4;
            a.out[p.base4 + i] = bswap32(slot[i]);
        }
    }
    if (a.index) {
        a.index_sub[p.blk * kWave + lane] = p.sub;
        if (lane == 0) a.index[p.blk] = p.bstart;
    }
    __builtin_amdgcn_wave_barrier();  // the slot's reads complete before the next emit rewrites it
}

// Lane bits, decode-chain offsets, wave scan of the bit counts.
template <int MODE>
HZ_DEV void pack_block_count(int lane, PackBlk<MODE>& b) {
    uint32_t n = 0;
#pragma unroll
    for (int k = 0; k < kSPT; ++k) {
        if (k % kChainSyms == 0) b.nc[k / kChainSyms] = n;
        n += ent_len<MODE>(b.e[k]);
    }
    const uint32_t sn = wave_incl_sum(n);
    b.n = n;
    b.ex_n = sn - n;
    b.bits = readlane(sn, 63);
}

// Writes block `blk` starting at absolute bit `bstart`, plus its index entries. SLOT_ONLY: the caller
// has checked that the block goes through the wave's LDS slot (not the last block, fits the slot), so
// the direct path is not compiled in.
template <int MODE, bool SLOT_ONLY = false>
HZ_DEV void pack_block_emit(const PackArgs& a, uint32_t* slot, uint64_t blk, int lane, const PackBlk<MODE>& b,
                            uint64_t bstart, uint64_t& max_bits, PackOut* defer = nullptr) {
    using T = typename PackEnt<MODE>::T;
    constexpr int SH = PackEnt<MODE>::kShift;
    constexpr T CMASK = (T(1) << SH) - 1;
    const uint64_t sym0 = blk * kBlockSyms + (uint64_t)lane * kSPT;
    const uint32_t n = b.n, ex_n = b.ex_n;
    const uint64_t bend = bstart + b.bits;
    // The 32 bits before the block: codes of the previous block's last 32
    // symbols (each code >= 1 bit), combined across lanes 0..31.
    uint32_t ptail = a.lead;
    if (blk > 0) {
        // Concatenation scan (associative; (0, 0) is its identity, which is what
        // DPP lanes without a source read) over lanes 0..31: rows, then row 0 into row 1.
        uint32_t pn = ent_len<MODE>(b.pe);
        uint32_t pt = (uint32_t)(b.pe & CMASK);  // low 32 bits of the code
        auto step = [&](uint32_t on, uint32_t ot) {
            pt = pn >= 32 ? pt : ((ot << pn) | pt);
            pn += on;
        };
        step(dpp0<kDppRowShr1>(pn), dpp0<kDppRowShr1>(pt));
        step(dpp0<kDppRowShr2>(pn), dpp0<kDppRowShr2>(pt));
        step(dpp0<kDppRowShr4>(pn), dpp0<kDppRowShr4>(pt));
        step(dpp0<kDppRowShr8>(pn), dpp0<kDppRowShr8>(pt));
        step(dpp0<kDppRowBcast15, 0xa>(pn), dpp0<kDppRowBcast15, 0xa>(pt));
        ptail = readlane(pt, 31);
    }
    const uint64_t o = bstart + ex_n;
    // every word this block writes lies below ceil(bend / 32)
    const bool fits = ((bend + 31) >> 5) <= a.out_words;
    if (!fits && lane == 0) atomicOr(a.err, 4u);
    const bool last = blk + 1 == a.nblocks;
    const uint64_t wfirst = bstart >> 5;
    const uint32_t nwords = (uint32_t)((bend >> 5) - wfirst);  // words completed inside the block
    const uint32_t sh4 = (uint32_t)(wfirst & 3);  // slot word i holds output word (wfirst & ~3) + i
    if (SLOT_ONLY || (slot && !last && nwords + sh4 <= a.slot_words)) {
        // Every lane holds 32 codes of >= 1 bit, so its last 32 bits are its
        // own: emit with the leading bits zero, then OR in the previous
        // lane's tail once all lanes are done. The slot is laid out like the
        // output modulo 16 bytes, so the copy-out moves aligned 16-byte chunks.
        uint32_t* sl = slot + sh4;  // sl[w] = output word wfirst + w
        uint64_t acc = 0;
        if constexpr (MODE == ENC_WIDE) {  // codes may exceed 32 bits
            uint32_t na = (uint32_t)(o & 31);
            pack_emit<MODE, true>(b.e, acc, na, sl + (uint32_t)((o >> 5) - wfirst), true);
        } else {
            pack_emit_lds<MODE>(b.e, acc, (uint32_t)(o - (wfirst << 5)), sl);
        }
        const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp((int)ptail, (int)(uint32_t)acc, kDppWaveShr1,
                                                                    0xf, 0xf, false);  // lane 0: ptail
        const uint32_t h = (uint32_t)(o & 31);
        if (h) sl[(uint32_t)((o >> 5) - wfirst)] |= prev << (32 - h);
        __builtin_amdgcn_wave_barrier();
        if (MODE != ENC_WIDE && defer) {
            defer->pending = true;
            defer->fits = fits;
            defer->base4 = wfirst & ~3ull;
            defer->sh4 = sh4;
            defer->nwords = nwords;
            defer->blk = blk;
            defer->bstart = bstart;
            uint64_t sub = 0;
#pragma unroll
            for (int c = 0; c < kChainsPerLane; ++c)
                sub |= (uint64_t)(((uint32_t)bstart + ex_n + b.nc[c]) & 0xffffu) << (16 * c);
            defer->sub = sub;
            max_bits = b.bits > max_bits ? b.bits : max_bits;
            return;
        }
        if (fits) {
            if constexpr (MODE != ENC_WIDE) {  // host: slot_words <= kPackCopyIters * kWave
                // Output words [wfirst, wfirst + nwords): a partial first 16-byte chunk
                // (its words before wfirst are the previous block's), whole chunks,
                // a partial last chunk. A fixed count of stores (1 + 4 + 1; lanes with
                // nothing to write rewrite the block's first word with its own value),
                // so later load waits count them statically. nwords >= 64.
                const uint64_t base4 = wfirst & ~3ull;
                const uint32_t wend = sh4 + nwords;                 // slot index past the block
                const uint32_t cf = sh4 ? 1u : 0u, cl = wend >> 2;  // whole chunks [cf, cl)
                const uint32_t nhead = sh4 ? 4u - sh4 : 0u, ntail = wend & 3u;
                {
                    const uint32_t i = (uint32_t)lane < nhead ? sh4 + (uint32_t)lane : sh4;
                    a.out[base4 + i] = bswap32(slot[i]);
                }
#pragma unroll
                for (int it = 0; it < kPackCopyIters / 4; ++it) {
                    uint32_t c = cf + (uint32_t)lane + (uint32_t)it * kWave;
                    c = c < cl ? c : cl - 1;
                    const uint4 v = reinterpret_cast<const uint4*>(slot)[c];
                    reinterpret_cast<uint4*>(a.out + base4)[c] =
                        make_uint4(bswap32(v.x), bswap32(v.y), bswap32(v.z), bswap32(v.w));
                }
                {
                    const uint32_t i = (uint32_t)lane < ntail ? 4u * cl + (uint32_t)lane : sh4;
                    a.out[base4 + i] = bswap32(slot[i]);
                }
            } else {
                for (uint32_t w = lane; w < nwords; w += kWave) a.out[wfirst + w] = bswap32(sl[w]);
            }
        }
        __builtin_amdgcn_wave_barrier();
    } else if constexpr (!SLOT_ONLY) {
        // direct path: each lane needs the 32 bits before its run from the
        // (bits, tail) scan, since a lane of the last block may hold < 32 bits
        uint64_t t64 = 0;
#pragma unroll
        for (int k = 0; k < kSPT; ++k) {
            const uint32_t L = ent_len<MODE>(b.e[k]);
            t64 = L ? ((t64 << L) | (uint64_t)(b.e[k] & CMASK)) : t64;
        }
        uint32_t tn = n, st = (uint32_t)t64;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t on = shfl_up_u32(tn, d), ot = shfl_up_u32(st, d);
            if (lane >= d) {
                st = tn >= 32 ? st : (tn == 0 ? ot : ((ot << tn) | st));
                tn += on;
            }
        }
        uint32_t ex_t = shfl_up_u32(st, 1);
        if (lane == 0) ex_t = 0;
        const uint32_t pre = ex_n >= 32 ? ex_t : (ex_n == 0 ? ptail : ((ptail << ex_n) | ex_t));
        uint32_t na = (uint32_t)(o & 31);
        uint64_t acc = na ? (uint64_t)(pre & ((1u << na) - 1u)) : 0ull;
        uint32_t* dst = a.out + (o >> 5);
        pack_emit<MODE, false>(b.e, acc, na, dst, fits);
        dst += (uint32_t)(((o & 31) + n) >> 5);
        if (fits && b.nvalid > 0 && sym0 + (uint64_t)b.nvalid == a.nsym && na > 0)
            *dst = bswap32((uint32_t)(acc << (32 - na)));
    }
    if (a.index) {  // block index (hz_internal.h): start bits + the lane's chain offsets
        uint64_t sub = 0;
#pragma unroll
        for (int c = 0; c < kChainsPerLane; ++c)
            sub |= (uint64_t)(((uint32_t)bstart + ex_n + b.nc[c]) & 0xffffu) << (16 * c);
        a.index_sub[blk * kWave + lane] = sub;
        if (lane == 0) {
            a.index[blk] = bstart;
            if (last) a.index[a.nblocks] = bend;
        }
        max_bits = bend - bstart > max_bits ? bend - bstart : max_bits;
    }
}


// Pack of blocks whose start bits are known: the three-pass pack (after
// k_pack_count + k_scan_*; wave w packs blocks w, w + W, ...) or, RNG, the
// range plan (after k_range_dot + k_range_scan; wave w packs the blocks of
// ranges w, w + W, ... in order, each block starting where the one before it
// ended: a running sum, no count pass).
template <int MODE, bool RNG, bool SPLIT>
__global__ __launch_bounds__(kPackWriteThreads) void k_pack_write(PackArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    load_lds_table<MODE>(lds, a.lds_img, a.lds_words);
    const int lane = threadIdx.x & 63;
    // Output slot of this wave: the block's words are assembled in LDS and
    // leave as contiguous 256-byte stores. A block that does not fit, and the
    // stream's last block, go to k_pack_cold (SPLIT: the host's choice when the
    // workgroup has slots; WIDE, and a DENSE table too large for slots beside
    // it, keep the in-line direct path): without that path in the loop the
    // kernel needs 70 SGPRs and 152 VGPRs instead of 106 (51 spilled to VGPR
    // lanes, reloaded every block) and 175 (pack 8.6 -> 8.1-8.3 ms, 16 GiB Zipf).
    constexpr bool kSplit = SPLIT && MODE != ENC_WIDE;
    // (the wave index stays a VGPR value here: as a scalar, 12.4-12.7 vs 11.8-12.2 ms pack stage)
    uint32_t* slot = a.slot_words ? lds + a.lds_words + (threadIdx.x >> 6) * a.slot_words : nullptr;
    const uint64_t W = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t gw = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    uint64_t max_bits = 0;  // largest block of this wave (index max_bits: one atomic per wave)
    uint64_t blk = gw, r = gw, rend = 0, run = 0;
    if (RNG) {
        blk = r < a.nranges ? r * a.bpr : a.nblocks;
        rend = blk + a.bpr < a.nblocks ? blk + a.bpr : a.nblocks;
        run = r < a.nranges ? a.rstart[r] : 0;
    }
    PackOut po;
    po.pending = false;
    if constexpr (MODE == ENC_HOT && kSplit) {
        // Pipelined: block k is finished (blends) and emitted while block k+1's escape loads and
        // block k+2's input are in flight; the wave's block sequence runs two ahead of the emit.
        // 239 VGPRs (LDS already holds the kernel at 2 waves per SIMD); pack 8.42 -> 8.33 ms mean
        // of 5 paired runs. The escapes cost issue/TA throughput more than latency: without them
        // pack takes 7.8-7.9 ms, and skipping a load no lane needs (a uniform branch) is slower
        // (8.95-9.06 ms: +2 VALU per symbol).
        auto next = [&](uint64_t b, bool& newr, uint64_t& nrun) -> uint64_t {
            newr = false;
            nrun = 0;
            if (!RNG) return b + W;
            if (b + 1 < rend) return b + 1;
            r += W;  // the wave's next range
            newr = true;
            const uint64_t n = r < a.nranges ? r * a.bpr : a.nblocks;
            rend = n + a.bpr < a.nblocks ? n + a.bpr : a.nblocks;
            nrun = r < a.nranges ? a.rstart[r] : 0;
            return n;
        };
        bool nb_newr;
        uint64_t nb_run;
        uint64_t nb = next(blk, nb_newr, nb_run);
        PackIn nx;
        HotLook hl;
        uint64_t bst_cur = run;
        if (blk < a.nblocks) {
            PackIn cur;
            pack_prefetch(a, blk, lane, cur);
            hot_issue<true>(a, cur.raw, cur.psym, hl);
            if (!RNG) bst_cur = cur.bstart;
            pack_prefetch(a, nb < a.nblocks ? nb : blk, lane, nx);
        }
        while (blk < a.nblocks) {
            bool nn_newr;
            uint64_t nn_run;
            const uint64_t nnb = next(nb, nn_newr, nn_run);
            PackBlk<MODE> b;
            hot_finish(hl, b.e, b.pe);
            b.nvalid = kSPT;
            // issue priority while the lookups and escape loads go out (the SIMD's other wave computes):
            // pack 8.31-8.33 -> 8.23-8.26 ms, A/B
            __builtin_amdgcn_s_setprio(2);
            hot_issue<true>(a, nx.raw, nx.psym, hl);  // block k+1 (past the wave's end: a repeat, unused)
            __builtin_amdgcn_s_setprio(0);
            const uint64_t nbst = nx.bstart;
            pack_copyout(a, slot, lane, po);  // block k-1's stores, behind the escape loads
            po.pending = false;
            const uint64_t pb = nnb < a.nblocks ? nnb : (nb < a.nblocks ? nb : blk);
            pack_prefetch(a, pb, lane, nx);
            pack_block_count<MODE>(lane, b);
            const uint64_t bst = bst_cur;
            const uint64_t wfirst = bst >> 5;
            const uint32_t nwords = (uint32_t)(((bst + b.bits) >> 5) - wfirst), sh4 = (uint32_t)(wfirst & 3);
            if (blk + 1 == a.nblocks || nwords + sh4 > a.slot_words) {
                if (lane == 0) {
                    const unsigned long long i = atomicAdd(a.cold, 1ull);
                    a.cold[1 + 2 * i] = blk;
                    a.cold[2 + 2 * i] = bst;
                }
            } else {
                pack_block_emit<MODE, true>(a, slot, blk, lane, b, bst, max_bits, &po);
            }
            if (RNG) run = nb_newr ? nb_run : run + b.bits;
            bst_cur = RNG ? run : nbst;
            blk = nb;
            nb = nnb;
            nb_newr = nn_newr;
            nb_run = nn_run;
        }
        pack_copyout(a, slot, lane, po);
        if (a.index && lane == 0 && max_bits) atomicMax(a.index + a.nblocks + 1, (unsigned long long)max_bits);
        return;
    }
    PackIn nx;  // the next block's inputs, in flight while this block is packed
    if (blk < a.nblocks) pack_prefetch(a, blk, lane, nx);
    while (blk < a.nblocks) {
        uint64_t nb = blk + W, nrun = 0;
        bool newr = false;
        if (RNG) {
            if (blk + 1 < rend) {
                nb = blk + 1;
            } else {  // the wave's next range: its start bit lands during this block
                r += W;
                newr = true;
                nb = r < a.nranges ? r * a.bpr : a.nblocks;
                rend = nb + a.bpr < a.nblocks ? nb + a.bpr : a.nblocks;
                nrun = r < a.nranges ? a.rstart[r] : 0;
            }
        }
        PackIn cur = nx;
        PackBlk<MODE> b;
        // the previous block's stores go out behind this block's escape loads
        pack_block_lookup<MODE, kSplit>(a, lds, blk, lane, cur, b, [&]() { pack_copyout(a, slot, lane, po); });
        po.pending = false;
        // next block's loads: after this block's escapes, so no wait covers them early
        pack_prefetch(a, nb < a.nblocks ? nb : blk, lane, nx);
        pack_block_count<MODE>(lane, b);
        const uint64_t bst = RNG ? run : cur.bstart;
        if constexpr (kSplit) {
            const uint64_t wfirst = bst >> 5;
            const uint32_t nwords = (uint32_t)(((bst + b.bits) >> 5) - wfirst), sh4 = (uint32_t)(wfirst & 3);
            if (blk + 1 == a.nblocks || nwords + sh4 > a.slot_words) {  // slot_words 0: no slots, all cold
                if (lane == 0) {
                    const unsigned long long i = atomicAdd(a.cold, 1ull);
                    a.cold[1 + 2 * i] = blk;
                    a.cold[2 + 2 * i] = bst;
                }
            } else {
                pack_block_emit<MODE, true>(a, slot, blk, lane, b, bst, max_bits, &po);
            }
        } else {
            pack_block_emit<MODE>(a, slot, blk, lane, b, bst, max_bits, &po);
        }
        if (RNG) run = newr ? nrun : run + b.bits;
        blk = nb;
    }
    pack_copyout(a, slot, lane, po);
    if (a.index && lane == 0 && max_bits) atomicMax(a.index + a.nblocks + 1, (unsigned long long)max_bits);
}

// The blocks k_pack_write listed in a.cold (the stream's last block, which may be partial, and blocks
// larger than a wave's LDS slot): per-symbol masked lookups, each lane's codes stored straight to the
// output, the index entries. Usually one block; workgroups past the list leave before loading the table.
template <int MODE>
__global__ __launch_bounds__(kPackWriteThreads) void k_pack_cold(PackArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint64_t n = a.cold[0];
    const uint64_t waves = blockDim.x >> 6, W = (uint64_t)gridDim.x * waves;
    if ((uint64_t)blockIdx.x * waves >= n) return;  // uniform over the workgroup
    load_lds_table<MODE>(lds, a.lds_img, a.lds_words);
    const int lane = threadIdx.x & 63;
    uint64_t max_bits = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * waves + (threadIdx.x >> 6); i < n; i += W) {
        const uint64_t blk = a.cold[1 + 2 * i], bst = a.cold[2 + 2 * i];
        PackIn in;
        pack_prefetch(a, blk, lane, in);
        PackBlk<MODE> b;
        pack_block_lookup<MODE>(a, lds, blk, lane, in, b);
        pack_block_count<MODE>(lane, b);
        pack_block_emit<MODE>(a, nullptr, blk, lane, b, bst, max_bits, nullptr);
    }
    if (a.index && lane == 0 && max_bits) atomicMax(a.index + a.nblocks + 1, (unsigned long long)max_bits);
}

// ---- every code 16 bits (U = 65 536, min_len = max_len = 16) ---------------
// Symbol i starts at bit start_bit + 16 i: no count pass and no scan. Lane j
// packs symbols [32 j, 32 j + 32) into the 16 words whose last bit lies in its
// run; word t is a funnel shift of code pairs t-1 and t by start_bit % 32.
// Full blocks [0, nb) of a FIXED16 stream: one wave per block; lane l's sub-run c is the block's symbols 8 (64 c + l) .. + 7, i.e. 16 input bytes and 4
// output words at 1 KiB-coalesced offsets (the lane-run kernel below moves 64 contiguous bytes per
// lane, so each of its 16-byte accesses touches 64 separate pieces). Word t of a sub-run is a funnel
// shift of code pairs t - 1 and t; pair -1 is lane l - 1's last (DPP), sub-run c - 1's lane 63 for
// lane 0, or, for the block's first, the pair before the block (loaded) or the header's pending bits.
__global__ __launch_bounds__(kPackThreads) void k_pack_fixed16_blk(PackArgs a, uint64_t start_bit, uint64_t nb) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    load_lds_table<ENC_FIXED16>(lds, a.lds_img, a.lds_words);
    const uint16_t* c16 = reinterpret_cast<const uint16_t*>(lds);
    const uint32_t sb = (uint32_t)(start_bit & 31);
    const int lane = threadIdx.x & 63;
    const uint4* in4 = reinterpret_cast<const uint4*>(a.in);
    u32x4a4* out4 = reinterpret_cast<u32x4a4*>(a.out + (start_bit >> 5));  // any word of the stream
    const uint64_t W = (uint64_t)gridDim.x * (blockDim.x >> 6);
    uint64_t b = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    auto load = [&](uint64_t bb, uint4 (&x)[kChainsPerLane]) {
        bb = bb < nb ? bb : 0;
#pragma unroll
        for (int c = 0; c < kChainsPerLane; ++c) x[c] = in4[bb * (kBlockSyms / 8) + c * kWave + lane];
    };
    uint4 nx[kChainsPerLane];
    if (b < nb) load(b, nx);
    for (; b < nb; b += W) {
        uint4 x[kChainsPerLane];
#pragma unroll
        for (int c = 0; c < kChainsPerLane; ++c) x[c] = nx[c];
        load(b + W, nx);
        uint32_t p0 = a.lead;  // the pair before the block (same address on every lane)
        if (b > 0) {
            const uint32_t pr = *reinterpret_cast<const uint32_t*>(a.in + 2 * (b * kBlockSyms - 2));
            p0 = ((uint32_t)c16[pr & 0xffffu] << 16) | c16[pr >> 16];
        }
        uint32_t last = p0;  // sub-run c - 1's last pair on lane 63 (wave-uniform)
#pragma unroll
        for (int c = 0; c < kChainsPerLane; ++c) {
            const uint32_t raw[4] = {x[c].x, x[c].y, x[c].z, x[c].w};
            uint32_t v[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) v[t] = ((uint32_t)c16[raw[t] & 0xffffu] << 16) | c16[raw[t] >> 16];
            uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[3], kDppWaveShr1, 0xf, 0xf, false);
            if (lane == 0) prev = last;
            last = readlane(v[3], 63);
            uint32_t o[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const uint32_t pp = t ? v[t - 1] : prev;
                o[t] = sb ? __builtin_amdgcn_alignbit(pp, v[t], sb) : v[t];
            }
            u32x4a4 ov;
            ov.x = bswap32(o[0]); ov.y = bswap32(o[1]); ov.z = bswap32(o[2]); ov.w = bswap32(o[3]);
            out4[b * (kBlockSyms / 8) + c * kWave + lane] = ov;
        }
        if (a.index) {
            const uint32_t bs = (uint32_t)(start_bit + (uint64_t)b * kBlockSyms * 16);
            uint64_t sub = 0;
#pragma unroll
            for (int c = 0; c < kChainsPerLane; ++c)
                sub |= (uint64_t)((bs + 16u * (kSPT * (uint32_t)lane + kChainSyms * c)) & 0xffffu) << (16 * c);
            a.index_sub[b * kWave + lane] = sub;
            if (lane == 0) a.index[b] = start_bit + (uint64_t)b * kBlockSyms * 16;
            if (b == 0 && lane == 0) a.index[a.nblocks + 1] = 16ull * kBlockSyms;
        }
    }
}

// Lane runs [j_begin, ...) of 32 symbols (the stream's tail after k_pack_fixed16_blk, or all of it).
__global__ __launch_bounds__(kPackThreads) void k_pack_fixed16(PackArgs a, uint64_t start_bit, uint64_t j_begin) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    load_lds_table<ENC_FIXED16>(lds, a.lds_img, a.lds_words);
    const uint16_t* c16 = reinterpret_cast<const uint16_t*>(lds);
    const uint32_t sb = (uint32_t)(start_bit & 31);
    const uint64_t W0 = start_bit >> 5;
    const uint64_t nl = (a.nsym + kSPT - 1) / kSPT;
    const uint64_t end_word = (start_bit + 16 * a.nsym + 31) >> 5;  // words holding stream bits
    const bool fits = end_word <= a.out_words;
    if (!fits && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.err, 4u);
    const bool vec_out = (W0 & 3) == 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    // the lane's 64 input bytes of run j (full runs; 0 past them), loaded one
    // iteration ahead so a load is always in flight beside the table lookups
    auto load_run = [&](uint64_t j, uint32_t (&raw)[kSPT / 2]) {
        const uint64_t ls = j < nl && (j + 1) * kSPT <= a.nsym ? j * kSPT : 0;
        const uint4* p = reinterpret_cast<const uint4*>(a.in + 2 * ls);
#pragma unroll
        for (int q = 0; q < kSPT / 8; ++q) {
            const uint4 v = p[q];
            raw[4 * q] = v.x; raw[4 * q + 1] = v.y; raw[4 * q + 2] = v.z; raw[4 * q + 3] = v.w;
        }
    };
    uint32_t nraw[kSPT / 2];
    const uint64_t j0 = j_begin + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    load_run(j0, nraw);
    for (uint64_t j = j0; j < nl; j += stride) {  // the loop is uniform except in the last round
        const uint64_t sym0 = j * kSPT;
        const int nvalid = a.nsym - sym0 >= (uint64_t)kSPT ? kSPT : (int)(a.nsym - sym0);
        uint32_t raw[kSPT / 2];
#pragma unroll
        for (int k = 0; k < kSPT / 2; ++k) raw[k] = nraw[k];
        load_run(j + stride, nraw);
        if (nvalid != kSPT) {
#pragma unroll
            for (int k = 0; k < kSPT / 2; ++k) raw[k] = 0;
            for (int k = 0; k < nvalid; ++k)
                raw[k >> 1] |= ((uint32_t)a.in[2 * (sym0 + k)] | ((uint32_t)a.in[2 * (sym0 + k) + 1] << 8)) << (16 * (k & 1));
        }
        uint32_t v[kSPT / 2];
#pragma unroll
        for (int t = 0; t < kSPT / 2; ++t) {
            const uint32_t lo = (uint32_t)c16[raw[t] & 0xffffu], hi = (uint32_t)c16[raw[t] >> 16];
            v[t] = (2 * t < nvalid ? lo << 16 : 0u) | (2 * t + 1 < nvalid ? hi : 0u);
        }
        // the previous run's last code pair (or the header's pending bits): from
        // lane - 1 by DPP (run j - 1 when that lane is active in this round), else loaded
        uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[kSPT / 2 - 1], kDppWaveShr1, 0xf, 0xf, false);
        if ((threadIdx.x & 63) == 0 && j > 0) {
            const uint32_t pr = *reinterpret_cast<const uint32_t*>(a.in + 2 * (sym0 - 2));
            prev = ((uint32_t)c16[pr & 0xffffu] << 16) | c16[pr >> 16];
        }
        if (j == 0) prev = a.lead;
        uint32_t o[kSPT / 2];
#pragma unroll
        for (int t = 0; t < kSPT / 2; ++t) {
            const uint32_t p = t ? v[t - 1] : prev;
            o[t] = sb ? (uint32_t)(((((uint64_t)p) << 32) | v[t]) >> sb) : v[t];
        }
        const uint64_t wj = W0 + 16 * j;
        if (fits) {
            if (nvalid == kSPT && j + 1 < nl && vec_out) {
                uint4* d = reinterpret_cast<uint4*>(a.out + wj);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    d[q] = make_uint4(bswap32(o[4 * q]), bswap32(o[4 * q + 1]), bswap32(o[4 * q + 2]), bswap32(o[4 * q + 3]));
            } else {
                // words whose first bit is a stream bit; the last lane also
                // writes the word its final bits spill into
#pragma unroll
                for (int t = 0; t < kSPT / 2; ++t)
                    if (wj + t < end_word) a.out[wj + t] = bswap32(o[t]);
                if (j + 1 == nl && wj + 16 < end_word)
                    a.out[wj + 16] = bswap32((uint32_t)(((uint64_t)v[15] << 32) >> sb));
            }
        }
        if (a.index) {
            const uint64_t blk = j / kWave;
            const uint32_t lane = (uint32_t)(j % kWave);
            const uint32_t cnt = (uint32_t)(a.nsym - blk * kBlockSyms < (uint64_t)kBlockSyms ? a.nsym - blk * kBlockSyms
                                                                                        : (uint64_t)kBlockSyms);
            uint64_t sub = 0;
            const uint32_t bs = (uint32_t)(start_bit + (uint64_t)blk * kBlockSyms * 16);
#pragma unroll
            for (int c = 0; c < kChainsPerLane; ++c) {
                const uint32_t at = kSPT * lane + kChainSyms * c;
                sub |= (uint64_t)((bs + 16 * (at < cnt ? at : cnt)) & 0xffffu) << (16 * c);
            }
            a.index_sub[j] = sub;
            if (lane == 0) a.index[blk] = start_bit + (uint64_t)blk * kBlockSyms * 16;
            if (j + 1 == nl) a.index[a.nblocks] = start_bit + 16 * a.nsym;
            if (j == 0) a.index[a.nblocks + 1] = 16ull * (a.nsym < (uint64_t)kBlockSyms ? a.nsym : (uint64_t)kBlockSyms);
        }
    }
}

// ---- exclusive scan of block bit counts (low 32 bits of blk[]) -------------
constexpr int kScanThreads = 1024;
constexpr int kScanPer = 16;                         // counts per thread
constexpr int kScanTile = kScanThreads * kScanPer;   // 16 384 blocks per tile

HZ_DEV uint64_t block_exclusive_scan(uint64_t v, uint64_t* sh, uint64_t& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t lo = shfl_up_u32((uint32_t)x, d), hi = shfl_up_u32((uint32_t)(x >> 32), d);
        if (lane >= d) x += ((uint64_t)hi << 32) | lo;
    }
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t s = 0;
        for (int w = 0; w < nw; ++w) { const uint64_t t = sh[w]; sh[w] = s; s += t; }
        sh[nw] = s;
    }
    __syncthreads();
    total = sh[nw];
    const uint64_t r = sh[wid] + x - v;
    __syncthreads();
    return r;
}

// mask: the bits of each entry that are its count (the pack's block entries: the low 32; chain counts: all)
__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const unsigned long long* blk, uint64_t nblocks,
                                                              unsigned long long* tile_sum, uint64_t mask) {
    __shared__ uint64_t sh[17];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPer;
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k)
        if (base + k < nblocks) s += blk[base + k] & mask;
    uint64_t total;
    block_exclusive_scan(s, sh, total);
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_tiles(unsigned long long* tile_sum, uint64_t ntiles,
                                                             uint64_t start_bit) {
    __shared__ uint64_t sh[17];
    uint64_t carry = start_bit;
    for (uint64_t b = 0; b < ntiles; b += kScanThreads) {
        const uint64_t i = b + threadIdx.x;
        const uint64_t v = i < ntiles ? tile_sum[i] : 0;
        uint64_t total;
        const uint64_t ex = block_exclusive_scan(v, sh, total);
        if (i < ntiles) tile_sum[i] = carry + ex;
        carry += total;
    }
}

__global__ __launch_bounds__(kScanThreads) void k_scan_apply(const unsigned long long* blk, uint64_t nblocks,
                                                             const unsigned long long* tile_off,
                                                             unsigned long long* blk_start, uint64_t mask) {
    __shared__ uint64_t sh[17];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPer;
    uint64_t c[kScanPer];
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        c[k] = base + k < nblocks ? blk[base + k] & mask : 0u;
        s += c[k];
    }
    uint64_t total;
    uint64_t run = tile_off[blockIdx.x] + block_exclusive_scan(s, sh, total);
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        if (base + k < nblocks) blk_start[base + k] = run;
        run += c[k];
    }
}

// ---- range plan: bits and start of every range ------------------------------
// dot[j] = sum over bins of len * (the cumulative count of workgroup j % groups
// after its range j): the snapshot's u16 halves plus 65 536 x its carry records
// up to range j. lenpair: the two code lengths of every histogram word (u8 each,
// hist_word order, hz_codebook_upload_encode).
constexpr int kDotThreads = 256;
__global__ __launch_bounds__(kDotThreads) void k_range_dot(RangeArgs r, const uint32_t* __restrict__ lenpair) {
    __shared__ unsigned long long red[kDotThreads / 64];
    const uint16_t* lp16 = reinterpret_cast<const uint16_t*>(lenpair);
    for (uint64_t j = blockIdx.x; j < r.nranges; j += gridDim.x) {
        const uint4* sp = reinterpret_cast<const uint4*>(r.snap) + j * 8192;
        const uint2* lp = reinterpret_cast<const uint2*>(lenpair);  // 4 length pairs per 16 snapshot bytes
        auto mac = [](uint32_t v, uint32_t l) { return (v & 0xffffu) * (l & 0xffu) + (v >> 16) * ((l >> 8) & 0xffu); };
        uint32_t acc = 0;  // <= 32 x 4 x 2 x 65535 x 56 < 2^32
        for (uint32_t q = threadIdx.x; q < 8192; q += kDotThreads) {
            const uint4 v = sp[q];
            const uint2 l = lp[q];
            acc += mac(v.x, l.x) + mac(v.y, l.x >> 16) + mac(v.z, l.y) + mac(v.w, l.y >> 16);
        }
        uint64_t sum = acc;
        const uint32_t g = (uint32_t)(j % r.groups), k = (uint32_t)(j / r.groups);
        const uint32_t* list = r.list + (uint64_t)g * (1 + r.list_cap);
        const uint32_t n = list[0] < r.list_cap ? list[0] : r.list_cap;
        for (uint32_t t = threadIdx.x; t < n; t += kDotThreads) {
            const uint32_t e = list[1 + t];
            if ((e >> 17) > k) continue;
            const uint32_t bin = e & 0xffffu;
            const uint64_t L = (lp16[hist_word(bin)] >> (8 * (bin & 1))) & 0xffu;
            sum += (e >> 16) & 1u ? (uint64_t)0 - (L << 16) : L << 16;  // mod 2^64: the total is >= 0
        }
        sum = wave_sum_u64(sum);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t t = 0;
            for (int w = 0; w < kDotThreads / 64; ++w) t += red[w];
            r.dot[j] = t;
        }
        __syncthreads();
    }
}

// start[j] = start_bit + sum of bits of ranges < j; bits_j = dot[j] - dot[j - groups]
// (the same workgroup's previous snapshot); start[nranges] = the stream's end.
__global__ __launch_bounds__(kScanThreads) void k_range_scan(RangeArgs r, uint64_t start_bit) {
    __shared__ uint64_t sh[17];
    uint64_t carry = start_bit;
    for (uint64_t b = 0; b < r.nranges; b += kScanThreads) {
        const uint64_t j = b + threadIdx.x;
        const uint64_t v = j < r.nranges ? r.dot[j] - (j >= r.groups ? r.dot[j - r.groups] : 0ull) : 0ull;
        uint64_t total;
        const uint64_t ex = block_exclusive_scan(v, sh, total);
        if (j < r.nranges) r.start[j] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0) r.start[r.nranges] = carry;
}

uint64_t pack_scratch_words(uint64_t nsym) {
    const uint64_t nblocks = (nsym + kBlockSyms - 1) / kBlockSyms;
    const uint64_t ntiles = (nblocks + kScanTile - 1) / kScanTile;
    return 2 * nblocks + ntiles + 1 + 2 * nblocks;  // counts, starts, scan tiles, k_pack_cold's list
}

// The k_pack_write instance: SPLIT (cold blocks to k_pack_cold) for HOT, and for DENSE when the
// workgroup has output slots; WIDE and a slot-less DENSE keep the direct path in the loop (split,
// every block of a slot-less pack would be looked up twice).
static const void* pack_write_fn(int mode, bool rng, bool split) {
    if (mode == ENC_HOT) return rng ? (const void*)k_pack_write<ENC_HOT, true, true> : (const void*)k_pack_write<ENC_HOT, false, true>;
    if (mode == ENC_DENSE) {
        if (split) return rng ? (const void*)k_pack_write<ENC_DENSE, true, true> : (const void*)k_pack_write<ENC_DENSE, false, true>;
        return rng ? (const void*)k_pack_write<ENC_DENSE, true, false> : (const void*)k_pack_write<ENC_DENSE, false, false>;
    }
    return rng ? (const void*)k_pack_write<ENC_WIDE, true, false> : (const void*)k_pack_write<ENC_WIDE, false, false>;
}
static hipError_t pack_write_launch(const void* fn, uint64_t grid, int threads, uint32_t lds, hipStream_t s, PackArgs a) {
    void* args[] = {&a};
    return hipLaunchKernel(fn, dim3((uint32_t)grid), dim3(threads), args, lds, s);
}

// k_pack_write's list of blocks for k_pack_cold: zero the count first, run the cold pass after.
static hipError_t pack_cold_reset(const PackArgs& a, hipStream_t s) {
    return hipMemsetAsync(a.cold, 0, sizeof(unsigned long long), s);
}
static void pack_cold_launch(const Tables& t, const PackArgs& a, uint32_t lds, int ncu, hipStream_t s) {
    const uint64_t waves = kPackWriteThreads / 64;
    uint64_t g = (a.nblocks + waves - 1) / waves;
    if (g > (uint64_t)ncu) g = ncu;  // table-sized LDS: one workgroup per CU
    switch (t.enc_mode) {
        case ENC_DENSE: hipLaunchKernelGGL(k_pack_cold<ENC_DENSE>, dim3(g), dim3(kPackWriteThreads), lds, s, a); break;
        case ENC_HOT: hipLaunchKernelGGL(k_pack_cold<ENC_HOT>, dim3(g), dim3(kPackWriteThreads), lds, s, a); break;
        default: break;  // WIDE keeps the direct path inside k_pack_write
    }
}

hipError_t launch_pack(const Tables& t, const uint8_t* d_in, uint64_t nsym, uint64_t start_bit, uint32_t lead,
                       uint32_t* d_out, uint64_t out_words, unsigned long long* d_scratch,
                       unsigned long long* d_index, uint32_t* d_err, int ncu, hipStream_t s, void* d_ranges,
                       int* used_ranges) {
    if (used_ranges) *used_ranges = 0;
    if (nsym == 0) return hipSuccess;
    const uint64_t nblocks = (nsym + kBlockSyms - 1) / kBlockSyms;
    const uint64_t ntiles = (nblocks + kScanTile - 1) / kScanTile;
    PackArgs a;
    a.in = d_in; a.nsym = nsym; a.nblocks = nblocks;
    a.lds_img = t.d_enc_lds; a.lds_words = t.enc_lds_bytes / 4;
    a.wide = reinterpret_cast<const unsigned long long*>(t.d_enc_wide);
    a.esc = t.d_enc_esc; a.len8_img = t.d_len8; a.hot_mask = t.hot_mask; a.hw_mask = 0x003f003fu;
    a.out = d_out; a.out_words = out_words; a.lead = lead;
    a.blk = d_scratch;
    unsigned long long* blk_start = d_scratch + nblocks;
    unsigned long long* tiles = d_scratch + 2 * nblocks;
    a.blk_start = blk_start; a.index = d_index; a.err = d_err;
    a.index_sub = d_index ? d_index + index_sub_offset(nblocks) : nullptr;
    a.rstart = nullptr; a.bpr = 0; a.nranges = 0;
    a.cold = tiles + ntiles;
    if (d_index && t.enc_mode != ENC_FIXED16) {
        hipError_t e = hipMemsetAsync(d_index + nblocks + 1, 0, 8, s);  // max_bits, raised per block
        if (e != hipSuccess) return e;
    }
    if (t.enc_mode == ENC_FIXED16) {
        hipError_t e = ensure_lds_limit((const void*)k_pack_fixed16, kFixed16LdsBytes);
        if (e != hipSuccess) return e;
        if ((e = ensure_lds_limit((const void*)k_pack_fixed16_blk, kFixed16LdsBytes)) != hipSuccess) return e;
        const uint64_t nl = (nsym + kSPT - 1) / kSPT;
        // every block but the last through the coalesced kernel when it fits; the lane-run kernel
        // takes the rest (the stream's end, the index end)
        const uint64_t nb = nblocks - 1;
        const bool blk = kFixed16Blk && nb > 0 && (start_bit >> 5) + nb * (kBlockSyms / 2) <= out_words;
        uint64_t jb = 0;
        if (blk) {
            uint64_t wgs = (nb + kPackThreads / 64 - 1) / (kPackThreads / 64);
            if (wgs > (uint64_t)ncu) wgs = ncu;  // 128 KiB table: one workgroup per CU
            hipLaunchKernelGGL(k_pack_fixed16_blk, dim3(wgs), dim3(kPackThreads), kFixed16LdsBytes, s, a, start_bit, nb);
            jb = nb * kWave;
        }
        uint64_t wgs = (nl - jb + kPackThreads - 1) / kPackThreads;
        if (wgs > (uint64_t)ncu) wgs = ncu;  // 128 KiB table: one workgroup per CU
        hipLaunchKernelGGL(k_pack_fixed16, dim3(wgs), dim3(kPackThreads), kFixed16LdsBytes, s, a, start_bit, jb);
        return hipGetLastError();
    }
    // Waves per workgroup: as many output slots of the expected block size
    // (Kraft estimate from the code lengths, +12 %) as fit beside the table.
    const uint32_t table_words = t.enc_mode == ENC_WIDE ? 0 : t.enc_lds_bytes / 4;
    a.lds_words = table_words;
    const uint32_t free_words = kLdsBytes / 4 - table_words;
    const uint32_t est_words = (uint32_t)(t.enc_avg_bits * kBlockSyms * kPackSlotMargin / 32.0) + 4;
    constexpr uint32_t kMaxWaves = kPackWriteThreads / 64;
    uint32_t waves = free_words / est_words;
    waves = waves > kMaxWaves ? kMaxWaves : waves;
    a.slot_words = 0;
    if (waves >= 6) a.slot_words = free_words / waves & ~3u;  // 16-byte aligned slots
    else waves = kMaxWaves;  // no room for slots: lanes store directly
    if (t.enc_mode != ENC_WIDE && a.slot_words > (uint32_t)(kPackCopyIters * kWave))
        a.slot_words = kPackCopyIters * kWave;  // larger blocks take the direct path
    const int threads = (int)waves * 64;
    uint64_t wgs = (nblocks + waves - 1) / waves;
    const uint32_t lds = 4 * (table_words + waves * a.slot_words);
    const uint64_t cap = (uint64_t)ncu * (lds ? kLdsBytes / lds : 4);
    if (wgs > cap) wgs = cap;
    // Range plan (the histogram's snapshots, hz_hist16_ranges): every pack wave takes whole ranges,
    // so the plan is used when the waves cover the ranges evenly; else count + scan + write.
    // k_pack_write leaves its cold blocks to k_pack_cold (HOT always has slots: mean code <= 17 bits)
    const bool split = t.enc_mode == ENC_HOT || (t.enc_mode == ENC_DENSE && a.slot_words > 0);
    if (split) {
        const void* fc = t.enc_mode == ENC_DENSE ? (const void*)k_pack_cold<ENC_DENSE> : (const void*)k_pack_cold<ENC_HOT>;
        hipError_t e = ensure_lds_limit(fc, kLdsBytes);
        if (e != hipSuccess) return e;
        if ((e = pack_cold_reset(a, s)) != hipSuccess) return e;
    }
    const RangeGeom g = d_ranges ? range_geom(nsym) : RangeGeom{};
    if (g.bytes && t.d_lenpair) {
        uint64_t rw = (g.nranges + waves - 1) / waves;
        if (rw > cap) rw = cap;
        const uint64_t W = rw * waves;
        if (W >= g.nranges || g.nranges % W == 0) {
            const void* fr = pack_write_fn(t.enc_mode, true, split);
            hipError_t e = ensure_lds_limit(fr, kLdsBytes);
            if (e != hipSuccess) return e;
            const RangeArgs r = range_args(d_ranges, g, d_err);
            uint64_t dg = g.nranges < (uint64_t)ncu * 4 ? g.nranges : (uint64_t)ncu * 4;
            hipLaunchKernelGGL(k_range_dot, dim3(dg), dim3(kDotThreads), 0, s, r, (const uint32_t*)t.d_lenpair);
            hipLaunchKernelGGL(k_range_scan, dim3(1), dim3(kScanThreads), 0, s, r, start_bit);
            a.rstart = r.start; a.bpr = g.bpr; a.nranges = g.nranges; a.blk_start = nullptr;
            if ((e = pack_write_launch(fr, rw, threads, lds, s, a)) != hipSuccess) return e;
            if (split) pack_cold_launch(t, a, 4 * table_words, ncu, s);
            if (used_ranges) *used_ranges = 1;
            return hipGetLastError();
        }
    }
    {
        hipError_t e = ensure_lds_limit((const void*)k_pack_count, kLen8LdsBytes);
        if (e != hipSuccess) return e;
        if ((e = ensure_lds_limit(pack_write_fn(t.enc_mode, false, split), kLdsBytes)) != hipSuccess) return e;
    }
    {
        const uint64_t cw = kCountThreads / 64;
        uint64_t cg = (nblocks + cw - 1) / cw;
        if (cg > (uint64_t)ncu * 2) cg = (uint64_t)ncu * 2;  // two 64 KiB-LDS workgroups per CU
        hipLaunchKernelGGL(k_pack_count, dim3(cg), dim3(kCountThreads), kLen8LdsBytes, s, a);
    }
    hipLaunchKernelGGL(k_scan_reduce, dim3(ntiles), dim3(kScanThreads), 0, s, (const unsigned long long*)a.blk,
                       nblocks, tiles, 0xffffffffull);
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kScanThreads), 0, s, tiles, ntiles, start_bit);
    hipLaunchKernelGGL(k_scan_apply, dim3(ntiles), dim3(kScanThreads), 0, s, (const unsigned long long*)a.blk,
                       nblocks, (const unsigned long long*)tiles, blk_start, 0xffffffffull);
    {
        hipError_t e = pack_write_launch(pack_write_fn(t.enc_mode, false, split), wgs, threads, lds, s, a);
        if (e != hipSuccess) return e;
    }
    if (split) pack_cold_launch(t, a, 4 * table_words, ncu, s);
    return hipGetLastError();
}

// ===========================================================================
// Decode (replaces translateFile, Decompressor.cu:259-291).
//
// Block decoder: one wave per 2048-symbol pack block. The block's payload
// bits [start[b], start[b+1]) are staged into the wave's LDS slot with
// coalesced 16-byte loads (byte-swapped once on the way in); then each lane
// decodes its 32 symbols as two independent 16-symbol chains whose start bits
// come from the block index, reading every window straight from LDS. There
// is no per-lane refill state, so a symbol costs a window read, a table
// lookup and an add. Tables (LDS, one copy per workgroup):
//   DENSE: 2^K u16 symbols + 2-bit (len - min_len), K = max_len;
//   LUT:   2^K1 u32 level-1 entries (leaf / link, hz_internal.h),
//          deeper levels in global memory.
// Every code 16 bits (FIXED16): symbol i sits at bit start + 16 i, so that
// decoder needs no index and no staging (k_decode_fixed16).
// ===========================================================================
struct DecArgs {
    const uint32_t* words;   // payload view, 64-byte aligned
    uint64_t nwords;
    uint32_t bit_adj;        // payload bit 0 = bit bit_adj of words
    uint64_t nsym;
    uint64_t nblocks;
    const unsigned long long* starts;  // block index (hz_internal.h)
    const unsigned long long* subs;    // four u16 chain start bits per lane (low 16 bits)
    uint64_t start0;         // FIXED16 without an index: the stream's first bit (starts null)
    const uint32_t* lds_img;
    uint32_t lds_words;      // table words; the staging region follows
    uint32_t region_words;   // staging region per workgroup (slots sized in-kernel from max_bits)
    int k;
    int min_len;
    int max_len;
    int level_bits;          // LUT: widest global subtable (Tables::dec_level_bits)
    const uint32_t* l2;
    uint8_t* out;
    uint32_t* err;
};

// LUT entries (hz_internal.h): a link's subtable index is the next nb window
// bits; pos (bits [4:0]) places them in a 32-bit window, so a pipelined
// decoder extracts them with one v_bfe_u32 and no depth bookkeeping.
HZ_DEV bool lut_leaf(uint32_t e) { return (int32_t)e < 0; }
HZ_DEV bool lut_lds_link(uint32_t e) { return e < (kLutGlobal << 10); }  // false for leaves (bit 31)
HZ_DEV uint32_t lut_nb(uint32_t e) { return (e >> 5) & 15u; }
// index (raw space: < kLutGlobal LDS, else global + kLutGlobal) of window W's entry under link e
HZ_DEV uint32_t lut_next32(uint32_t e, uint32_t W) { return (e >> 10) + __builtin_amdgcn_ubfe(W, e, e >> 5); }
// entry at raw index i
HZ_DEV uint32_t lut_at(const uint32_t* lds, const uint32_t* l2, uint32_t i) {
    return i < kLutGlobal ? lds[i] : l2[i - kLutGlobal];
}
// l2 index of window W's entry under a global link e (one v_add3 after the bfe)
HZ_DEV uint32_t lut_gnext32(uint32_t e, uint32_t W) {
    return (e >> 10) + __builtin_amdgcn_ubfe(W, e, e >> 5) - kLutGlobal;
}

template <int MODE>
HZ_DEV void dec_lookup(const DecArgs& a, const uint32_t* lds, uint64_t win, uint32_t& sym, uint32_t& L) {
    if (MODE == DEC_FIXED16) {
        sym = reinterpret_cast<const uint16_t*>(lds)[(uint32_t)(win >> 48)];
        L = 16;
    } else if (MODE == DEC_DENSE) {
        const uint32_t idx = (uint32_t)(win >> (64 - a.k));
        sym = reinterpret_cast<const uint16_t*>(lds)[idx];
        const uint32_t lw = lds[(1u << a.k) / 2 + (idx >> 4)];
        L = (uint32_t)a.min_len + ((lw >> ((idx & 15) * 2)) & 3u);
    } else {
        uint32_t e = lds[(uint32_t)(win >> (64 - a.k))];
        uint32_t D = (uint32_t)a.k;
        while (!lut_leaf(e)) {  // 64-bit windows: depth tracked here (pos covers 32-bit windows only)
            const uint32_t nb = lut_nb(e);
            e = lut_at(lds, a.l2, (e >> 10) + (uint32_t)((win << D) >> (64 - nb)));
            D += nb;
        }
        L = lut_leaf_len(e);
        sym = lut_leaf_sym(e);
    }
}

HZ_DEV void copy_lds_table(uint32_t* lds, const uint32_t* img, uint32_t words) {
    const uint4* src = reinterpret_cast<const uint4*>(img);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (uint32_t i = threadIdx.x; i < words / 4; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

// MSB-first window at bit `pos` of a staged (byte-swapped) slot: the top 33+
// bits are valid, or all 64 when WIDE (codes longer than 32 bits).
template <bool WIDE>
HZ_DEV uint64_t stage_window(const uint32_t* stg, uint32_t pos) {
    const uint32_t wi = pos >> 5, sh = pos & 31;
    const uint64_t two = (((uint64_t)stg[wi]) << 32) | stg[wi + 1];
    if (!WIDE) return two << sh;
    return (two << sh) | ((((uint64_t)stg[wi + 2]) << sh) >> 32);
}

// 16 staged payload bytes at word w (zeros past the payload; w may have wrapped below 0).
HZ_DEV uint4 dec_stage_load(const DecArgs& a, uint64_t w) {
    uint4 v;
    if (w < a.nwords && w + 4 <= a.nwords) {
        v = *reinterpret_cast<const uint4*>(a.words + w);
    } else {
        v.x = w < a.nwords ? a.words[w] : 0u;
        v.y = w + 1 < a.nwords ? a.words[w + 1] : 0u;
        v.z = w + 2 < a.nwords ? a.words[w + 2] : 0u;
        v.w = 0u;
    }
    return v;
}

// Stage payload words [w0, w0 + 4 npc) of block b into `stg`, byte-swapped.
// The first kStageUnroll 16-byte loads of every lane are issued before any
// is used (one memory round trip for blocks up to 4 KiB of payload).
constexpr int kStageUnroll = 4;
template <bool WIDE>
HZ_DEV void dec_stage(const DecArgs& a, uint64_t b0, uint64_t b1, uint32_t npc_max, uint32_t* stg, int lane,
                      uint64_t& w0) {
    w0 = ((b0 >> 5) & ~3ull) - 4;  // one 16-byte pad before the block: every position is >= 128 (may wrap: zeros)
    const uint64_t wend = (b1 >> 5) + (WIDE ? 3 : 2);
    uint32_t npc = (uint32_t)((wend - w0 + 3) >> 2);
    npc = npc < npc_max ? npc : npc_max;
    uint4 v[kStageUnroll];
#pragma unroll
    for (int u = 0; u < kStageUnroll; ++u) {
        const uint32_t p = (uint32_t)lane + (uint32_t)u * kWave;
        if (p < npc) v[u] = dec_stage_load(a, w0 + 4ull * p);
    }
#pragma unroll
    for (int u = 0; u < kStageUnroll; ++u) {
        const uint32_t p = (uint32_t)lane + (uint32_t)u * kWave;
        if (p < npc)
            reinterpret_cast<uint4*>(stg)[p] = make_uint4(bswap32(v[u].x), bswap32(v[u].y), bswap32(v[u].z), bswap32(v[u].w));
    }
    for (uint32_t p = (uint32_t)lane + kStageUnroll * kWave; p < npc; p += kWave) {
        const uint4 x = dec_stage_load(a, w0 + 4ull * p);
        reinterpret_cast<uint4*>(stg)[p] = make_uint4(bswap32(x.x), bswap32(x.y), bswap32(x.z), bswap32(x.w));
    }
}

// Chain slot c of lane l decodes the block's chain 64 c + l (its symbols 8 (64 c + l) .. + 7), so the
// lane's chain-c symbols are the 16 output bytes at 1024 c + 16 l and each of a block's four output stores
// covers 1 KiB (lane-major chains -- the lane's 32 symbols as 64 contiguous bytes -- left every store
// touching 64 separate 64-byte pieces: 12.3 vs 11.15 ms at 16 GiB Zipf, round 3 A/B). The index keeps
// its layout (sub[b * 64 + l] = chains 4 l .. 4 l + 3), so a lane reads its four chain starts as u16s.
HZ_DEV uint64_t dec_sub_load(const DecArgs& a, uint64_t b, int lane) {
    const uint16_t* s16 = reinterpret_cast<const uint16_t*>(a.subs) + b * kChainsPerBlock + (uint32_t)lane;
    return (uint64_t)s16[0] | ((uint64_t)s16[64] << 16) | ((uint64_t)s16[128] << 32) | ((uint64_t)s16[192] << 48);
}

// Chain start bits relative to the block start (chain 64 c + l in slot c of lane l): sub holds the
// low 16 bits of each chain's stream bit, bs the block's start bit; offsets are mod 2^16, rebuilt from
// deltas when the block is that long.
HZ_DEV void dec_chain_offsets(uint64_t sub, uint64_t bs, uint64_t bits, int lane,
                                   uint32_t (&off)[kChainsPerLane]) {
    constexpr int C = kChainsPerLane;
#pragma unroll
    for (int c = 0; c < C; ++c) off[c] = ((uint32_t)(sub >> (16 * c)) - (uint32_t)bs) & 0xffffu;
    if (bits >= 65536) {  // rebuild from deltas in chain order: (c, l - 1) precedes (c, l), (c - 1, 63) (c, 0)
        uint32_t carry = 0, last = 0;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            uint32_t pv = shfl_up_u32(off[c], 1);
            if (lane == 0) pv = last;
            last = __builtin_amdgcn_readlane(off[c], 63);
            uint32_t sc = (off[c] - pv) & 0xffffu;
#pragma unroll
            for (int dd = 1; dd < 64; dd <<= 1) {
                const uint32_t o = shfl_up_u32(sc, dd);
                if (lane >= dd) sc += o;
            }
            off[c] = carry + sc;
            carry = __builtin_amdgcn_readlane(off[c], 63);
        }
    }
}

HZ_DEV void dec_store(const DecArgs& a, uint64_t b, int lane, const uint32_t* pk) {
    const uint64_t sym0 = b * kBlockSyms;
    if (sym0 + kBlockSyms <= a.nsym) {
        // non-temporal (streaming) stores: the output is not read again by this kernel
        // (10.70 vs 11.15-11.37 ms at 16 GiB Zipf, round 3 A/B; buffer stores with nt / sc0 nt /
        // nt sc1 / sc0 nt sc1 10.13-10.48 vs 10.01-10.02 ms)
        uint4* o = reinterpret_cast<uint4*>(a.out + 2 * sym0) + lane;
#pragma unroll
        for (int c = 0; c < kChainsPerLane; ++c)
            store_nt16(o + c * kWave, make_uint4(pk[4 * c], pk[4 * c + 1], pk[4 * c + 2], pk[4 * c + 3]));
    } else {
#pragma unroll
        for (int c = 0; c < kChainsPerLane; ++c) {
            const uint64_t s0 = sym0 + (uint64_t)kChainSyms * (uint32_t)(c * kWave + lane);
            if (s0 >= a.nsym) continue;
            uint8_t* ob = a.out + 2 * s0;
            const uint32_t cnt = a.nsym - s0 < (uint64_t)kChainSyms ? (uint32_t)(a.nsym - s0) : kChainSyms;
            for (uint32_t q = 0; q < cnt; ++q) {
                const uint32_t v = (pk[4 * c + (q >> 1)] >> (16 * (q & 1))) & 0xffffu;
                ob[2 * q] = (uint8_t)v;
                ob[2 * q + 1] = (uint8_t)(v >> 8);
            }
        }
    }
}

// One wave decodes NB blocks at once (NB * kChainsPerLane independent chains
// per lane: every table wait covers more symbols). Block g of the group uses
// staging slot g. Blocks past the stream's end decode nothing.
template <int MODE, bool WIDE, int NB>
HZ_DEV void dec_group(const DecArgs& a, const uint32_t* lds, uint32_t* stg0, uint32_t slot, uint64_t bfirst,
                      int lane) {
    constexpr int C1 = kChainsPerLane;
    constexpr int C = NB * C1;
    const uint32_t npc_max = slot >> 2;
    uint32_t pos[C];
#pragma unroll
    for (int g = 0; g < NB; ++g) {
        const uint64_t b = bfirst + g < a.nblocks ? bfirst + g : a.nblocks - 1;  // duplicates decode, never store
        const uint64_t b0 = a.starts[b] + a.bit_adj, b1 = a.starts[b + 1] + a.bit_adj;
        const uint64_t sub = dec_sub_load(a, b, lane);
        uint64_t w0;
        dec_stage<WIDE>(a, b0, b1, npc_max, stg0 + g * slot, lane, w0);
        uint32_t off[C1];
        dec_chain_offsets(sub, b0 - a.bit_adj, b1 - b0, lane, off);
        const uint32_t base = (uint32_t)(b0 - (w0 << 5)) + (uint32_t)g * slot * 32u;
#pragma unroll
        for (int c = 0; c < C1; ++c) pos[g * C1 + c] = base + off[c];
    }
    __builtin_amdgcn_wave_barrier();  // LDS ops of one wave complete in order
    uint32_t pk[NB][kSPT / 2];
    // Windows: 32 bits (bit 31 = the chain's next bit) for codes <= 32 bits,
    // one funnel shift of two staged words; 64 bits for WIDE.
    using Win = typename std::conditional<WIDE, uint64_t, uint32_t>::type;
    constexpr uint32_t WB = WIDE ? 64 : 32;
#pragma unroll
    for (int q = 0; q < kChainSyms; ++q) {
        Win win[C];
        uint32_t sym[C], L[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            if constexpr (WIDE) {
                win[c] = stage_window<true>(stg0, pos[c]);
            } else {
                const uint32_t p1 = pos[c] - 1u;  // >= 127 (staging pad)
                const uint32_t* w = stg0 + (p1 >> 5);
                win[c] = __builtin_amdgcn_alignbit(w[0], w[1], 31u - p1);
            }
        }
        if (MODE == DEC_DENSE) {
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const uint32_t idx = (uint32_t)(win[c] >> (WB - (uint32_t)a.k));
                sym[c] = reinterpret_cast<const uint16_t*>(lds)[idx];
                const uint32_t lw = lds[(1u << a.k) / 2 + (idx >> 4)];
                L[c] = (uint32_t)a.min_len + ((lw >> ((idx & 15) * 2)) & 3u);
            }
        } else {
            uint32_t e[C], e2[C], D[C];
#pragma unroll
            for (int c = 0; c < C; ++c) { e[c] = lds[(uint32_t)(win[c] >> (WB - (uint32_t)a.k))]; D[c] = (uint32_t)a.k; }
#pragma unroll
            for (int c = 0; c < C; ++c) {  // LDS-resident second level (hot subtables)
                if (lut_lds_link(e[c])) {
                    const uint32_t nb = lut_nb(e[c]);
                    e[c] = lds[(e[c] >> 10) + (uint32_t)((Win)(win[c] << D[c]) >> (WB - nb))];
                    D[c] += nb;
                }
            }
#pragma unroll
            for (int c = 0; c < C; ++c) {  // first global level of every chain before one wait
                e2[c] = e[c];
                if (!lut_leaf(e[c])) {
                    const uint32_t nb = lut_nb(e[c]);
                    e2[c] = a.l2[(e[c] >> 10) - kLutGlobal + (uint32_t)((Win)(win[c] << D[c]) >> (WB - nb))];
                }
            }
#pragma unroll
            for (int c = 0; c < C; ++c) {
                uint32_t ee = e2[c];
                if (!lut_leaf(e[c])) {
                    uint32_t Dd = D[c] + lut_nb(e[c]);
                    while (!lut_leaf(ee)) {  // deeper global levels: rare
                        const uint32_t nb = lut_nb(ee);
                        ee = a.l2[(ee >> 10) - kLutGlobal + (uint32_t)((Win)(win[c] << Dd) >> (WB - nb))];
                        Dd += nb;
                    }
                }
                L[c] = lut_leaf_len(ee);
                sym[c] = lut_leaf_sym(ee);
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
            pos[c] += L[c];
            const int g = c / C1;
            const int i = ((c % C1) * kChainSyms + q) >> 1;  // symbol (c%C1)*8+q of the lane in block g
            if (q & 1) pk[g][i] |= sym[c] << 16;
            else pk[g][i] = sym[c];
        }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int g = 0; g < NB; ++g)
        if (bfirst + g < a.nblocks) dec_store(a, bfirst + g, lane, pk[g]);
}

// Two-level LUT decode of one block with the global lookups software
// pipelined. Needs max_len <= k + level bits (every global lookup ends in
// a leaf) and max_len <= 32. The lane's chains are two halves, {0,1} and
// {2,3}; a half's LDS step (window, level 1, LDS second level) issues its
// global lookups unconditionally (lanes that do not need one read l2[0]:
// same-address lanes coalesce), and those are consumed only after the other
// half's LDS step has issued its own, so every wait is vmcnt(2) in
// straight-line code and one half's table walk hides the other's gather.
struct PipeLane {
    uint32_t e, gi;
};

// One chain's LDS step: window, level 1, the LDS second level (hot heads).
// r.gi: the l2 index of the global entry to read (0 -- one coalesced address
// -- when the chain is resolved in LDS).
HZ_DEV PipeLane dec_pipe_lds(const DecArgs& a, const uint32_t* lds, const uint32_t* stg, uint32_t pos) {
    const uint32_t p1 = pos - 1u;  // >= 127 (staging pad)
    const uint32_t* w = stg + (p1 >> 5);
    const uint32_t W = __builtin_amdgcn_alignbit(w[0], w[1], 31u - p1);
    uint32_t e = lds[W >> (32 - a.k)];
    if (lut_lds_link(e)) e = lds[lut_next32(e, W)];
    PipeLane r;
    r.e = e;
    r.gi = lut_leaf(e) ? 0u : lut_gnext32(e, W);
    return r;
}

// The LDS steps of two chains at once, branch-free so the compiler keeps one
// basic block: both window reads, then both level-1 reads, then both
// LDS-second-level reads are in flight together (three LDS round trips for the
// pair instead of three per chain). Lanes without an LDS second level read
// word 0 (a broadcast, no bank conflict) and keep their level-1 entry.
HZ_DEV void dec_pipe_lds2(const DecArgs& a, const uint32_t* lds, const uint32_t* stg, uint32_t pos0, uint32_t pos1,
                          PipeLane& r0, PipeLane& r1) {
    const uint32_t k = (uint32_t)a.k;
    const uint32_t pa = pos0 - 1u, pb = pos1 - 1u;  // >= 127 (staging pad)
    const uint32_t* wa = stg + (pa >> 5);
    const uint32_t* wb = stg + (pb >> 5);
    const uint32_t a0 = wa[0], a1 = wa[1], b0 = wb[0], b1 = wb[1];
    const uint32_t Wa = __builtin_amdgcn_alignbit(a0, a1, 31u - pa);
    const uint32_t Wb = __builtin_amdgcn_alignbit(b0, b1, 31u - pb);
    uint32_t ea = lds[Wa >> (32 - k)];
    uint32_t eb = lds[Wb >> (32 - k)];
    const bool ha = lut_lds_link(ea), hb = lut_lds_link(eb);
    const uint32_t xa = lds[ha ? lut_next32(ea, Wa) : 0u], xb = lds[hb ? lut_next32(eb, Wb) : 0u];
    ea = ha ? xa : ea;
    eb = hb ? xb : eb;
    r0.e = ea;
    r1.e = eb;
    r0.gi = lut_leaf(ea) ? 0u : lut_gnext32(ea, Wa);
    r1.gi = lut_leaf(eb) ? 0u : lut_gnext32(eb, Wb);
}

// The LDS steps of NC chains at once (dec_pipe_lds2 generalised): all window
// reads, then all level-1 reads, then all LDS-second-level reads in flight
// together, so NC chain steps cost three LDS round trips.
// Phase fences of the NC-chain walk: keep each phase's LDS reads issued
// together whatever the scheduler would do (the decoder is order-sensitive).
#define HZ_WALK_FENCE() __builtin_amdgcn_sched_barrier(0)


// Global table l2 as a buffer whose byte 0 lies kLutGlobal words before l2[0]:
// the byte offset of a global link's entry is (raw + index bits) * 4, one
// v_add_lshl_u32; num_records covers the largest table (kLutMaxL2 entries).
// Lanes resolved in LDS read past num_records (0, no memory access) instead of l2[0]:
// 12.27-12.29 vs 12.33-12.37 ms at 16 GiB Zipf (round 3, A/B in one run). A leaf's offset
// computed as a link's is >= 4 * 2^21 and < 2^27 (hz_internal.h lut_leaf_entry): no wrap.
static_assert(kLutGlobal + kLutMaxL2 == (1u << 21), "a leaf (bit 31) read as a link lands past num_records");
HZ_DEV __amdgpu_buffer_rsrc_t lut_l2_rsrc(const uint32_t* l2) {
    return __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(reinterpret_cast<uintptr_t>(l2) - 4ull * kLutGlobal), 0,
        4u * (kLutGlobal + kLutMaxL2), 0x00020000);
}

// The LDS steps of NC chains at once: all window reads, then all level-1
// reads, then all LDS-second-level reads in flight together, so NC chain
// steps cost three LDS round trips. p1[c] = the LDS bit address of chain c's
// next bit, minus 1 (>= 127 bits into its staging slot); k_decode has no
// static LDS, so the table and slots are addressed from LDS byte 0. r[c].e: the entry
// after LDS; r[c].gi: byte offset of its global entry in lut_l2_rsrc.
template <int NC>
HZ_DEV void dec_pipe_ldsn(const DecArgs& a, const uint32_t* lds, const uint32_t* p1, PipeLane* r, uint32_t adj = 0) {
    const uint32_t k = (uint32_t)a.k;
    uint32_t W[NC], e[NC], x[NC];
    bool h[NC];
    // descending slot (dec_stage_commit<true>): p1 holds m, stream word t + 1 at byte (m >> 3) & ~3,
    // word t just above it, and m & 31 is the funnel shift (no v_not per step); adj: bytes the
    // window lies above (p1 short by 128 bits per step taken, a multiple of 32: the shift holds).
    // All window reads issue before the first shift: without the fence the chain decoder's register
    // allocation reused one pair for all four (four serial LDS round trips per step; extract
    // 21.14-21.23 -> 20.91-21.01 ms, A/B).
    uint32_t whi[NC], wlo[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const uint32_t wb = ((p1[c] >> 3) & ~3u) + adj;
        whi[c] = lds_at(wb + 4);
        wlo[c] = lds_at(wb);
    }
    HZ_WALK_FENCE();
#pragma unroll
    for (int c = 0; c < NC; ++c) W[c] = __builtin_amdgcn_alignbit(whi[c], wlo[c], p1[c]);
    HZ_WALK_FENCE();
#pragma unroll
    for (int c = 0; c < NC; ++c) e[c] = lds_at((W[c] >> (32 - k)) << 2);
    HZ_WALK_FENCE();
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        h[c] = lut_lds_link(e[c]);
        const uint32_t byte = ((e[c] >> 10) + __builtin_amdgcn_ubfe(W[c], e[c], e[c] >> 5)) << 2;
        // a leaf's or a global link's byte address is >= 256 KiB, past the workgroup's LDS: that
        // read returns nothing anyone uses (the select below keeps e), so no address select
        x[c] = lds_at(byte);
    }
    HZ_WALK_FENCE();
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const uint32_t ee = h[c] ? x[c] : e[c];
        const uint32_t byte = ((ee >> 10) + __builtin_amdgcn_ubfe(W[c], ee, ee >> 5)) << 2;
        r[c].e = ee;
        // a leaf's byte offset lies in [4 * 2^21, 2^27): past num_records of lut_l2_rsrc, so the
        // load returns 0 without a memory access, with no select (lut_leaf_entry)
        r[c].gi = byte;
    }
}

// Block metadata of the pipelined decoder: start and end bit, the lane's chain offsets.
struct PipeMeta {
    uint64_t b0, b1, sub;
};

HZ_DEV void dec_meta_load(const DecArgs& a, uint64_t b, int lane, PipeMeta& m) {
    const uint64_t bb = b < a.nblocks ? b : a.nblocks - 1;  // past the end: any block, never used
    // the block's bounds through the scalar cache (the index is read-only here): the window
    // arithmetic that follows stays on the scalar unit
    typedef const __attribute__((address_space(4))) unsigned long long* cu64p;
    const uint64_t bu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(bb >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)bb);
    m.b0 = ((cu64p)a.starts)[bu];
    m.b1 = ((cu64p)a.starts)[bu + 1];
    m.sub = dec_sub_load(a, bb, lane);
}

// The first kStageUnroll 16-byte chunks of a block's staging window, always
// exactly kStageUnroll loads per lane (static vmcnt for the pipelined waits):
// chunks past the window or the payload read a clamped address and are fixed
// up in registers. Requires nwords >= 4 (host check).
HZ_DEV void dec_stage_prefetch(const DecArgs& a, const PipeMeta& m, int lane, uint4 (&v)[kStageUnroll]) {
    const uint64_t w0 = (((m.b0 + a.bit_adj) >> 5) & ~3ull) - 4;
#pragma unroll
    for (int u = 0; u < kStageUnroll; ++u) {
        const uint64_t w = w0 + 4ull * ((uint32_t)lane + (uint32_t)u * kWave);
        const bool in = w < a.nwords;  // also false for a window that wrapped below word 0
        const uint64_t wl = !in ? 0 : (w + 4 <= a.nwords ? w : a.nwords - 4);
        v[u] = *reinterpret_cast<const uint4*>(a.words + wl);
    }
}

HZ_DEV uint32_t pick4(const uint4& v, uint32_t i) {
    return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

// Writes the prefetched chunks (fixed up for the payload's end) and any
// further chunks of an oversized window into the slot.
// DESC: the slot holds the words in descending order (stream word t at slot word 4 npc_max - 1 - t).
template <bool DESC = false>
HZ_DEV void dec_stage_commit(const DecArgs& a, const PipeMeta& m, uint32_t npc_max, uint32_t* stg, int lane,
                             const uint4 (&v)[kStageUnroll], uint64_t& w0) {
    const uint64_t b0 = m.b0 + a.bit_adj, b1 = m.b1 + a.bit_adj;
    w0 = ((b0 >> 5) & ~3ull) - 4;
    const uint64_t wend = (b1 >> 5) + 2;
    uint32_t npc = (uint32_t)((wend - w0 + 3) >> 2);
    npc = npc < npc_max ? npc : npc_max;
#pragma unroll
    for (int u = 0; u < kStageUnroll; ++u) {
        const uint32_t p = (uint32_t)lane + (uint32_t)u * kWave;
        if (p < npc) {
            const uint64_t w = w0 + 4ull * p;
            uint4 x = v[u];
            if (!(w < a.nwords && w + 4 <= a.nwords)) {  // tail of the payload (or wrapped): shift, zero-fill
                const uint64_t base = a.nwords - 4;
                uint32_t q[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const uint64_t wt = w + t;
                    q[t] = wt < a.nwords && w < a.nwords ? pick4(x, (uint32_t)(wt - base)) : 0u;
                }
                x = make_uint4(q[0], q[1], q[2], q[3]);
            }
            if (DESC)
                reinterpret_cast<uint4*>(stg)[npc_max - 1 - p] = make_uint4(bswap32(x.w), bswap32(x.z), bswap32(x.y), bswap32(x.x));
            else
                reinterpret_cast<uint4*>(stg)[p] = make_uint4(bswap32(x.x), bswap32(x.y), bswap32(x.z), bswap32(x.w));
        }
    }
    for (uint32_t p = (uint32_t)lane + kStageUnroll * kWave; p < npc; p += kWave) {  // oversized block: rare
        const uint4 x = dec_stage_load(a, w0 + 4ull * p);
        if (DESC)
            reinterpret_cast<uint4*>(stg)[npc_max - 1 - p] = make_uint4(bswap32(x.w), bswap32(x.z), bswap32(x.y), bswap32(x.x));
        else
            reinterpret_cast<uint4*>(stg)[p] = make_uint4(bswap32(x.x), bswap32(x.y), bswap32(x.z), bswap32(x.w));
    }
}

constexpr int kPfStep = 4;  // chain step at which the next block's staging loads issue (2-6 measured equal)
// Persistent pipelined decoder of one wave: blocks b, b + stride, ... The
// staging chunks of the next block and the metadata of the one after are
// loaded halfway through this block's steps, so no block waits on HBM.
HZ_DEV void dec_wave_pipe(const DecArgs& a, const uint32_t* lds, uint32_t* stg, uint32_t slot, uint64_t b,
                          uint64_t stride, int lane) {
    const uint32_t* l2g = a.l2;
    constexpr int C = kChainsPerLane;
    static_assert(C == 4, "two halves of two chains");
    PipeMeta mc, mn, mn2;
    uint4 sc[kStageUnroll], sn[kStageUnroll];
    dec_meta_load(a, b, lane, mc);
    dec_meta_load(a, b + stride, lane, mn);
    dec_stage_prefetch(a, mc, lane, sc);
    for (; b < a.nblocks; b += stride) {
        uint64_t w0;
        dec_stage_commit(a, mc, slot >> 2, stg, lane, sc, w0);
        uint32_t off[C];
        dec_chain_offsets(mc.sub, mc.b0, mc.b1 - mc.b0, lane, off);
        const uint32_t base = (uint32_t)(mc.b0 + a.bit_adj - (w0 << 5));
        uint32_t pos[C];
#pragma unroll
        for (int c = 0; c < C; ++c) pos[c] = base + off[c];
        __builtin_amdgcn_wave_barrier();  // LDS ops of one wave complete in order
        uint32_t pk[kSPT / 2];
        PipeLane st[C];
        uint32_t g[C];
        auto finish = [&](int c, int q) {
            const uint32_t ee = (st[c].e >> 31) ? st[c].e : g[c];
            pos[c] += lut_leaf_len(ee);
            const uint32_t sym = lut_leaf_sym(ee);
            const int i = (c * kChainSyms + q) >> 1;
            if (q & 1) pk[i] |= sym << 16;
            else pk[i] = sym;
        };
        auto issue2 = [&](int c) {
            dec_pipe_lds2(a, lds, stg, pos[c], pos[c + 1], st[c], st[c + 1]);
            g[c] = l2g[st[c].gi];
            g[c + 1] = l2g[st[c + 1].gi];
        };
        issue2(0);
#pragma unroll
        for (int q = 0; q < kChainSyms; ++q) {
            issue2(2);
            if (q == kPfStep) {  // next block's staging chunks, the metadata after it
                dec_stage_prefetch(a, mn, lane, sn);
                dec_meta_load(a, b + 2 * stride, lane, mn2);
            }
            finish(0, q);
            finish(1, q);
            if (q + 1 < kChainSyms) issue2(0);
            finish(2, q);
            finish(3, q);
        }
        __builtin_amdgcn_wave_barrier();
        dec_store(a, b, lane, pk);
        mc = mn;
        mn = mn2;
#pragma unroll
        for (int u = 0; u < kStageUnroll; ++u) sc[u] = sn[u];
    }
}

// Two blocks per wave (8 chains per lane in 4 pairs): each pair's global
// lookups are consumed after the other three pairs' LDS walks, so a gather
// has three walks to land in instead of one. Half as many waves (two staging
// slots each) hold the same LDS; blocks b, b + 1, then b + stride, ...
HZ_DEV void dec_wave_pipe2(const DecArgs& a, const uint32_t* lds, uint32_t* stg, uint32_t slot, uint64_t b,
                           uint64_t stride, int lane) {
    constexpr int C = 2 * kChainsPerLane;
    static_assert(kChainsPerLane == 4, "four pairs of chains over two blocks");
    const __amdgpu_buffer_rsrc_t l2r = lut_l2_rsrc(a.l2);
    [[maybe_unused]] const uint32_t stg_bit = (uint32_t)(stg - lds) * 32u - 1u;  // LDS bit address of the slots, minus 1
    PipeMeta mc[2], mn[2], mn2[2];
    uint4 sc[2][kStageUnroll], sn[2][kStageUnroll];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        dec_meta_load(a, b + j, lane, mc[j]);
        dec_meta_load(a, b + stride + j, lane, mn[j]);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) dec_stage_prefetch(a, mc[j], lane, sc[j]);
    for (; b < a.nblocks; b += stride) {
        uint32_t p1[C];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            uint64_t w0;
            dec_stage_commit<true>(a, mc[j], slot >> 2, stg + j * slot, lane, sc[j], w0);
            uint32_t off[kChainsPerLane];
            dec_chain_offsets(mc[j].sub, mc[j].b0, mc[j].b1 - mc[j].b0, lane, off);
            // m = (E - 1) * 32 + 31 - r for the slot's top word E and r = the chain's next bit - 1,
            // relative to stream word w0; a step of L bits subtracts L
            const uint32_t top = (uint32_t)(stg - lds) + (uint32_t)(j + 1) * slot - 1u;
            const uint32_t base = top * 32u - (uint32_t)(mc[j].b0 + a.bit_adj - (w0 << 5));
#pragma unroll
            for (int c = 0; c < kChainsPerLane; ++c) p1[j * kChainsPerLane + c] = base - off[c];
        }
        __builtin_amdgcn_wave_barrier();  // LDS ops of one wave complete in order
        uint32_t pk[2][kSPT / 2];
        PipeLane st[C];
        uint32_t g[C];
        auto finish = [&](int c, int q) {
            // a leaf in LDS (bit 31) beats its gather's 0 (read past num_records); a link loses to its
            // gathered leaf: one v_max; and the leaf's byte 3 is 0x80 | L, subtracted whole (128 bits
            // more per step, which the window address takes back: dec_pipe_ldsn's adj). 12 % fewer VALU
            // per block pair; k_decode 10.09 -> 9.97 ms, chain decode 11.30 -> 11.13 ms (A/B, 16 GiB Zipf)
            const uint32_t ee = st[c].e > g[c] ? st[c].e : g[c];
            p1[c] -= ee >> 24;
            const int i = ((c % kChainsPerLane) * kChainSyms + q) >> 1;
            // an even step keeps the whole entry; the odd step packs both symbols (leaf bytes 1-2) by one v_perm
            if (q & 1) pk[c / kChainsPerLane][i] = __builtin_amdgcn_perm(ee, pk[c / kChainsPerLane][i], 0x06050201u);
            else pk[c / kChainsPerLane][i] = ee;
        };
        // two quads (one per block): a quad's gathers land behind the other quad's walk
        auto issue4 = [&](int c, int q) {
            // issue priority over the quad's LDS walk and gathers (decode 9.96-9.99 -> 9.88-9.91 ms, A/B)
            __builtin_amdgcn_s_setprio(2);
            dec_pipe_ldsn<4>(a, lds, p1 + c, st + c, 16u * (uint32_t)q);  // q steps taken: 16 q bytes
#pragma unroll
            for (int t = 0; t < 4; ++t)
                g[c + t] = __builtin_amdgcn_raw_buffer_load_b32(l2r, st[c + t].gi, 0, 0);
            __builtin_amdgcn_s_setprio(0);
        };
        issue4(0, 0);
#pragma unroll
        for (int q = 0; q < kChainSyms; ++q) {
            issue4(4, q);
            if (q == kPfStep) {  // the next two blocks' staging chunks, the metadata after them
#pragma unroll
                for (int j = 0; j < 2; ++j) dec_stage_prefetch(a, mn[j], lane, sn[j]);
#pragma unroll
                for (int j = 0; j < 2; ++j) dec_meta_load(a, b + 2 * stride + j, lane, mn2[j]);
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) finish(c, q);
            if (q + 1 < kChainSyms) issue4(0, q + 1);
#pragma unroll
            for (int c = 4; c < 8; ++c) finish(c, q);
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < 2; ++j)
            if (b + j < a.nblocks) dec_store(a, b + j, lane, pk[j]);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            mc[j] = mn[j];
            mn[j] = mn2[j];
#pragma unroll
            for (int u = 0; u < kStageUnroll; ++u) sc[j][u] = sn[j][u];
        }
    }
}

constexpr int kDecPipe2Threads = 512;  // two staging slots per wave (1024 with smaller hot heads: 15.2 ms vs 13.1)
// PIPE: 0 plain block loop, 1 pipelined (one block per wave), 2 pipelined, two blocks per wave
template <int MODE, bool WIDE, int PIPE>
__global__ __launch_bounds__(PIPE == 2 ? kDecPipe2Threads : 1024) void k_decode(DecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    copy_lds_table(lds, a.lds_img, a.lds_words);
    const int lane = threadIdx.x & 63;
    const uint32_t wid = wave_id();
    // slots fit the stream's largest block; waves without a slot have nothing to do
    const uint32_t slot = (uint32_t)__builtin_amdgcn_readfirstlane((int)dec_slot_words(a.starts[a.nblocks + 1], a.max_len));
    const uint32_t nwave = blockDim.x >> 6;
    if constexpr (PIPE == 2) {
        uint32_t nw2 = a.region_words / (2 * slot);
        nw2 = nw2 < nwave ? nw2 : nwave;
        if (nw2 > 0) {  // else one block per wave below (a stream whose largest block needs more)
            if (wid >= nw2) return;
            const uint64_t b = 2 * ((uint64_t)blockIdx.x * nw2 + wid), stride = 2 * (uint64_t)gridDim.x * nw2;
            dec_wave_pipe2(a, lds, lds + a.lds_words + wid * 2 * slot, slot, b, stride, lane);
            return;
        }
    }
    uint32_t nw = a.region_words / slot;
    nw = nw < nwave ? nw : nwave;
    if (wid >= nw) return;
    uint32_t* stg = lds + a.lds_words + wid * slot;
    const uint64_t b = (uint64_t)blockIdx.x * nw + wid, stride = (uint64_t)gridDim.x * nw;
    if constexpr (PIPE != 0) {
        dec_wave_pipe(a, lds, stg, slot, b, stride, lane);
    } else {
        for (uint64_t bb = b; bb < a.nblocks; bb += stride) dec_group<MODE, WIDE, 1>(a, lds, stg, slot, bb, lane);
    }
}

// Every code 16 bits: lane j decodes symbols [32 j, 32 j + 32) from the 17
// words starting at stream word (p0 >> 5) + 16 j.
// Full blocks [0, nb) of a FIXED16 stream (k_pack_fixed16_blk's mapping): lane l's sub-run c decodes the block's symbols 8 (64 c + l) .. + 7 from 4 words at a
// 1 KiB-coalesced offset plus the next sub-run's first word (lane l + 1 by DPP, sub-run c + 1's lane 0,
// or the next block's first word), and stores 16 bytes at a 1 KiB-coalesced offset.
__global__ __launch_bounds__(1024) void k_decode_fixed16_blk(DecArgs a, uint64_t nb) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    copy_lds_table(lds, a.lds_img, a.lds_words);
    const uint16_t* t16 = reinterpret_cast<const uint16_t*>(lds);
    const uint64_t p0 = (a.starts ? a.starts[0] : a.start0) + a.bit_adj;
    const uint32_t sh = (uint32_t)(p0 & 31);
    const uint32_t* w = a.words + (p0 >> 5);  // any word of the payload view
    const u32x4a4* w4 = reinterpret_cast<const u32x4a4*>(w);
    uint4* o4 = reinterpret_cast<uint4*>(a.out);
    const int lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * (blockDim.x >> 6);
    uint64_t b = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    constexpr uint32_t kBW = kBlockSyms / 2;  // words per block
    auto load = [&](uint64_t bb, u32x4a4 (&x)[kChainsPerLane], uint32_t& nw) {
        bb = bb < nb ? bb : 0;
#pragma unroll
        for (int c = 0; c < kChainsPerLane; ++c) x[c] = w4[bb * (kBW / 4) + c * kWave + lane];
        nw = w[(bb + 1) * kBW];  // the next block's first word (the stream's last block follows block nb - 1)
    };
    u32x4a4 nx[kChainsPerLane];
    uint32_t nn = 0;
    if (b < nb) load(b, nx, nn);
    for (; b < nb; b += W) {
        u32x4a4 x[kChainsPerLane];
#pragma unroll
        for (int c = 0; c < kChainsPerLane; ++c) x[c] = nx[c];
        const uint32_t after = nn;
        load(b + W, nx, nn);
#pragma unroll
        for (int c = 0; c < kChainsPerLane; ++c) {
            uint32_t nxt = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x[c].x, kDppWaveShl1, 0xf, 0xf, false);
            const uint32_t first_next = c + 1 < kChainsPerLane ? readlane(x[c + 1 < kChainsPerLane ? c + 1 : c].x, 0) : after;
            if (lane == 63) nxt = first_next;
            const uint32_t ww[5] = {bswap32(x[c].x), bswap32(x[c].y), bswap32(x[c].z), bswap32(x[c].w), bswap32(nxt)};
            uint32_t o[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const uint32_t cw = sh ? __builtin_amdgcn_alignbit(ww[t], ww[t + 1], 32u - sh) : ww[t];
                o[t] = (uint32_t)t16[cw >> 16] | ((uint32_t)t16[cw & 0xffffu] << 16);
            }
            store_nt16(o4 + b * (kBlockSyms / 8) + c * kWave + lane, make_uint4(o[0], o[1], o[2], o[3]));
        }
    }
}

// Lane runs of 32 symbols: those after the nb blocks k_decode_fixed16_blk decodes, or all of them.
__global__ __launch_bounds__(1024) void k_decode_fixed16(DecArgs a, uint64_t nb) {
    const uint64_t j_begin = nb * kWave;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    copy_lds_table(lds, a.lds_img, a.lds_words);
    const uint64_t p0 = (a.starts ? a.starts[0] : a.start0) + a.bit_adj;  // the stream's first bit (all FIXED16 needs)
    const uint16_t* t16 = reinterpret_cast<const uint16_t*>(lds);
    const uint32_t sh = (uint32_t)(p0 & 31);
    const uint64_t W0 = p0 >> 5;
    const bool vec = (W0 & 3) == 0;
    const uint64_t nl = (a.nsym + kSPT - 1) / kSPT;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = j_begin + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nl; j += stride) {
        const uint64_t ws = W0 + 16 * j;
        uint32_t w[17];
        if (vec && ws + 17 <= a.nwords) {
            const uint4* p = reinterpret_cast<const uint4*>(a.words + ws);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint4 v = p[q];
                w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
            }
            w[16] = a.words[ws + 16];
        } else {
#pragma unroll
            for (int k = 0; k < 17; ++k) w[k] = ws + k < a.nwords ? a.words[ws + k] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 17; ++k) w[k] = bswap32(w[k]);
        uint32_t o[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const uint32_t c = (uint32_t)(((((uint64_t)w[t]) << 32 | w[t + 1]) << sh) >> 32);
            o[t] = (uint32_t)t16[c >> 16] | ((uint32_t)t16[c & 0xffffu] << 16);
        }
        const uint64_t sym0 = j * kSPT;
        if (sym0 + kSPT <= a.nsym) {
            uint4* d = reinterpret_cast<uint4*>(a.out + 2 * sym0);
#pragma unroll
            for (int q = 0; q < 4; ++q) d[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
        } else {
            uint8_t* ob = a.out + 2 * sym0;
            const uint32_t cnt = (uint32_t)(a.nsym - sym0);
            for (uint32_t q = 0; q < cnt; ++q) {
                const uint32_t v = (o[q >> 1] >> (16 * (q & 1))) & 0xffffu;
                ob[2 * q] = (uint8_t)v;
                ob[2 * q + 1] = (uint8_t)(v >> 8);
            }
        }
    }
}

static void fill_dec_args(DecArgs& a, const Tables& t, const uint8_t* d_payload, uint64_t payload_bytes,
                          uint64_t nsym) {
    // View the payload from the 64-byte boundary at or below it (inside the
    // same allocation: device allocations are 256-byte aligned). The last word
    // may extend up to 3 bytes past payload_bytes (include/huffman_amd.h).
    const uintptr_t base = (uintptr_t)d_payload & ~(uintptr_t)63;
    a.words = reinterpret_cast<const uint32_t*>(base);
    a.bit_adj = (uint32_t)(((uintptr_t)d_payload & 63) * 8);
    a.nwords = (payload_bytes + ((uintptr_t)d_payload & 63) + 3) / 4;
    a.nsym = nsym;
    a.nblocks = index_blocks(nsym);
    a.lds_img = t.d_dec_lds;
    a.lds_words = t.dec_lds_bytes / 4;
    a.k = t.dec_k;
    a.level_bits = t.dec_level_bits;
    a.min_len = t.dec_min_len;
    a.max_len = t.dec_max_len;
    a.l2 = t.d_dec_l2;
}

// Launch shape: slots are sized for the average block (estimated from the
// payload size) with headroom; the kernel sizes the real slots from the
// index's max_bits and idles the waves that do not get one. Up to two
// workgroups per CU (each holds its own table copy): whichever shape runs
// more waves.
template <int MODE, bool WIDE, int PIPE>
static hipError_t run_decode(const DecArgs& a, uint64_t payload_bits, int ncu, hipStream_t s) {
    {
        hipError_t e = ensure_lds_limit((const void*)k_decode<MODE, WIDE, PIPE>, kLdsBytes);
        if (e != hipSuccess) return e;
    }
    // a block never exceeds 2048 x max_len bits, whatever follows the stream in the buffer
    uint64_t avg = (payload_bits + a.nblocks - 1) / a.nblocks;
    avg = avg < (uint64_t)kBlockSyms * (uint32_t)a.max_len ? avg : (uint64_t)kBlockSyms * (uint32_t)a.max_len;
    const uint32_t worst = dec_slot_words_max(a.max_len);
    uint32_t est = dec_slot_words(avg + avg / 16 + 256, a.max_len);
    est = est < worst ? est : worst;
    const uint32_t table = a.lds_words;
    if (MODE == DEC_LUT && PIPE == 2 && table < kDecMinLdsWords) return hipErrorInvalidValue;  // biased windows
    int best_w = 0, best_g = 1;
    for (int g = 1; g <= 2; ++g) {
        const uint32_t room = kLdsBytes / 4 / (uint32_t)g;
        if (room <= table + est) continue;
        int w = (int)((room - table) / est);
        const int maxw = PIPE == 2 ? 2 * kDecPipe2Threads / 64 : kDecMaxWaves;  // slots
        w = w > maxw ? maxw : w;
        if (g * w > best_g * best_w) { best_w = w; best_g = g; }
    }
    if (best_w == 0) return hipErrorInvalidValue;
    DecArgs b = a;
    b.region_words = (uint32_t)best_w * est;
    if (b.region_words < worst && table + worst <= kLdsBytes / 4) b.region_words = worst;  // any stream decodes
    if (table + b.region_words > kLdsBytes / 4 / (uint32_t)best_g) best_g = 1;
    if (table + b.region_words > kLdsBytes / 4) return hipErrorInvalidValue;
    const uint32_t lds = 4 * (table + b.region_words);
    uint64_t wgs = (a.nblocks + best_w - 1) / best_w;
    const uint64_t cap = (uint64_t)ncu * best_g;
    if (wgs > cap) wgs = cap;
    // PIPE 2: a wave takes two slots
    const int threads = PIPE == 2 ? (64 * ((best_w + 1) / 2) < kDecPipe2Threads ? 64 * ((best_w + 1) / 2)
                                                                                 : kDecPipe2Threads)
                                  : 64 * best_w;
    hipLaunchKernelGGL((k_decode<MODE, WIDE, PIPE>), dim3(wgs), dim3(threads), lds, s, b);
    return hipGetLastError();
}

hipError_t launch_decode(const Tables& t, const uint8_t* d_payload, uint64_t payload_bytes, uint64_t nsym,
                         const unsigned long long* d_index, uint8_t* d_out, uint32_t* d_err, int ncu,
                         hipStream_t s, uint64_t start0) {
    if (nsym == 0) return hipSuccess;
    if (!d_index && t.dec_mode != DEC_FIXED16) return hipErrorInvalidValue;
    DecArgs a;
    fill_dec_args(a, t, d_payload, payload_bytes, nsym);
    a.starts = d_index;
    a.subs = d_index ? d_index + index_sub_offset(a.nblocks) : nullptr;
    a.start0 = start0;
    a.out = d_out; a.err = d_err;
    if (t.dec_mode == DEC_FIXED16) {
        hipError_t e = ensure_lds_limit((const void*)k_decode_fixed16, kFixed16LdsBytes);
        if (e != hipSuccess) return e;
        if ((e = ensure_lds_limit((const void*)k_decode_fixed16_blk, kFixed16LdsBytes)) != hipSuccess) return e;
        const uint64_t nl = (nsym + kSPT - 1) / kSPT;
        // every block but the last through the coalesced kernel; the lane-run kernel takes the last
        const uint64_t nb = kFixed16Blk && a.nblocks > 1 ? a.nblocks - 1 : 0;
        if (nb) {
            uint64_t wgs = (nb + 15) / 16;
            if (wgs > (uint64_t)ncu) wgs = ncu;
            hipLaunchKernelGGL(k_decode_fixed16_blk, dim3(wgs), dim3(1024), kFixed16LdsBytes, s, a, nb);
        }
        uint64_t wgs = (nl + 1023) / 1024;
        if (wgs > (uint64_t)ncu) wgs = ncu;
        hipLaunchKernelGGL(k_decode_fixed16, dim3(wgs), dim3(1024), kFixed16LdsBytes, s, a, nb);
        return hipGetLastError();
    }
    const uint64_t pbits = payload_bytes * 8;
    const bool wide = t.dec_max_len > 32;
    if (t.dec_mode == DEC_DENSE) return run_decode<DEC_DENSE, false, 0>(a, pbits, ncu, s);
    if (wide) return run_decode<DEC_LUT, true, 0>(a, pbits, ncu, s);
    // two levels suffice (no lookup chain past a global subtable): pipelined gathers
    static const int pipe_env = [] { const char* v = getenv("HZ_DEC_PIPE"); return v ? atoi(v) : 2; }();
    if (pipe_env && t.dec_max_len <= t.dec_k + t.dec_level_bits && a.nwords >= 4)
        return pipe_env == 1 ? run_decode<DEC_LUT, false, 1>(a, pbits, ncu, s)
                             : run_decode<DEC_LUT, false, 2>(a, pbits, ncu, s);
    return run_decode<DEC_LUT, false, 0>(a, pbits, ncu, s);
}

// ===========================================================================
// Block index of an index-less stream (a .compressed file from the reference
// encoder; Decompressor.cu:259-291 decodes it serially). Huffman codes
// resynchronise: a decoder started at an arbitrary bit falls onto the true
// codeword boundaries after some codewords (measured on Zipf(1.1): median 83
// bits, p99 590). The stream is cut into 4096-bit segments, one lane each, and
// every segment keeps a BOUNDARY BITMAP (bit d of its row = a codeword starts
// at segment bit d), one bit per payload bit:
//   k_sync_scan   : decode segment k from its first bit to the first boundary
//                   past its end -> exit[k], count[k] and the bitmap of every
//                   boundary of that path in the segment
//   k_sync_iter   : the true path enters k at exit[k-1]; follow it until it
//                   lands on a bitmap boundary (from there both paths agree)
//                   or leaves the segment, rewriting the bitmap up to there
//                   with the true boundaries (count and exit follow). Repeated
//                   (host loop) for segments whose entry changed, until no
//                   exit changes: chains of unsynchronised segments are rare.
//   k_scan_*      : exclusive scan of counts -> first codeword number per segment
//   k_sync_select : the bitmap now holds exactly the true boundaries; every
//                   8th one (a chain start) and every 2048th (a block start)
//                   is picked by popcounts -- no second walk of the stream
//   k_sync_subs   : chain positions relative to their block, max block bits
// ===========================================================================
constexpr uint32_t kSegBits = 4096;
constexpr int kSyncThreads = 1024;
constexpr uint32_t kBmpWords = kSegBits / 32;  // bitmap row of a segment

// Per-lane bit reader over the payload. Words come from 16-byte chunks with
// the next chunk always in flight (128 bits of lookahead, a quarter of the
// load instructions of word reads); past the payload it reads zeros.
struct BitReader {
    uint64_t buf;
    uint32_t nb;
    uint32_t nxt;
    uint4 cur, ahead;   // current chunk (raw words), the next one (in flight)
    uint32_t ci;        // next word of cur
    uint64_t abase;     // word index of `ahead`
};

template <typename A>
HZ_DEV uint4 ld_chunk(const A& a, uint64_t w) {  // w % 4 == 0
    if (w + 4 <= a.nwords) return *reinterpret_cast<const uint4*>(a.words + w);
    uint4 v;
    v.x = w < a.nwords ? a.words[w] : 0u;
    v.y = w + 1 < a.nwords ? a.words[w + 1] : 0u;
    v.z = w + 2 < a.nwords ? a.words[w + 2] : 0u;
    v.w = 0u;
    return v;
}

template <typename A>
HZ_DEV uint32_t br_word(BitReader& r, const A& a) {
    const uint32_t v = pick4(r.cur, r.ci);
    if (++r.ci == 4) {
        r.cur = r.ahead;
        r.ci = 0;
        r.abase += 4;
        r.ahead = ld_chunk(a, r.abase);
    }
    return bswap32(v);
}

template <typename A>
HZ_DEV void br_init(BitReader& r, const A& a, uint64_t p) {
    const uint64_t w = p >> 5;
    const uint32_t sh = (uint32_t)(p & 31);
    const uint64_t base = w & ~3ull;
    r.cur = ld_chunk(a, base);
    r.abase = base + 4;
    r.ahead = ld_chunk(a, r.abase);
    r.ci = (uint32_t)(w & 3);
    const uint32_t w0 = br_word(r, a);
    const uint32_t w1 = br_word(r, a);
    r.buf = (((uint64_t)w0 << 32) | w1) << sh;
    r.nb = 64 - sh;
    r.nxt = br_word(r, a);
}

// Length (and symbol) of the codeword at the reader, then advance past it.
template <int MODE>
HZ_DEV uint32_t br_next(BitReader& r, const DecArgs& a, const uint32_t* lds, uint32_t& sym) {
    if (r.nb <= 32) {
        r.buf |= (uint64_t)r.nxt << (32 - r.nb);
        r.nb += 32;
        r.nxt = br_word(r, a);
    }
    const uint64_t win = r.nb >= 56 ? r.buf : (r.buf | ((uint64_t)r.nxt >> (r.nb - 32)));
    uint32_t L;
    dec_lookup<MODE>(a, lds, win, sym, L);
    if (L < r.nb) {
        r.buf <<= L;
        r.nb -= L;
    } else {
        const uint32_t rr = L - r.nb;
        r.buf = (uint64_t)r.nxt << (32 + rr);
        r.nb = 32 - rr;
        r.nxt = br_word(r, a);
    }
    return L;
}

struct SyncArgs {
    uint64_t start;                 // stream bit of the first symbol (payload view: + bit_adj)
    uint64_t nseg;
    uint32_t* bmp;                  // boundary bitmap, kBmpWords per segment
    unsigned long long* ent;        // entry of a dirty segment: the previous segment's exit
    unsigned long long* cnt;        // boundaries in the segment's bitmap row
    uint32_t* dirty[2];             // segments to check against their entry, ping-pong between iterations
    uint32_t* changed;              // segments whose walk left them in this iteration
};

template <int MODE>
__global__ __launch_bounds__(kSyncThreads) void k_sync_scan(DecArgs a, SyncArgs y) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    copy_lds_table(lds, a.lds_img, a.lds_words);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < y.nseg; k += stride) {
        const uint64_t s0 = y.start + k * kSegBits, s1 = s0 + kSegBits;
        // bitmap words leave four at a time (16-byte stores): every store is a
        // vmcnt entry that later load waits queue behind
        uint4* bm = reinterpret_cast<uint4*>(y.bmp + k * kBmpWords);
        BitReader r;
        br_init(r, a, s0 + a.bit_adj);
        uint64_t pos = s0, n = 0;
        uint32_t cw = 0, cur = 0;  // bitmap word being filled
        uint4 q = make_uint4(0, 0, 0, 0);
        auto put = [&]() {
            const uint32_t j = cw & 3;
            q.x = j == 0 ? cur : q.x;
            q.y = j == 1 ? cur : q.y;
            q.z = j == 2 ? cur : q.z;
            q.w = j == 3 ? cur : q.w;
            if (j == 3) bm[cw >> 2] = q;
            cur = 0;
            ++cw;
        };
        while (pos < s1) {
            const uint32_t d = (uint32_t)(pos - s0);
            while ((d >> 5) != cw) put();
            cur |= 1u << (d & 31);
            uint32_t sym;
            const uint32_t L = br_next<MODE>(r, a, lds, sym);
            if (L == 0) { atomicOr(a.err, 2u); break; }
            pos += L;
            ++n;
        }
        while (cw < kBmpWords) put();
        if (k + 1 < y.nseg) { y.ent[k + 1] = pos; y.dirty[0][k + 1] = 1u; }
        y.cnt[k] = n;
    }
}

// Two segments per lane in lockstep (codebooks the pipelined decoder takes:
// codes <= 32 bits, every global lookup a leaf): both streams' LUT walks and
// gathers are in flight together, so one stream's lookup latency hides the
// other's. Same outputs as the one-segment kernel.
template <typename A>
HZ_DEV void br_refill(BitReader& r, const A& a) {
    if (r.nb <= 32) {
        r.buf |= (uint64_t)r.nxt << (32 - r.nb);
        r.nb += 32;
        r.nxt = br_word(r, a);
    }
}

// Lengths of the codewords at two readers (top 32 bits of each window).
HZ_DEV void lut_len2(const DecArgs& a, const uint32_t* lds, const BitReader (&r)[2], uint32_t (&L)[2]) {
    const uint32_t k = (uint32_t)a.k;
    uint32_t W[2], e[2], x[2], gi[2];
    bool h[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) W[c] = (uint32_t)(r[c].buf >> 32);
#pragma unroll
    for (int c = 0; c < 2; ++c) e[c] = lds[W[c] >> (32 - k)];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        h[c] = lut_lds_link(e[c]);
        x[c] = lds[h[c] ? lut_next32(e[c], W[c]) : 0u];
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        e[c] = h[c] ? x[c] : e[c];
        gi[c] = lut_leaf(e[c]) ? 0u : lut_gnext32(e[c], W[c]);
    }
    const uint32_t g0 = a.l2[gi[0]], g1 = a.l2[gi[1]];
    L[0] = lut_leaf_len((e[0] >> 31) ? e[0] : g0);
    L[1] = lut_leaf_len((e[1] >> 31) ? e[1] : g1);
}

__global__ __launch_bounds__(kSyncThreads) void k_sync_scan2(DecArgs a, SyncArgs y) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    copy_lds_table(lds, a.lds_img, a.lds_words);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k0 < y.nseg; k0 += 2 * stride) {
        BitReader r[2];
        uint64_t s0[2];
        uint32_t d[2], n[2], cw[2], cur[2];  // 32-bit: bits and codewords relative to the segment
        uint4 q[2];
        bool act[2];
        uint4* bm[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const uint64_t k = k0 + c * stride;
            act[c] = k < y.nseg;
            s0[c] = y.start + (act[c] ? k : k0) * kSegBits;
            d[c] = n[c] = 0;
            cw[c] = cur[c] = 0;
            q[c] = make_uint4(0, 0, 0, 0);
            bm[c] = reinterpret_cast<uint4*>(y.bmp + (act[c] ? k : k0) * kBmpWords);
            br_init(r[c], a, s0[c] + a.bit_adj);
        }
        auto put = [&](int c) {
            const uint32_t j = cw[c] & 3;
            q[c].x = j == 0 ? cur[c] : q[c].x;
            q[c].y = j == 1 ? cur[c] : q[c].y;
            q[c].z = j == 2 ? cur[c] : q[c].z;
            q[c].w = j == 3 ? cur[c] : q[c].w;
            if (j == 3) bm[c][cw[c] >> 2] = q[c];
            cur[c] = 0;
            ++cw[c];
        };
        while (act[0] || act[1]) {
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                // codes <= 32 bits: the boundary's bitmap word advances by at most one per step
                if (act[c]) {
                    if ((d[c] >> 5) != cw[c]) put(c);
                    cur[c] |= 1u << (d[c] & 31);
                }
                br_refill(r[c], a);
            }
            uint32_t L[2];
            lut_len2(a, lds, r, L);
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (!act[c]) continue;
                if (L[c] == 0) { atomicOr(a.err, 2u); act[c] = false; continue; }
                r[c].buf <<= L[c];
                r[c].nb -= L[c];
                d[c] += L[c];
                ++n[c];
                act[c] = d[c] < kSegBits;
            }
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const uint64_t k = k0 + c * stride;
            if (k >= y.nseg) continue;
            while (cw[c] < kBmpWords) put(c);
            if (k + 1 < y.nseg) { y.ent[k + 1] = s0[c] + d[c]; y.dirty[0][k + 1] = 1u; }
            y.cnt[k] = n[c];
        }
    }
}

// ---------------------------------------------------------------------------
// Index walker for the pipelined decoder's codebooks (codes <= 32 bits, one
// global LUT level): LONG chains -- each lane walks kWalkChains stretches of spc whole
// segments, each starting kWalkLead bits early so the walk has resynchronised
// (P(not) ~ 4e-4 on Zipf) when it reaches its first segment: one start per
// ~10^5 codewords instead of one per segment. Each chain streams its payload
// through a 4-chunk LDS ring (16-byte chunks, one refill load per round,
// issued a round ahead) and marks boundaries into a 4-chunk LDS mark ring
// (ds_or), flushed one chunk per round as a 16-byte store into the bitmap;
// per-segment counts come from popcounts of the flushed chunks.
// Lookups use the decoder's level 1 with hot heads sized to the LDS the rings
// leave; a chain whose code needs the global level PARKS for the rest of the
// round, and the round ends with one gather for all parked chains: every wait
// is the round's single vmcnt(0) (refill + gathers), never a gather queued
// behind a refill in mid-walk.
// A chain's exit becomes the entry of the next chain's first segment
// (ent/dirty): k_sync_iter checks it against the bitmap, which lands at once
// when the lead-in resynchronised.
// ---------------------------------------------------------------------------
// steps per round: u8 table 8: 25.5 ms, 10: 25.3 ms; 4-bit table 10/12/14: 24.7/24.4/24.6 ms;
// round 4 (16 GiB Zipf, A/B in one run, k_idx_walk alone): 12 / 14 / 16 steps 17.32 / 17.11 / 17.44 ms
constexpr int kWalkSteps = 14;
// parked chains resume after each part of a round: 2 parts of 6 steps 23.6-23.9 ms, 1 part
// 23.7-24.3, 2 x 8 23.4-23.9, 3 x 6 23.2-24.3, 3 x 4 24.8, 4 x 4 23.5-24.2 (A/B in one run);
// round 3 (2.3 % escapes): 2 / 1 / 3 parts 22.1 / 22.1-22.3 / 23.4 ms
constexpr int kWalkHalves = 2;
constexpr uint32_t kWalkLead = 1024;    // lead-in bits before a chain's first segment

struct WalkArgs {
    const uint32_t* words;    // payload view, 64-byte aligned
    uint64_t nwords;          // >= 4 (host check)
    uint32_t bit_adj;         // payload bit 0 = bit bit_adj of words
    uint64_t start;           // stream bit of the first symbol
    uint64_t nseg, spc, nchains;
    const uint32_t* lds_img;  // 4-bit code length - bias per k-bit window (0: longer than k bits)
    uint32_t lds_words;
    int k, bias;
    const uint8_t* esc;       // u8 code length per m-bit window (escapes only)
    int m;
    uint32_t* bmp;
    unsigned long long* cnt;
    unsigned long long* ent;
    uint32_t* dirty;
    uint32_t lead;            // k_chain_walk: lead-in bits before a chain's first bit
    const uint32_t* w8_img;   // k_chain_walk: u8 code length per k8-bit window (0: escape)
    uint32_t w8_words;
    int k8;
    const uint32_t* lut1;     // k_chain_walk<DEEP>: the decode LUT (level-1 image, global levels) that
    const uint32_t* lut2;     // resolves escapes the m-bit escape table leaves at 0 (codes > m bits)
    int lutk;
};

// 16 payload bytes at word w (4-aligned): zeros before word 0 / past the end.
HZ_DEV uint4 walk_load(const WalkArgs& a, uint64_t w) {
    const bool in = w < a.nwords;  // false for a window that wrapped below word 0
    const uint64_t wl = !in ? 0 : (w + 4 <= a.nwords ? w : a.nwords - 4);
    return *reinterpret_cast<const uint4*>(a.words + wl);
}
HZ_DEV uint4 walk_fix(const WalkArgs& a, uint64_t w, uint4 x) {
    if (w < a.nwords && w + 4 <= a.nwords) return x;
    const uint64_t base = a.nwords - 4;
    uint32_t q[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const uint64_t wt = w + t;
        q[t] = wt < a.nwords && w < a.nwords ? pick4(x, (uint32_t)(wt - base)) : 0u;
    }
    return make_uint4(q[0], q[1], q[2], q[3]);
}

// Chunk slot q (0..3) of a payload ring, byte-swapped.
template <uint32_t ROW>
HZ_DEV void ring_put(uint32_t* ring, uint32_t q, const uint4& x) {
    const uint32_t v[4] = {bswap32(x.x), bswap32(x.y), bswap32(x.z), bswap32(x.w)};
#pragma unroll
    for (int i = 0; i < 4; ++i) ring[(4 * q + i) * ROW] = v[i];
}

// Payload chunks reach a chain's ring from a register group of kWalkGroup
// chunks loaded together (one 64/128-byte run per lane, issued as soon as the
// previous group is in the ring), and finished mark chunks leave as a run of
// kWalkMarkGroup chunks: every lane touches a different stretch of the stream,
// so 16-byte accesses spread over many rounds let L2 evict a line between them
// (fetches ~10x the payload, writes ~3.5x the bitmap with single chunks).
// Measured (u32 LUT walker): 1/1 chunks 41.7 ms, 4/4 38.7, 1/8 38.9, 8/8 41.7; (4-bit walker)
// 4/4 23.9-24.3 ms, 2/4 24.9, 8/4 24.9, 4/2 26.8, 4/8 24.1, 8/8 25.0.
constexpr uint32_t kWalkGroup = 4;
constexpr uint32_t kWalkMarkGroup = 4;
static_assert((kWalkGroup & (kWalkGroup - 1)) == 0 && kWalkGroup >= 1 && kWalkGroup <= 8, "walk group");
static_assert((kWalkMarkGroup & (kWalkMarkGroup - 1)) == 0 && kWalkMarkGroup >= 1 && kWalkMarkGroup <= 8,
              "mark group");

template <uint32_t G>
HZ_DEV uint4 pick_group(const uint4 (&g)[G], uint32_t i) {
    uint4 x = g[0];
#pragma unroll
    for (uint32_t t = 1; t < G; ++t) {
        const bool s = i == t;
        x.x = s ? g[t].x : x.x;
        x.y = s ? g[t].y : x.y;
        x.z = s ? g[t].z : x.z;
        x.w = s ? g[t].w : x.w;
    }
    return x;
}

__global__ __launch_bounds__(kWalkWaves * 64) void k_idx_walk(WalkArgs a) {
    // the length table at LDS address 0 (a static array: its address folds into
    // the ds_read offset), the rings after it
    __shared__ __attribute__((aligned(16))) uint32_t wtab[(1u << kWalkK) / 8];
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    copy_lds_table(wtab, a.lds_img, a.lds_words);
    const uint8_t* lds8 = reinterpret_cast<const uint8_t*>(wtab);
    constexpr int C = kWalkChains;
    constexpr uint32_t kRow = 1;  // ring word stride
    constexpr uint32_t G = kWalkGroup, GM = kWalkMarkGroup;
    constexpr uint32_t kMarkRow = 16;  // ring words 0..15 payload, then kWalkMarkChunks mark chunks, 1 pad
    constexpr uint32_t kMW = 4 * kWalkMarkChunks;  // mark ring words
    const uint32_t k = (uint32_t)a.k, bias = (uint32_t)a.bias;
    const int lane = threadIdx.x & 63;
    const uint32_t wid = threadIdx.x >> 6;
    const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t* ring[C];
    uint32_t off[C], off0[C], ms[C], end[C], f[C], mcount[C], nmc[C], rc[C];
    uint64_t bch[C], x0[C], seg0[C], seg1[C];
    bool live[C], pk[C], on[C];  // on: the walk has reached ms (marks count)
    uint4 pre[C][G];   // payload group holding chunk f
    uint4 mk[C][GM];   // finished mark chunks of the current run
    // window registers: the 32 bits at off are alignbit(w0, w1, sh) (sh in 0..31;
    // 32 - sh bits of w0 consumed), nxt = ring word wn, the one after w1
    uint32_t w0[C], w1[C], sh[C], wn[C], nxt[C];
    bool gin[C];  // the payload group in pre[] lies inside the payload (no clamping)
#pragma unroll
    for (int c = 0; c < C; ++c) {
        ring[c] = lds + ((wid * C + c) * 64 + lane) * kRingWords;
        const uint64_t ch = tid + c * T;
        live[c] = ch < a.nchains;
        const uint64_t chc = live[c] ? ch : 0;
        seg0[c] = chc * a.spc;
        seg1[c] = seg0[c] + a.spc < a.nseg ? seg0[c] + a.spc : a.nseg;
        const uint64_t cs = seg0[c] * kSegBits, ce = seg1[c] * kSegBits;
        x0[c] = cs - (cs < kWalkLead ? cs : kWalkLead);
        const uint64_t P0 = a.start + a.bit_adj + x0[c];
        bch[c] = (P0 >> 7) - 1;  // one chunk before the walk (wraps to ~0 at the payload's start: zeros)
        off0[c] = off[c] = (uint32_t)(P0 - 128 * bch[c]);
        ms[c] = off[c] + (uint32_t)(cs - x0[c]);
        end[c] = live[c] ? off[c] + (uint32_t)(ce - x0[c]) : off[c];
        nmc[c] = live[c] ? (uint32_t)((ce - cs) / 128) : 0u;
        mcount[c] = rc[c] = 0;
        pk[c] = false;
        on[c] = ms[c] == off[c];
#pragma unroll
        for (uint32_t i = kMarkRow; i < kRingWords; ++i) ring[c][i * kRow] = 0u;
#pragma unroll
        for (uint32_t i = 0; i < GM; ++i) mk[c][i] = make_uint4(0, 0, 0, 0);
    }
    // prologue: chunks 0..2 of every chain, and the group holding chunk 3
#pragma unroll
    for (int c = 0; c < C; ++c) {
        uint4 v[3];
#pragma unroll
        for (int g = 0; g < 3; ++g) v[g] = walk_load(a, 4 * (bch[c] + g));
        const uint64_t gb = (bch[c] + 3) & ~(uint64_t)(G - 1);
        gin[c] = 4 * (gb + G) <= a.nwords && gb < a.nwords;
#pragma unroll
        for (uint32_t g = 0; g < G; ++g) pre[c][g] = walk_load(a, 4 * (gb + g));
#pragma unroll
        for (int g = 0; g < 3; ++g) {
            ring_put<kRow>(ring[c], (uint32_t)g, walk_fix(a, 4 * (bch[c] + g), v[g]));
        }
        f[c] = 3;
        const uint32_t q0 = (off[c] - 1) >> 5;
        w0[c] = ring[c][q0 * kRow];
        w1[c] = ring[c][(q0 + 1) * kRow];
        sh[c] = (0u - off[c]) & 31;
        wn[c] = q0 + 2;
    }
    uint32_t pW[C];  // a parked chain's window
    // chunk f goes into the ring at a round's end when it fits (the chain no
    // longer needs chunk f - 4), ahead of the round's bitmap stores
    for (;;) {
        bool alive = false;
#pragma unroll
        for (int c = 0; c < C; ++c) alive |= off[c] < end[c] || mcount[c] < nmc[c];
        if (!__any(alive)) break;
        // the round's steps stay below: chain end, filled data (w0, w1 and nxt: the
        // bits below off + 96), free mark slots
        uint32_t lim[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            lim[c] = min(on[c] ? end[c] : ms[c], min(128 * f[c] - 96, ms[c] + 128 * (mcount[c] + kWalkMarkChunks)));
            nxt[c] = ring[c][(wn[c] & 15) * kRow];  // (re)read after the ring's refill
        }
        // branch-free steps: one LDS length lookup per chain and step; a chain that
        // cannot step only leaves off unchanged, a code longer than k bits parks the
        // chain for the rest of the round
        // parked chains: one gather from the escape table for all of them, then
        // the codeword is marked and stepped over (mid-round and at the round's end)
        auto resolve = [&]() {
            uint32_t g[C];
#pragma unroll
            for (int c = 0; c < C; ++c)
                if (pk[c]) g[c] = a.esc[pW[c] >> (32 - a.m)];
#pragma unroll
            for (int c = 0; c < C; ++c) {
                if (!pk[c]) continue;
                if (off[c] >= ms[c]) {
                    const uint32_t rel = off[c] - ms[c];
                    atomicOr(ring[c] + (kMarkRow + ((rel >> 5) & (kMW - 1))) * kRow, 1u << (rel & 31));
                }
                const uint32_t L = g[c];
                off[c] += L;
                const int32_t r = (int32_t)sh[c] - (int32_t)L;
                if (r < 0) {
                    w0[c] = w1[c];
                    w1[c] = nxt[c];
                    ++wn[c];
                    nxt[c] = ring[c][(wn[c] & 15) * kRow];
                }
                sh[c] = (uint32_t)(r < 0 ? r + 32 : r);
                pk[c] = false;
            }
        };
#pragma unroll
        for (int half = 0; half < kWalkHalves; ++half) {
#pragma unroll
            for (int t = 0; t < kWalkSteps / kWalkHalves; ++t) {
                uint32_t W[C], e[C];
                bool ok[C];
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    ok[c] = !pk[c] & (off[c] < lim[c]);
                    W[c] = __builtin_amdgcn_alignbit(w0[c], w1[c], sh[c]);
                    e[c] = lds8[W[c] >> (33 - k)];  // two windows per byte (k >= 2)
                }
                HZ_WALK_FENCE();
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    e[c] = __builtin_amdgcn_ubfe(e[c], (W[c] >> (30 - k)) & 4u, 4);  // the window's nibble
                    const bool adv = ok[c] & (e[c] != 0u), park = ok[c] ^ adv;
                    // lead-in marks (off < ms) land in the ring too; it is cleared when
                    // the walk reaches ms
                    const uint32_t rel = off[c] - ms[c];
                    const uint32_t bit = adv ? (1u << (rel & 31)) : 0u;
                    atomicOr(ring[c] + (kMarkRow + ((rel >> 5) & (kMW - 1))) * kRow, bit);  // the mark ring (a zero bit: no mark)
                    const uint32_t L = adv ? e[c] + bias : 0u;
                    off[c] += L;
                    const int32_t r = (int32_t)sh[c] - (int32_t)L;  // >= -32 (codes <= 32 bits)
                    const bool cr = r < 0;                         // w0 used up: shift the words
                    w0[c] = cr ? w1[c] : w0[c];
                    w1[c] = cr ? nxt[c] : w1[c];
                    sh[c] = (uint32_t)(cr ? r + 32 : r);
                    wn[c] += cr ? 1u : 0u;
                    nxt[c] = ring[c][(wn[c] & 15) * kRow];
                    pk[c] |= park;
                    pW[c] = park ? W[c] : pW[c];
                }
            }
            resolve();
        }
        bool fl[C], ld[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            if (!on[c] && off[c] >= ms[c]) {  // the lead-in is over: drop its marks
#pragma unroll
                for (uint32_t i = kMarkRow; i < kMarkRow + kMW; ++i) ring[c][i * kRow] = 0u;
                on[c] = true;
            }
            ld[c] = false;
            if (f[c] <= ((off[c] - 1) >> 7) + 3) {
                const uint64_t q = bch[c] + f[c];
                uint4 x = pick_group<G>(pre[c], (uint32_t)q & (G - 1));
                if (!gin[c]) x = walk_fix(a, 4 * q, x);
                ring_put<kRow>(ring[c], f[c] & 3, x);
                ++f[c];
                ld[c] = ((q + 1) & (G - 1)) == 0;  // the group is in the ring: load the next one
            }
            // mark chunk mcount is done once the walk is past it
            fl[c] = mcount[c] < nmc[c] && off[c] >= ms[c] && off[c] - ms[c] >= 128 * (mcount[c] + 1);
            if (fl[c]) {
                uint32_t* slot = ring[c] + (kMarkRow + 4 * (mcount[c] & (kWalkMarkChunks - 1))) * kRow;
                const uint4 m = make_uint4(slot[0], slot[kRow], slot[2 * kRow], slot[3 * kRow]);
#pragma unroll
                for (int i = 0; i < 4; ++i) slot[i * kRow] = 0u;
                rc[c] = ((mcount[c] & 31) ? rc[c] : 0u) + __popc(m.x) + __popc(m.y) + __popc(m.z) + __popc(m.w);
#pragma unroll
                for (uint32_t i = 0; i + 1 < GM; ++i) mk[c][i] = mk[c][i + 1];  // shift in (constant indices)
                mk[c][GM - 1] = m;
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {  // the next group's loads, then this round's bitmap stores
            if (!ld[c]) continue;
            const uint64_t q = bch[c] + f[c];
            gin[c] = 4 * (q + G) <= a.nwords;
            if (gin[c]) {
                const uint4* src = reinterpret_cast<const uint4*>(a.words) + q;
#pragma unroll
                for (uint32_t i = 0; i < G; ++i) pre[c][i] = src[i];
            } else {
#pragma unroll
                for (uint32_t i = 0; i < G; ++i) pre[c][i] = walk_load(a, 4 * (q + i));
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
            if (!fl[c]) continue;
            const uint64_t j = seg0[c] * (kSegBits / 128) + mcount[c];
            if ((mcount[c] & (GM - 1)) == GM - 1) {
                uint4* dst = reinterpret_cast<uint4*>(a.bmp) + (j - (GM - 1));
#pragma unroll
                for (uint32_t i = 0; i < GM; ++i)
                    store_nt16(dst + i, mk[c][i]);  // read back by k_sync_select only (16.0 vs 16.3 ms walk, round 3)
            }
            if ((mcount[c] & 31) == 31) a.cnt[j >> 5] = rc[c];
            ++mcount[c];
        }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
        if (!live[c] || seg1[c] >= a.nseg) continue;
        a.ent[seg1[c]] = a.start + x0[c] + (off[c] - off0[c]);
        a.dirty[seg1[c]] = 1u;
    }
}

// Fix-up of a dirty segment k from its true entry ent[k] (the previous
// segment's exit): walk until the path lands on a boundary of the segment's
// bitmap (the paths agree from there) or leaves the segment. The bitmap words
// the walk passes are rewritten with the walked boundaries (the landing word
// keeps its bits from the landing point on), so the row keeps holding one
// consistent path, and its count follows. A walk that leaves the segment
// hands its end to segment k + 1 for the next iteration.
template <int MODE>
__global__ __launch_bounds__(kSyncThreads) void k_sync_iter(DecArgs a, SyncArgs y, int it) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    copy_lds_table(lds, a.lds_img, a.lds_words);
    const uint32_t* dr = y.dirty[it & 1];
    uint32_t* dw = y.dirty[(it + 1) & 1];
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < y.nseg; k += stride) {
        if (!dr[k]) continue;
        const uint64_t s0 = y.start + k * kSegBits, s1 = s0 + kSegBits;
        uint32_t* bm = y.bmp + k * kBmpWords;
        uint64_t p = y.ent[k];
        uint32_t walked = 0, below = 0, acc = 0, cw = 0;
        uint32_t old = bm[0];  // the row's word cw before the rewrite
        bool landed = false;
        BitReader r;
        br_init(r, a, p + a.bit_adj);
        while (p < s1) {
            const uint32_t d = (uint32_t)(p - s0);
            while ((d >> 5) != cw) {  // words the walk has passed: the walked boundaries replace them
                below += __popc(old);
                bm[cw] = acc;
                acc = 0;
                old = bm[++cw];
            }
            if ((old >> (d & 31)) & 1u) { landed = true; break; }
            acc |= 1u << (d & 31);
            uint32_t sym;
            const uint32_t L = br_next<MODE>(r, a, lds, sym);
            if (L == 0) { atomicOr(a.err, 2u); break; }
            p += L;
            ++walked;
        }
        if (landed) {
            const uint32_t lowm = (1u << ((uint32_t)(p - s0) & 31)) - 1u;
            below += __popc(old & lowm);
            bm[cw] = acc | (old & ~lowm);
            y.cnt[k] = y.cnt[k] - below + walked;
        } else {
            for (; cw < kBmpWords; ++cw) { bm[cw] = acc; acc = 0; }
            y.cnt[k] = walked;
            if (k + 1 < y.nseg) { y.ent[k + 1] = p; dw[k + 1] = 1u; }
            atomicAdd(y.changed, 1u);
        }
    }
}

// Position (0..31) of the r-th (0-based) set bit of m; r < popc(m).
HZ_DEV uint32_t select_bit(uint32_t m, uint32_t r) {
    uint32_t pos = 0, c;
    c = __popc(m & 0xffffu); if (r >= c) { r -= c; pos += 16; m >>= 16; }
    c = __popc(m & 0xffu);   if (r >= c) { r -= c; pos += 8;  m >>= 8; }
    c = __popc(m & 0xfu);    if (r >= c) { r -= c; pos += 4;  m >>= 4; }
    c = __popc(m & 0x3u);    if (r >= c) { r -= c; pos += 2;  m >>= 2; }
    return pos + ((r >= (m & 1u)) ? 1u : 0u);
}

// One workgroup per tile of kSelTileSegs bitmap rows (64 Kbit); thread t
// holds words [8 t, 8 t + 8). A workgroup scan of popcounts numbers every
// boundary from the tile's first (first[] of its first row). Boundary i < nsym
// with i % 8 == 0 is a chain start (raw position, low 16 bits, staged in LDS
// and stored as one contiguous run, the form hz_pack writes),
// i % 2048 == 0 also a block start; boundary nsym is the end of the stream.
constexpr int kSelectThreads = 256;
constexpr uint32_t kSelTileSegs = 16;
constexpr uint32_t kSelTileWords = kSelTileSegs * kBmpWords;  // 2048 = 8 words per thread
constexpr uint32_t kSelMaxChains = kSelTileWords * 32 / kChainSyms + 2;
constexpr int kSelAhead = 1;
__global__ __launch_bounds__(kSelectThreads) void k_sync_select(SyncArgs y, uint64_t nsym, uint64_t nblocks,
                                                                const unsigned long long* first,
                                                                unsigned long long* starts, uint16_t* subs) {
    __shared__ uint16_t ch[kSelMaxChains];
    __shared__ uint32_t wsum[kSelectThreads / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t ntile = (y.nseg + kSelTileSegs - 1) / kSelTileSegs;
    const uint64_t nch_all = (nsym + kChainSyms - 1) / kChainSyms;  // chains with a start inside the stream
    const uint64_t nw = y.nseg * kBmpWords;
    // the next tile's first[] and bitmap words are loaded while this one is processed
    auto load = [&](uint64_t tile, uint64_t& f, uint32_t (&mm)[8]) {
        const uint64_t w0 = tile * kSelTileWords + 8u * threadIdx.x;
        f = first[tile * kSelTileSegs];
        if (w0 + 8 <= nw) {
            const uint4* q = reinterpret_cast<const uint4*>(y.bmp + w0);
            const uint4 a = q[0], b = q[1];
            mm[0] = a.x; mm[1] = a.y; mm[2] = a.z; mm[3] = a.w; mm[4] = b.x; mm[5] = b.y; mm[6] = b.z; mm[7] = b.w;
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) mm[i] = w0 + i < nw ? y.bmp[w0 + i] : 0u;
        }
    };
    // kSelAhead tiles in flight per thread (16 GiB Zipf: 1 / 3 / 5 ahead 4.61 / 4.89 / 5.03 ms, round 3)
    uint64_t fn[kSelAhead] = {};
    uint32_t mn[kSelAhead][8];
#pragma unroll
    for (int d = 0; d < kSelAhead; ++d)
        if (blockIdx.x + d * (uint64_t)gridDim.x < ntile) load(blockIdx.x + d * (uint64_t)gridDim.x, fn[d], mn[d]);
    for (uint64_t tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
        const uint64_t seg0 = tile * kSelTileSegs;
        const uint64_t f0 = fn[0];
        uint32_t m[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) m[i] = mn[0][i];
#pragma unroll
        for (int d = 0; d + 1 < kSelAhead; ++d) {
            fn[d] = fn[d + 1];
#pragma unroll
            for (int i = 0; i < 8; ++i) mn[d][i] = mn[d + 1][i];
        }
        if (tile + kSelAhead * (uint64_t)gridDim.x < ntile)
            load(tile + kSelAhead * (uint64_t)gridDim.x, fn[kSelAhead - 1], mn[kSelAhead - 1]);
        if (f0 > nsym) break;  // workgroup-uniform; later tiles start later still
        const uint64_t w0 = seg0 * kBmpWords + 8u * threadIdx.x;
        uint32_t c[8], tot = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) { c[i] = __popc(m[i]); tot += c[i]; }
        const uint32_t incl = wave_incl_sum(tot);
        if (lane == 63) wsum[wid] = incl;
        __syncthreads();
        uint32_t wpre = 0, all = 0;
#pragma unroll
        for (int w = 0; w < kSelectThreads / 64; ++w) {
            const uint32_t v = wsum[w];
            wpre += w < wid ? v : 0u;
            all += v;
        }
        // 32-bit arithmetic relative to the tile's first boundary f0
        const uint32_t d0 = wpre + incl - tot;  // the thread's first boundary: number f0 + d0
        const uint64_t left = nsym - f0;
        const uint32_t dn = left < 0xffffffffull ? (uint32_t)left : 0xffffffffu;  // boundaries before nsym
        const uint32_t q = (uint32_t)(f0 & 7), qb = (uint32_t)(f0 & (kBlockSyms - 1));
        const uint64_t base = y.start + w0 * 32;
        const uint64_t cb = (f0 + kChainSyms - 1) / kChainSyms;  // first chain starting in the tile
        uint32_t cum[8];
        cum[0] = 0;
#pragma unroll
        for (int h = 1; h < 8; ++h) cum[h] = cum[h - 1] + c[h - 1];
        // the thread's boundary of rank r (0-based): word h = #(cum[1..7] <= r), bit = select in m[h]
        // the select operands pass through an empty asm: a select between two loads
        // of m[] / cum[] is otherwise folded into one dynamically indexed (scratch) load
        auto pos_of = [&](uint32_t r) -> uint64_t {
            uint32_t mh = m[0], ch0 = 0, sh = 0;
            asm volatile("" : "+v"(mh));
#pragma unroll
            for (int h = 1; h < 8; ++h) {
                uint32_t mv = m[h], cv = cum[h];
                asm volatile("" : "+v"(mv), "+v"(cv));
                const bool in = r >= cv;
                mh = in ? mv : mh;
                ch0 = in ? cv : ch0;
                sh = in ? 32u * h : sh;
            }
            return base + sh + select_bit(mh, r - ch0);
        };
        if (d0 <= dn && dn < d0 + tot) starts[nblocks] = pos_of(dn - d0);
        // chain starts: boundaries whose number is a multiple of 8
        for (uint32_t r = (8u - ((q + d0) & 7)) & 7; r < tot && d0 + r < dn; r += 8) {
            const uint32_t d = d0 + r;
            const uint64_t pos = pos_of(r);
            ch[((q + d) >> 3) - (q ? 1u : 0u)] = (uint16_t)pos;
            if (((qb + d) & (kBlockSyms - 1)) == 0) starts[(f0 + d) / kBlockSyms] = pos;
        }
        // the rows hold exactly nsym boundaries: the last codeword ends at the bitmap's end
        if (threadIdx.x == 0 && seg0 + kSelTileSegs >= y.nseg && f0 + all == nsym)
            starts[nblocks] = y.start + y.nseg * kSegBits;
        __syncthreads();
        uint64_t ce = (f0 + all + kChainSyms - 1) / kChainSyms;
        ce = ce < nch_all ? ce : nch_all;
        for (uint64_t t = cb + threadIdx.x; t < ce; t += kSelectThreads) subs[t] = ch[t - cb];
        __syncthreads();
    }
}

// Chains past the stream's end (all in the last block) start at the end, and
// the largest block's bits. The select already wrote every other chain's
// start (low 16 bits of its stream bit, as hz_pack does).
__global__ __launch_bounds__(256) void k_sync_subs(uint64_t nsym, uint64_t nblocks, unsigned long long* starts,
                                                   unsigned long long* sub64) {
    if (nblocks == 0) return;  // no block: nothing to fix (the launcher never sends one; a guard, not a path)
    const uint64_t end = starts[nblocks];
    if (blockIdx.x == 0 && threadIdx.x < kWave) {
        const uint64_t q = (nblocks - 1) * kWave + threadIdx.x;
        const uint64_t raw = sub64[q];
        uint64_t out = 0;
#pragma unroll
        for (int t = 0; t < kChainsPerLane; ++t) {
            const uint64_t c = q * kChainsPerLane + t;
            const uint64_t p = c * kChainSyms < nsym ? (raw >> (16 * t)) & 0xffffu : end & 0xffffu;
            out |= p << (16 * t);
        }
        sub64[q] = out;
    }
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long mx = 0;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nblocks; b += stride) {
        const unsigned long long bits = starts[b + 1] - starts[b];
        mx = bits > mx ? bits : mx;
    }
    for (int m = 32; m >= 1; m >>= 1) {
        const uint32_t lo = shfl_xor_u32((uint32_t)mx, m), hi = shfl_xor_u32((uint32_t)(mx >> 32), m);
        const unsigned long long o = ((unsigned long long)hi << 32) | lo;
        mx = o > mx ? o : mx;
    }
    if ((threadIdx.x & 63) == 0 && mx) atomicMax(starts + nblocks + 1, mx);
}

uint64_t index_scratch_words(uint64_t payload_bytes, uint64_t start_bit) {
    const uint64_t bits = payload_bytes * 8 > start_bit ? payload_bytes * 8 - start_bit : 0;
    const uint64_t nseg = (bits + kSegBits - 1) / kSegBits;
    const uint64_t ntiles = (nseg + kScanTile - 1) / kScanTile;
    // ent, cnt, first (u64), bitmap (kBmpWords u32), dirty[2] (u32), counter, tiles
    return nseg * (3 + kBmpWords / 2 + 1) + 1 + ntiles + 24;
}

// Common tail of the index build, after the boundary bitmap and the dirty
// entries exist: fix-ups to a fixed point, count scan, select, subs.
template <int MODE>
static hipError_t finish_index(const DecArgs& a, SyncArgs y, unsigned long long* first, unsigned long long* tiles,
                               unsigned long long* d_index, uint32_t* h_changed, uint32_t lds, int ncu,
                               hipStream_t s) {
    {
        hipError_t e = ensure_lds_limit((const void*)k_sync_iter<MODE>, kLdsBytes);
        if (e != hipSuccess) return e;
    }
    uint64_t wgs = (y.nseg + kSyncThreads - 1) / kSyncThreads;
    const uint64_t cap = (uint64_t)ncu * (lds ? (kLdsBytes / lds < 2 ? 1 : 2) : 2);
    wgs = wgs < cap ? (wgs ? wgs : 1) : cap;
    // resolve entries until no walk leaves its segment (host loop; typically 1-2 passes)
    for (int it = 0;; ++it) {
        hipError_t e = hipMemsetAsync(y.changed, 0, 4, s);
        if (e != hipSuccess) return e;
        if ((e = hipMemsetAsync(y.dirty[(it + 1) & 1], 0, 4 * y.nseg, s)) != hipSuccess) return e;
        hipLaunchKernelGGL(k_sync_iter<MODE>, dim3(wgs), dim3(kSyncThreads), lds, s, a, y, it);
        if ((e = hipMemcpyAsync(h_changed, y.changed, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        if (*h_changed == 0 || it > (int)y.nseg) break;
    }
    const uint64_t ntiles = (y.nseg + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(k_scan_reduce, dim3(ntiles), dim3(kScanThreads), 0, s, (const unsigned long long*)y.cnt, y.nseg,
                       tiles, 0xffffffffull);
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kScanThreads), 0, s, tiles, ntiles, 0ull);
    hipLaunchKernelGGL(k_scan_apply, dim3(ntiles), dim3(kScanThreads), 0, s, (const unsigned long long*)y.cnt, y.nseg,
                       (const unsigned long long*)tiles, first, 0xffffffffull);
    uint16_t* subs = reinterpret_cast<uint16_t*>(d_index + index_sub_offset(a.nblocks));
    // end bit = all ones unless the payload holds nsym codewords (k_sync_select writes it then)
    hipError_t e = hipMemsetAsync(d_index + a.nblocks, 0xff, 8, s);
    if (e != hipSuccess) return e;
    if ((e = hipMemsetAsync(d_index + a.nblocks + 1, 0, 8, s)) != hipSuccess) return e;
    {
        // tiles in order over a grid-stride loop: a workgroup stops at the first tile past the stream
        uint64_t sg = (y.nseg + kSelTileSegs - 1) / kSelTileSegs;
        sg = sg < (uint64_t)ncu * 8 ? sg : (uint64_t)ncu * 8;
        hipLaunchKernelGGL(k_sync_select, dim3(sg), dim3(kSelectThreads), 0, s, y, a.nsym, a.nblocks,
                           (const unsigned long long*)first, d_index, subs);
    }
    uint64_t sw = (a.nblocks + 255) / 256;
    sw = sw < (uint64_t)ncu * 4 ? (sw ? sw : 1) : (uint64_t)ncu * 4;
    hipLaunchKernelGGL(k_sync_subs, dim3(sw), dim3(256), 0, s, a.nsym, a.nblocks, d_index,
                       d_index + index_sub_offset(a.nblocks));
    return hipGetLastError();
}

// Boundary bitmap by the LUT walkers (one or two 4096-bit segments per lane).
template <int MODE>
static hipError_t scan_lut(const DecArgs& a, SyncArgs y, uint32_t lds, int ncu, hipStream_t s) {
    {
        hipError_t e = ensure_lds_limit((const void*)k_sync_scan<MODE>, kLdsBytes);
        if (e != hipSuccess) return e;
    }
    // 16-wave workgroups: one table copy per workgroup, as many waves as a CU holds
    uint64_t wgs = (y.nseg + kSyncThreads - 1) / kSyncThreads;
    const uint64_t cap = (uint64_t)ncu * (lds ? (kLdsBytes / lds < 2 ? 1 : 2) : 2);
    wgs = wgs < cap ? (wgs ? wgs : 1) : cap;
    // two segments per lane where the pipelined decoder's table shape holds
    const bool two = MODE == DEC_LUT && a.max_len <= 32 && a.max_len <= a.k + a.level_bits;
    if (two) {
        hipError_t e = ensure_lds_limit((const void*)k_sync_scan2, kLdsBytes);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_sync_scan2, dim3(wgs), dim3(kSyncThreads), lds, s, a, y);
    } else {
        hipLaunchKernelGGL(k_sync_scan<MODE>, dim3(wgs), dim3(kSyncThreads), lds, s, a, y);
    }
    return hipGetLastError();
}

// Boundary bitmap by the long-chain walker.
static hipError_t scan_walk(const Tables& t, const DecArgs& a, SyncArgs y, int ncu, hipStream_t s) {
    hipError_t e = ensure_lds_limit((const void*)k_idx_walk, (int)kWalkLdsRingBytes);  // + the static table
    if (e != hipSuccess) return e;
    WalkArgs w;
    w.words = a.words; w.nwords = a.nwords; w.bit_adj = a.bit_adj;
    w.start = y.start; w.nseg = y.nseg;
    const uint64_t per_wg = (uint64_t)kWalkWaves * 64 * kWalkChains;
    const uint64_t target = per_wg * (uint64_t)ncu;
    w.spc = (y.nseg + target - 1) / target;
    w.nchains = (y.nseg + w.spc - 1) / w.spc;
    w.lds_img = t.d_walk_lds; w.lds_words = t.walk_lds_bytes / 4;
    w.k = t.walk_k; w.bias = t.walk_bias; w.esc = reinterpret_cast<const uint8_t*>(t.d_walk_esc); w.m = t.walk_m;
    w.bmp = y.bmp; w.cnt = y.cnt; w.ent = y.ent; w.dirty = y.dirty[0]; w.lead = kWalkLead;
    w.w8_img = nullptr; w.w8_words = 0; w.k8 = 0;
    // chains tid and tid + T of every thread
    const uint64_t threads_needed = (w.nchains + kWalkChains - 1) / kWalkChains;
    uint64_t wgs = (threads_needed + kWalkWaves * 64 - 1) / (kWalkWaves * 64);
    wgs = wgs ? wgs : 1;
    hipLaunchKernelGGL(k_idx_walk, dim3(wgs), dim3(kWalkWaves * 64), kWalkLdsRingBytes, s, w);
    return hipGetLastError();
}

// Every code 16 bits: codeword i starts at start + 16 i, so the index is
// arithmetic (no walk). Same layout as k_pack_fixed16 writes.
__global__ __launch_bounds__(256) void k_idx_fixed16(uint64_t start, uint64_t nsym, uint64_t nblocks,
                                                     unsigned long long* index) {
    unsigned long long* sub = index + index_sub_offset(nblocks);
    const uint64_t nl = nblocks * kWave;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nl; j += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t blk = j / kWave;
        const uint32_t lane = (uint32_t)(j % kWave);
        const uint64_t left = nsym - blk * kBlockSyms;
        const uint32_t cnt = (uint32_t)(left < (uint64_t)kBlockSyms ? left : (uint64_t)kBlockSyms);
        uint64_t v = 0;
#pragma unroll
        for (int c = 0; c < kChainsPerLane; ++c) {
            const uint32_t at = kSPT * lane + kChainSyms * c;
            v |= (uint64_t)(((uint32_t)(start + blk * kBlockSyms * 16) + 16 * (at < cnt ? at : cnt)) & 0xffffu)
                 << (16 * c);
        }
        sub[j] = v;
        if (lane == 0) index[blk] = start + blk * kBlockSyms * 16;
        if (j == 0) {
            index[nblocks] = start + 16 * nsym;
            index[nblocks + 1] = 16ull * (nsym < (uint64_t)kBlockSyms ? nsym : (uint64_t)kBlockSyms);
        }
    }
}

hipError_t launch_index_build(const Tables& t, const uint8_t* d_payload, uint64_t payload_bytes, uint64_t start_bit,
                              uint64_t nsym, unsigned long long* d_index, unsigned long long* d_scratch, uint32_t* d_err,
                              uint32_t* h_scratch, int ncu, hipStream_t s) {
    if (nsym == 0) return hipSuccess;
    DecArgs a;
    fill_dec_args(a, t, d_payload, payload_bytes, nsym);
    a.starts = nullptr; a.subs = nullptr; a.out = nullptr; a.err = d_err;
    const uint64_t bits = payload_bytes * 8 > start_bit ? payload_bytes * 8 - start_bit : 0;
    SyncArgs y;
    y.start = start_bit;
    y.nseg = (bits + kSegBits - 1) / kSegBits;
    if (y.nseg == 0) return hipErrorInvalidValue;
    unsigned long long* p = d_scratch;
    y.ent = p; p += y.nseg;
    y.cnt = p; p += y.nseg;
    unsigned long long* first = p; p += y.nseg;
    p += ((128 - (reinterpret_cast<uintptr_t>(p) & 127)) & 127) / 8;  // 128-byte aligned bitmap (run stores)
    y.bmp = reinterpret_cast<uint32_t*>(p); p += y.nseg * (kBmpWords / 2);
    y.dirty[0] = reinterpret_cast<uint32_t*>(p);
    y.dirty[1] = y.dirty[0] + y.nseg;
    p += y.nseg;
    y.changed = reinterpret_cast<uint32_t*>(p); p += 1;
    unsigned long long* tiles = p;
    if (t.dec_mode == DEC_FIXED16) {
        uint64_t w = (a.nblocks * kWave + 255) / 256;
        w = w < (uint64_t)ncu * 8 ? (w ? w : 1) : (uint64_t)ncu * 8;
        hipLaunchKernelGGL(k_idx_fixed16, dim3(w), dim3(256), 0, s, start_bit, nsym, a.nblocks, d_index);
        return hipGetLastError();
    }
    const uint32_t lds = t.dec_lds_bytes;
    hipError_t e = hipMemsetAsync(y.dirty[0], 0, 4 * y.nseg, s);  // the scan marks the segments to check
    if (e != hipSuccess) return e;
    const bool walk = t.walk_lds_bytes > 0 && a.nwords >= 4;
    if (walk) e = scan_walk(t, a, y, ncu, s);
    else if (t.dec_mode == DEC_DENSE) e = scan_lut<DEC_DENSE>(a, y, lds, ncu, s);
    else e = scan_lut<DEC_LUT>(a, y, lds, ncu, s);
    if (e != hipSuccess) return e;
    if (t.dec_mode == DEC_DENSE) return finish_index<DEC_DENSE>(a, y, first, tiles, d_index, h_scratch, lds, ncu, s);
    return finish_index<DEC_LUT>(a, y, first, tiles, d_index, h_scratch, lds, ncu, s);
}

// ===========================================================================
// Index-less decode in CHAIN BLOCKS: the `extract` path of a reference file
// (Decompressor.cu:259-291 decodes it serially; the format carries no index,
// Compressor.cu:427-601). Stream-ordered end to end (no host synchronisation):
//   k_chain_walk    : one walk CHAIN per lane over cbits payload bits (lengths
//                     only: k_idx_walk's 4-bit table, payload ring, escape
//                     parking), starting kWalkLead bits early so it has
//                     resynchronised by its first bit. From its ENTRY (the first
//                     codeword start at or after the chain's first bit) it
//                     records the stream bit of every 8th codeword (u16 low
//                     bits, the block index's sub[] format) and of every 2048th
//                     (u64 checkpoint: a decode BLOCK of 256 records); per chain
//                     its EXIT (the first codeword start at or after its end)
//                     and codeword count
//   k_chain_fix     : a chain whose entry disagrees with the previous chain's
//                     exit walks the true path from that exit until it lands on
//                     one of its own records: the codewords before it are the
//                     chain's HEAD (decoded serially by k_chain_tail), the
//                     records from it on are valid. One grid pass, then one
//                     workgroup iterating on the chains whose exit moved
//                     (rare: the lead-in resynchronises with P ~ 1 - 4e-4)
//   k_scan_*        : output index of every chain, first decode block of every chain
//   k_chain_meta    : block descriptors (start, end, records, output index)
//   k_chain_decode  : k_decode's pipelined block decoder (two blocks per wave,
//                     quad walks, hot heads, gathers consumed a quad later) over
//                     the chain blocks, each written at its chain's output index
//   k_chain_tail    : heads, records past a chain's capacity, the end bit
// Records are chain-phased: every piece but a chain's last decodes exactly 8
// codewords, so the decoder has no partial pieces at segment ends.
// ===========================================================================
constexpr int kChainWalkWaves = 16;
constexpr uint32_t kChainRecs = 256;  // records per decode block (2048 codewords)
// Per-lane payload ring of k_chain_walk: 4 chunks of 4 words, then a copy of word 0 (so the window's two
// words q, q + 1 never wrap).
constexpr uint32_t kSegRing = 16 + 1;
// Ring word j of lane t at LDS word j * kRingRow + t: all of a lane's words lie in bank t mod 32, so the
// window's two words (one ds_read2st64_b32) and the chunk stores never conflict between lanes (a ring
// per lane at an odd stride: random banks, 12.43 vs 12.10 ms at 16 GiB Zipf, A/B in one run).
constexpr uint32_t kRingRow = kChainWalkWaves * 64;

struct ChainBlk {
    unsigned long long b0, b1;  // stream bits of the block's first record and of the one after its last
    unsigned long long rec;     // index of the block's first record in ChainArgs::rec
    long long out;              // output index of the block's first record's first symbol
    uint32_t lo, hi;            // valid records [lo, hi) of the block
    uint32_t last;              // symbols of record hi - 1 (8 unless it is the chain's last codewords)
    uint32_t lhl;               // lo | hi << 9 | last << 18: one SGPR per block in the block decoder
};
static_assert(sizeof(ChainBlk) == 48, "ChainBlk");

struct ChainArgs {
    uint64_t nchains, cbits;         // chain c walks payload bits [pbeg + c cbits, min(pbeg + (c + 1) cbits, pend))
    uint64_t pbeg, pend;             // the part of the payload (bits after start) these chains cover
    uint64_t start;                  // stream bit of the first symbol
    uint64_t entry0;                 // true entry of chain 0 (~0: its walked entry -- the stream's start)
    uint32_t bpc, cap;               // decode blocks per chain, records per chain (kChainRecs * bpc)
    uint16_t* rec;                   // [nchains][cap] low 16 bits of the stream bit of chain codeword 8 r
    unsigned long long* ckpt;        // [nchains][bpc + 1] stream bit of record 256 j; after the last block, the exit
    unsigned long long* ent;         // [nchains] walked entry
    unsigned long long* xit;         // [nchains] walked exit (first codeword start >= the chain's end)
    unsigned long long* txit;        // [nchains] true exit (k_chain_fix): the next chain's true entry
    unsigned long long* cnt;         // [nchains] codewords from the walked entry to the exit
    unsigned long long* tcnt;        // [nchains] codewords of the chain on the true path
    unsigned long long* nblk;        // [nchains] decode blocks of the chain
    unsigned long long* first;       // [nchains] output index of the chain's first true codeword
    unsigned long long* bbase;       // [nchains] the chain's first decode block
    uint32_t* hd;                    // [nchains] head: true codewords before the first valid record
    uint32_t* r0;                    // [nchains] first valid record (nrec: none)
    uint32_t* list[2];               // k_chain_fix_loop: chains to check, ping-pong
    uint32_t* lcnt;                  // [2] their counts
    ChainBlk* blk;                   // [nchains * bpc] decode block descriptors
    unsigned long long* info;        // [0] decode blocks, [1] largest block (bits), [2] end bit, [3] codewords,
                                     // [4] true exit of the last chain, [5] entry of chain 0 in use
    uint32_t* err;
};

// The ring holds its 16 words in DESCENDING order: ring word u (bit 32 u .. 32 u + 31 of the ring) at
// index 15 - (u & 15), plus index 16 = a copy of index 0, so a window's two words are adjacent
// (ds_read2_b32) and never wrap. The walk keeps its position as m = kRingM0 - p (decreasing): then the
// pair's lower index is (m >> 5) & 15 and the funnel shift is m itself (kRingM0 = 0 mod 512; m's low 5
// bits are 31 - ((p - 1) & 31)): two VALU for the address, none for the shift.
constexpr uint32_t kRingM0 = 0x7fffffe0u;
HZ_DEV uint32_t seg_window(const uint32_t* ring, uint32_t m) {
    uint32_t i;
    asm("v_bfe_u32 %0, %1, 5, 4" : "=v"(i) : "v"(m));  // (kept whole: the compiler's shift + and + add is one more)
    const uint32_t* w = ring + i * kRingRow;
    return __builtin_amdgcn_alignbit(w[kRingRow], w[0], m);
}

// Chunk slot q of a ring (ring words 4 q .. 4 q + 3), byte-swapped, descending; slot 3's last word
// (index 0) also at index 16.
HZ_DEV void seg_ring_put(uint32_t* ring, uint32_t q, const uint4& x) {
    const uint32_t v[4] = {bswap32(x.x), bswap32(x.y), bswap32(x.z), bswap32(x.w)};
#pragma unroll
    for (int i = 0; i < 4; ++i) ring[(15 - 4 * q - i) * kRingRow] = v[i];
    if (q == 3) ring[16 * kRingRow] = v[3];
}

// The ring's loader state: the next chunk f and the 64-byte register group it comes from.
struct SegFeed {
    uint4 pre[kWalkGroup];
    bool gin;
    uint64_t bch;  // payload chunk of ring chunk 0
    uint32_t f;    // next chunk to put (chunks below f are in the ring)
};

// Chunks 0..2 of a ring whose bit 0 is payload word 4 * bch, and the group holding chunk 3.
HZ_DEV void seg_feed_init(const WalkArgs& a, uint32_t* ring, SegFeed& fd, uint64_t bch) {
    constexpr uint32_t G = kWalkGroup;
    fd.bch = bch;
    uint4 v[3];
#pragma unroll
    for (int g = 0; g < 3; ++g) v[g] = walk_load(a, 4 * (bch + g));
    const uint64_t gb = (bch + 3) & ~(uint64_t)(G - 1);
    fd.gin = 4 * (gb + G) <= a.nwords && gb < a.nwords;
#pragma unroll
    for (uint32_t g = 0; g < G; ++g) fd.pre[g] = walk_load(a, 4 * (gb + g));
#pragma unroll
    for (int g = 0; g < 3; ++g) seg_ring_put(ring, (uint32_t)g, walk_fix(a, 4 * (bch + g), v[g]));
    fd.f = 3;
}

// Once per round: chunk f goes into the ring when the chain at p no longer needs chunk f - 4; the
// next group is loaded once the current one is in the ring.
HZ_DEV void seg_feed(const WalkArgs& a, uint32_t* ring, SegFeed& fd, uint32_t p) {
    constexpr uint32_t G = kWalkGroup;
    bool ld = false;
    if (fd.f <= ((p - 1) >> 7) + 3) {
        const uint64_t q = fd.bch + fd.f;
        uint4 x = pick_group<G>(fd.pre, (uint32_t)q & (G - 1));
        if (!fd.gin) x = walk_fix(a, 4 * q, x);
        seg_ring_put(ring, fd.f & 3, x);
        ++fd.f;
        ld = ((q + 1) & (G - 1)) == 0;
    }
    if (ld) {
        const uint64_t q = fd.bch + fd.f;
        fd.gin = 4 * (q + G) <= a.nwords;
        if (fd.gin) {
            const uint4* src = reinterpret_cast<const uint4*>(a.words) + q;
#pragma unroll
            for (uint32_t i = 0; i < G; ++i) fd.pre[i] = src[i];
        } else {
#pragma unroll
            for (uint32_t i = 0; i < G; ++i) fd.pre[i] = walk_load(a, 4 * (q + i));
        }
    }
}

// Steps per round of the walk: two halves of 7 steps, so a half-round (plus its escape gather) moves
// at most 8 codewords and takes at most one record. (Segment walk, 16 GiB Zipf, round 4: 10 / 12 / 14
// steps 14.4 / 13.9 / 13.4 ms; 3 parts of 6 steps 14.4 ms; a second chunk fed per round 15.2 ms.)
constexpr int kSegSteps = 14;
static_assert(kSegSteps / kWalkHalves + 1 <= 8, "one record per half-round");

// Length of the code at view bit P through the decode LUT in global memory (k_chain_walk<DEEP>: codes
// longer than the escape table's m bits; rare, never on the path of codebooks within m bits).
HZ_DEV uint32_t deep_len(const WalkArgs& a, uint64_t P) {
    const uint64_t w = P >> 5;
    const uint32_t sh = (uint32_t)(P & 31);
    const uint32_t w0 = w < a.nwords ? bswap32(a.words[w]) : 0u;
    const uint32_t w1 = w + 1 < a.nwords ? bswap32(a.words[w + 1]) : 0u;
    const uint32_t w2 = w + 2 < a.nwords ? bswap32(a.words[w + 2]) : 0u;
    const uint64_t win = ((((uint64_t)w0 << 32) | w1) << sh) | (sh ? ((uint64_t)w2 << sh) >> 32 : 0ull);
    uint32_t e = a.lut1[(uint32_t)(win >> (64 - a.lutk))];
    uint32_t D = (uint32_t)a.lutk;
    while (!(e >> 31)) {
        const uint32_t nb = (e >> 5) & 15u;
        const uint32_t idx = (e >> 10) + (uint32_t)((win << D) >> (64 - nb));
        e = idx < kLutGlobal ? a.lut1[idx] : a.lut2[idx - kLutGlobal];
        D += nb;
    }
    return lut_leaf_len(e);
}

template <bool DEEP>
__global__ __launch_bounds__(kChainWalkWaves * 64) void k_chain_walk(WalkArgs a, ChainArgs y) {
    // the byte length table (build_walk8: 2^16 windows at most, 64 KiB) at LDS address 0, the rings and
    // record buffers after it (+ one zero word: the byte a lane past its limit reads)
    __shared__ __attribute__((aligned(16))) uint32_t wtab[(1u << 16) / 4 + 4];
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    if (threadIdx.x == 0) wtab[(1u << 16) / 4] = 0;
    copy_lds_table(wtab, a.w8_img, a.w8_words);
    const uint8_t* lds8 = reinterpret_cast<const uint8_t*>(wtab);
    const uint32_t k8 = (uint32_t)a.k8;
    uint32_t* ring = lds + threadIdx.x;
    uint16_t* rbuf = reinterpret_cast<uint16_t*>(lds + kSegRing * kRingRow) + 8 * threadIdx.x;
    const uint64_t ch = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = ch < y.nchains;
    const uint64_t chc = live ? ch : 0;
    const uint64_t cs = y.pbeg + chc * y.cbits;
    const uint64_t ce = cs + y.cbits < y.pend ? cs + y.cbits : y.pend;
    const uint64_t x0 = cs - (cs < a.lead ? cs : a.lead);  // lead-in: resynchronised by cs (mostly)
    const uint64_t P0 = y.start + a.bit_adj + x0;
    SegFeed fd;
    seg_feed_init(a, ring, fd, (P0 >> 7) - 1);  // one chunk before the walk (wraps to ~0 at the payload's start: zeros)
    uint32_t p = (uint32_t)(P0 - 128 * fd.bch);    // ring bit position of the walk (>= 128)
    const uint64_t abs0 = y.start + x0 - p;        // absolute stream bit of ring position q: abs0 + q
    const uint32_t end = live ? p + (uint32_t)(ce - x0) : p;
    const uint32_t csr = p + (uint32_t)(cs - x0);  // the chain's first bit
    uint16_t* recp = y.rec + chc * y.cap;
    unsigned long long* ckp = y.ckpt + chc * (y.bpc + 1);
    uint32_t rj = 0;  // records so far (record r = chain codeword 8 r)
    uint32_t cc = 0;  // codewords since the entry
    // record r: the codeword's stream bit, low 16 bits, into the lane's 16-byte LDS buffer (stored 8 at
    // a time); every 256th also as a u64 checkpoint (a decode block's start). Past the capacity
    // nothing is stored (k_chain_tail decodes those codewords).
    // (the buffer write needs no capacity test: rows past the capacity are never stored)
    auto rec_put = [&](uint32_t rp) {
        const uint64_t ab = abs0 + rp;
        rbuf[rj & 7] = (uint16_t)ab;
        const bool in = rj < y.cap;
        const bool row = in & ((rj & 7) == 7);
        const bool ck = (in & ((rj & (kChainRecs - 1)) == 0)) | (rj == y.cap);  // at the capacity: the first codeword past it
        if (row | ck) {  // one branch for both rare stores
            if (row) *reinterpret_cast<uint4*>(recp + (rj & ~7u)) = *reinterpret_cast<const uint4*>(rbuf);
            if (ck) ckp[in ? rj / kChainRecs : y.bpc] = ab;
        }
        ++rj;
    };
    bool on = p >= csr;  // past the lead-in: counting from the entry
    uint32_t ent = p;
    if (on && p < end) rec_put(p);
    uint32_t m = kRingM0 - p;  // the walk's position, descending (seg_window)
    const uint32_t mend = kRingM0 - end;
    for (;;) {
        if (!__any(m > mend)) break;
        const uint32_t fill = 128 * fd.f - 96;  // filled data: both window words lie below p + 64
        const uint32_t mlim = kRingM0 - min(on ? end : csr, fill);  // a step needs m > mlim
#pragma unroll
        for (int half = 0; half < kWalkHalves; ++half) {
            // the half's codewords end at q[0 .. na - 1] (the advancing steps are a prefix: a chain
            // that parks or reaches its limit stays put for the rest of the half), then at m for an escape
            // A step reads the code's length (0: an escape), or, past the limit, the zero byte after the
            // table: a chain that reads 0 stays put and reads 0 again, so the advancing steps are a prefix
            // with no park flags, and an escape's window is the half's last (no lane masks and no SALU
            // per step: 281 vs 330 clocks per step in tools/microbench/mb_walk_step.hip).
            constexpr int S = kSegSteps / kWalkHalves;
            uint32_t q[S];
            uint32_t na = 0, W = 0, e = 0;
            bool ok = false;
            // issue priority over the dependent steps and the escape gather's issue, normal for the
            // record select, feed and stores (extract 21.14-21.45 -> 20.48-20.62 ms, A/B)
            __builtin_amdgcn_s_setprio(2);
#pragma unroll
            for (int t = 0; t < S; ++t) {
                ok = m > mlim;
                W = seg_window(ring, m);
                e = lds8[ok ? W >> (32 - k8) : 1u << 16];
                HZ_WALK_FENCE();
                m -= e;
                na += e != 0u ? 1u : 0u;
                q[t] = m;
            }
            const bool pk = ok & (e == 0u);  // parked on an escape
            const uint32_t nm = na + (pk ? 1u : 0u);
            // the escape's gather by every lane (the others read byte 0): no branch, and its wait sits at
            // the first use, behind the record select (11.2 vs 11.5 ms, A/B in one run)
            uint32_t ev = a.esc[pk ? W >> (32 - a.m) : 0u];
            __builtin_amdgcn_s_setprio(0);
            // record of codeword 8 i: it starts where the half's codeword j1 ends (1-based): q[j1 - 1],
            // or m after the escape when j1 is the escaped codeword (jj = 0); a three-level select
            const uint32_t j1 = 8u - (cc & 7u);
            const uint32_t jj = j1 <= na ? j1 : 0u;
            static_assert(S <= 7, "q[jj - 1] for jj < 8");
            uint32_t v[8];
            v[0] = 0;
#pragma unroll
            for (int t = 0; t < 7; ++t) v[t + 1] = t < S ? q[t < S ? t : 0] : 0u;
            const bool b0 = jj & 1u, b1 = jj & 2u, b2 = jj & 4u;
            const uint32_t a0 = b0 ? v[1] : v[0], a1 = b0 ? v[3] : v[2], a2 = b0 ? v[5] : v[4], a3 = b0 ? v[7] : v[6];
            const uint32_t sel = b2 ? (b1 ? a3 : a2) : (b1 ? a1 : a0);
            if constexpr (DEEP) {  // the escape table holds 0: a code longer than its m bits (decode LUT)
                const bool deep = pk & (ev == 0u);
                if (__any(deep)) {
                    if (deep) ev = deep_len(a, abs0 + (kRingM0 - m) + a.bit_adj);
                }
            }
            m -= pk ? ev : 0u;
            // the round's feed right after its last escape wait and before the half's record stores: its
            // wait on the group registers then waits for no fresh store (12.23 vs 12.60 ms at the round's
            // end, 16 GiB Zipf, A/B in one run; without the record stores 11.67 ms)
            if (half == kWalkHalves - 1) seg_feed(a, ring, fd, kRingM0 - m);
            const uint32_t pc = kRingM0 - m;
            const uint32_t rm = jj ? sel : m;
            // the lead-in's last step lands on the entry: the entry is the record, counting starts there
            const bool enter = !on & (pc >= csr);
            const uint32_t rp = on ? kRingM0 - rm : pc;
            const bool rec = (on ? j1 <= nm : enter) & (rp < end);  // (a codeword starting at the end is the next chain's)
            ent = enter ? pc : ent;
            cc = on ? cc + nm : 0u;
            on |= enter;
            if (rec) rec_put(rp);
        }
    }
    p = kRingM0 - m;
    if (!live) return;
    if ((rj & 7u) && (rj & ~7u) < y.cap)  // the last, partial group of records
        *reinterpret_cast<uint4*>(recp + (rj & ~7u)) = *reinterpret_cast<const uint4*>(rbuf);
    if (rj <= y.cap) ckp[(rj + kChainRecs - 1) / kChainRecs] = abs0 + p;  // after the last block: the exit
    y.ent[ch] = abs0 + (on ? ent : p);
    y.xit[ch] = abs0 + p;
    y.txit[ch] = abs0 + p;
    y.cnt[ch] = cc;
}

// Stream bit of record r (< cap) of chain c.
HZ_DEV uint64_t chain_rec_pos(const ChainArgs& y, uint64_t c, uint32_t r) {
    const uint64_t ck = y.ckpt[c * (y.bpc + 1) + r / kChainRecs];
    return ck + (uint16_t)(y.rec[c * y.cap + r] - (uint16_t)ck);
}

HZ_DEV uint32_t chain_nrec(uint64_t n) { return (uint32_t)((n + 7) / 8); }
HZ_DEV uint64_t chain_blocks(uint32_t navail, uint32_t r0) {
    const uint32_t nb = (navail + kChainRecs - 1) / kChainRecs, j0 = r0 / kChainRecs;
    return r0 < navail ? nb - j0 : 0;
}

// Chain i against chain i - 1's true exit (its true entry; chain 0: entry0). When that is not the walked entry,
// walk the true path until it lands on one of the chain's records (from there both paths agree):
// head, first valid record, true count and decode blocks follow. The chain's true exit is its walked
// exit when a record was met, else where the true path left the chain (the whole chain is head).
// Returns true when the true exit changed (the next chain must be checked again). Idempotent: a chain
// checked against a stale entry (another chain's exit moving concurrently) is checked again.
template <int MODE>
HZ_DEV bool chain_fix_one(const DecArgs& a, const ChainArgs& y, const uint32_t* lds, uint64_t i) {
    uint64_t p = i ? y.txit[i - 1] : y.entry0;
    const uint64_t n = y.cnt[i];
    const uint32_t nrec = chain_nrec(n), navail = nrec < y.cap ? nrec : y.cap;
    uint32_t rr = 0;
    uint64_t h = 0;
    bool met = p == y.ent[i];
    if (!met) {
        const uint64_t cend = y.pbeg + (i + 1) * y.cbits;
        const uint64_t ce = y.start + (cend < y.pend ? cend : y.pend);
        BitReader r;
        br_init(r, a, p + a.bit_adj);
        uint64_t R = navail ? chain_rec_pos(y, i, 0) : ~0ull;
        for (;;) {
            while (rr < navail && R < p) {
                ++rr;
                R = rr < navail ? chain_rec_pos(y, i, rr) : ~0ull;
            }
            if (rr < navail && R == p) { met = true; break; }
            if (p >= ce) break;
            uint32_t sym;
            const uint32_t L = br_next<MODE>(r, a, lds, sym);
            if (L == 0) { atomicOr(a.err, 2u); break; }
            p += L;
            ++h;
        }
    }
    y.hd[i] = (uint32_t)h;
    y.r0[i] = met ? rr : nrec;
    y.tcnt[i] = met ? h + n - 8ull * rr : h;
    y.nblk[i] = met ? chain_blocks(navail, rr) : 0;
    const uint64_t tx = met ? y.xit[i] : p;
    if (tx != y.txit[i]) {
        y.txit[i] = tx;
        return true;
    }
    return false;
}

// Every chain once (chain 0 starts on its walked entry unless entry0 says otherwise); chains whose
// predecessor's exit moved go on a list.
template <int MODE>
__global__ __launch_bounds__(kSyncThreads) void k_chain_fix(DecArgs a, ChainArgs y) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    copy_lds_table(lds, a.lds_img, a.lds_words);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < y.nchains; i += stride) {
        if (i == 0 && y.entry0 == ~0ull) {
            const uint64_t n = y.cnt[0];
            const uint32_t nrec = chain_nrec(n);
            y.hd[0] = 0;
            y.r0[0] = 0;
            y.tcnt[0] = n;
            y.nblk[0] = chain_blocks(nrec < y.cap ? nrec : y.cap, 0);
            y.txit[0] = y.xit[0];
            continue;
        }
        if (chain_fix_one<MODE>(a, y, lds, i) && i + 1 < y.nchains) {
            const uint32_t s = atomicAdd(y.lcnt, 1u);
            y.list[0][s] = (uint32_t)(i + 1);
        }
    }
}

// The listed chains again, one workgroup, until no exit moves: each pass moves the frontier of a run
// of unsynchronised chains by one chain (bounded by nchains passes).
template <int MODE>
__global__ __launch_bounds__(kSyncThreads) void k_chain_fix_loop(DecArgs a, ChainArgs y) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    copy_lds_table(lds, a.lds_img, a.lds_words);
    for (uint64_t it = 0; it <= y.nchains; ++it) {
        const uint32_t cur = (uint32_t)(it & 1);
        const uint32_t n = __hip_atomic_load(y.lcnt + cur, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (n == 0) break;  // every thread read the same count (the adds happened before the barrier)
        for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) {
            const uint64_t i = y.list[cur][j];
            if (chain_fix_one<MODE>(a, y, lds, i) && i + 1 < y.nchains) {
                const uint32_t s = atomicAdd(y.lcnt + (cur ^ 1u), 1u);
                y.list[cur ^ 1u][s] = (uint32_t)(i + 1);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(y.lcnt + cur, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
    }
}

// Decode block descriptors of every chain (after the scans of tcnt -> first and nblk -> bbase), the
// largest block and the number of blocks.
__global__ __launch_bounds__(256) void k_chain_meta(ChainArgs y) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t maxb = 0;
    if (c < y.nchains) {
        const uint64_t nb = y.nblk[c];
        if (c + 1 == y.nchains) {  // the part's summary
            y.info[0] = y.bbase[c] + nb;
            y.info[3] = y.first[c] + y.tcnt[c];
            y.info[4] = y.txit[c];
            y.info[5] = y.entry0 != ~0ull ? y.entry0 : y.ent[0];  // the entry in use
        }
        if (nb) {
            const uint64_t n = y.cnt[c];
            const uint32_t nrec = chain_nrec(n), navail = nrec < y.cap ? nrec : y.cap;
            const uint32_t r0 = y.r0[c], j0 = r0 / kChainRecs;
            const long long out0 = (long long)(y.first[c] + y.hd[c]) - 8ll * r0;  // output index of record 0
            const unsigned long long* ckp = y.ckpt + c * (y.bpc + 1);
            ChainBlk* bk = y.blk + y.bbase[c];
            for (uint32_t j = j0; j < j0 + (uint32_t)nb; ++j) {
                ChainBlk d;
                d.b0 = ckp[j];
                d.b1 = ckp[j + 1];
                d.rec = c * y.cap + (uint64_t)kChainRecs * j;
                d.out = out0 + 8ll * kChainRecs * j;
                d.lo = r0 > kChainRecs * j ? r0 - kChainRecs * j : 0u;
                const uint32_t hi = navail - kChainRecs * j;
                d.hi = hi < kChainRecs ? hi : kChainRecs;
                // the chain's last record (not cut by the capacity) holds n - 8 (nrec - 1) codewords
                d.last = nrec <= y.cap && kChainRecs * j + d.hi == nrec ? (uint32_t)(n - 8ull * (nrec - 1)) : 8u;
                d.lhl = d.lo | d.hi << 9 | d.last << 18;
                bk[j - j0] = d;
                maxb = d.b1 - d.b0 > maxb ? d.b1 - d.b0 : maxb;
            }
        }
    }
    // one atomic per wave
#pragma unroll
    for (int mm = 1; mm < 64; mm <<= 1) {
        const uint64_t o = ((uint64_t)shfl_xor_u32((uint32_t)(maxb >> 32), mm) << 32) | shfl_xor_u32((uint32_t)maxb, mm);
        maxb = o > maxb ? o : maxb;
    }
    if ((threadIdx.x & 63) == 0 && maxb) atomicMax(y.info + 1, (unsigned long long)maxb);
}

// Block metadata of the chain decoder, as loaded: the descriptor (scalar loads that nothing waits for
// until the next block iteration, so they never turn an LDS wait of the current one into lgkmcnt(0))
// and the lane's four record low bits (chain slots 64 k + lane), loaded a whole block iteration
// before they are used (chain_rec_load) and unconditionally: a select of the loaded values in the same
// iteration made the compiler branch around each load, splitting the block loop (k_chain_decode 10.76
// against k_decode's 9.89 ms). Records past hi read stale rows of the chain's capacity and are
// replaced by the block start in chain_meta_sub.
struct ChainMeta {
    uint64_t b0, b1, rec;
    long long out;
    uint32_t lhl;  // ChainBlk::lhl
    bool valid;    // a block of the decode (else: any block, decoded, never stored)
    uint64_t sub;  // the four record words as loaded
};

HZ_DEV void chain_meta_load(const ChainArgs& y, uint64_t b, uint64_t nb, ChainMeta& m) {
    const uint64_t bb = b < nb ? b : (nb ? nb - 1 : 0);  // past the end: any block, never stored
    // the descriptor through the scalar cache (b0, b1, rec, out, lhl)
    typedef const __attribute__((address_space(4))) unsigned long long* cu64p;
    const uint64_t bu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(bb >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)bb);
    const cu64p d = (cu64p)y.blk + 6 * bu;
    m.b0 = d[0];
    m.b1 = d[1];
    m.rec = d[2];
    m.out = (long long)d[3];
    m.lhl = (uint32_t)(d[5] >> 32);
    m.valid = b < nb;
}

// The lane's four records of a block whose descriptor has landed (one load per slot, always issued;
// y.rec holds a whole capacity of rows per chain, so rows past the block's valid ones exist).
HZ_DEV void chain_rec_load(const ChainArgs& y, int lane, ChainMeta& m) {
    const uint16_t* s16 = y.rec + m.rec + (uint32_t)lane;
    uint64_t sub = 0;
#pragma unroll
    for (int c = 0; c < kChainsPerLane; ++c) sub |= (uint64_t)s16[64 * c] << (16 * c);
    m.sub = sub;
}

HZ_DEV uint32_t chain_meta_hi(const ChainMeta& m) { return m.valid ? (m.lhl >> 9) & 0x1ffu : 0u; }

// The lane's chain starts (low 16 bits): its records below hi, else the block start.
HZ_DEV uint64_t chain_meta_sub(const ChainMeta& m, int lane) {
    const uint32_t hi = chain_meta_hi(m);
    uint64_t sub = 0;
#pragma unroll
    for (int c = 0; c < kChainsPerLane; ++c) {
        const uint32_t t = 64u * c + (uint32_t)lane;
        const uint64_t v = t < hi ? (m.sub >> (16 * c)) & 0xffffu : (uint64_t)(uint16_t)m.b0;
        sub |= v << (16 * c);
    }
    return sub;
}

// A chain block's symbols: record t = 64 c + lane of the block, 8 symbols at output index out + 8 t
// (2-byte aligned: the 16-byte stores of adjacent lanes are adjacent), the last record's and the
// stream end's symbol by symbol.
HZ_DEV void chain_store(const DecArgs& a, const ChainMeta& m, int lane, const uint32_t* pk) {
    uint16_t* out16 = reinterpret_cast<uint16_t*>(a.out);
    const uint32_t lo = m.lhl & 0x1ffu, hi = chain_meta_hi(m), last = m.lhl >> 18;
    const bool full = lo == 0 && hi == kChainRecs && last == 8 && m.out >= 0 &&
                      (uint64_t)m.out + (uint64_t)kBlockSyms <= a.nsym;
    if (full) {
        const long long ob = m.out;
#pragma unroll
        for (int c = 0; c < kChainsPerLane; ++c) {
            uint32_t* q = reinterpret_cast<uint32_t*>(out16 + ob + 8 * (64 * c + lane));
            u32x4a2 v = u32x4a2{pk[4 * c], pk[4 * c + 1], pk[4 * c + 2], pk[4 * c + 3]};
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4a2*>(q));
        }
        return;
    }
#pragma unroll
    for (int c = 0; c < kChainsPerLane; ++c) {
        const uint32_t t = 64u * c + (uint32_t)lane;
        if (t < lo || t >= hi) continue;
        const long long o = m.out + 8ll * t;
        if (o < 0 || (uint64_t)o >= a.nsym) continue;
        uint32_t cn = t + 1 == hi ? last : 8u;
        cn = a.nsym - (uint64_t)o < cn ? (uint32_t)(a.nsym - (uint64_t)o) : cn;
        if (cn == 8) {
            *reinterpret_cast<u32x4a2*>(out16 + o) = u32x4a2{pk[4 * c], pk[4 * c + 1], pk[4 * c + 2], pk[4 * c + 3]};
        } else {
            for (uint32_t q = 0; q < cn; ++q) out16[o + q] = (uint16_t)(pk[4 * c + (q >> 1)] >> (16 * (q & 1)));
        }
    }
}

// k_decode's two-blocks-per-wave pipelined walk (dec_wave_pipe2) over chain blocks b, b + 1, then
// b + stride, ...: the same staging, quad walks and deferred gathers; block metadata from the
// descriptors, output at each block's chain position.
HZ_DEV void dec_wave_chain(const DecArgs& a, const ChainArgs& y, uint64_t nb, const uint32_t* lds, uint32_t* stg,
                           uint32_t slot, uint64_t b, uint64_t stride, int lane) {
    constexpr int C = 2 * kChainsPerLane;
    const __amdgpu_buffer_rsrc_t l2r = lut_l2_rsrc(a.l2);
    ChainMeta mc[2], mn[2], mn2[2];
    uint4 sc[2][kStageUnroll], sn[2][kStageUnroll];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        chain_meta_load(y, b + j, nb, mc[j]);
        chain_meta_load(y, b + stride + j, nb, mn[j]);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) chain_rec_load(y, lane, mc[j]);
    auto as_pipe = [](const ChainMeta& m) { PipeMeta p; p.b0 = m.b0; p.b1 = m.b1; p.sub = 0; return p; };
#pragma unroll
    for (int j = 0; j < 2; ++j) dec_stage_prefetch(a, as_pipe(mc[j]), lane, sc[j]);
    for (; b < nb; b += stride) {
        // the next blocks' records, a block iteration ahead (their descriptors landed last iteration)
#pragma unroll
        for (int j = 0; j < 2; ++j) chain_rec_load(y, lane, mn[j]);
        uint32_t p1[C];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            uint64_t w0;
            dec_stage_commit<true>(a, as_pipe(mc[j]), slot >> 2, stg + j * slot, lane, sc[j], w0);
            uint32_t off[kChainsPerLane];
            dec_chain_offsets(chain_meta_sub(mc[j], lane), mc[j].b0, mc[j].b1 - mc[j].b0, lane, off);
            const uint32_t top = (uint32_t)(stg - lds) + (uint32_t)(j + 1) * slot - 1u;
            const uint32_t base = top * 32u - (uint32_t)(mc[j].b0 + a.bit_adj - (w0 << 5));
#pragma unroll
            for (int c = 0; c < kChainsPerLane; ++c) p1[j * kChainsPerLane + c] = base - off[c];
        }
        __builtin_amdgcn_wave_barrier();  // LDS ops of one wave complete in order
        uint32_t pk[2][kSPT / 2];
        PipeLane st[C];
        uint32_t g[C];
        auto finish = [&](int c, int q) {
            // a leaf in LDS (bit 31) beats its gather's 0 (read past num_records); a link loses to its
            // gathered leaf: one v_max; and the leaf's byte 3 is 0x80 | L, subtracted whole (128 bits
            // more per step, which the window address takes back: dec_pipe_ldsn's adj). 12 % fewer VALU
            // per block pair; k_decode 10.09 -> 9.97 ms, chain decode 11.30 -> 11.13 ms (A/B, 16 GiB Zipf)
            const uint32_t ee = st[c].e > g[c] ? st[c].e : g[c];
            p1[c] -= ee >> 24;
            const int i = ((c % kChainsPerLane) * kChainSyms + q) >> 1;
            if (q & 1) pk[c / kChainsPerLane][i] = __builtin_amdgcn_perm(ee, pk[c / kChainsPerLane][i], 0x06050201u);
            else pk[c / kChainsPerLane][i] = ee;
        };
        auto issue4 = [&](int c, int q) {
            // issue priority over the quad's LDS walk and gathers (decode 9.96-9.99 -> 9.88-9.91 ms, A/B)
            __builtin_amdgcn_s_setprio(2);
            dec_pipe_ldsn<4>(a, lds, p1 + c, st + c, 16u * (uint32_t)q);  // q steps taken: 16 q bytes
#pragma unroll
            for (int t = 0; t < 4; ++t)
                g[c + t] = __builtin_amdgcn_raw_buffer_load_b32(l2r, st[c + t].gi, 0, 0);
            __builtin_amdgcn_s_setprio(0);
        };
        issue4(0, 0);
#pragma unroll
        for (int q = 0; q < kChainSyms; ++q) {
            issue4(4, q);
            if (q == kPfStep) {  // the next two blocks' staging chunks, the metadata after them
#pragma unroll
                for (int j = 0; j < 2; ++j) dec_stage_prefetch(a, as_pipe(mn[j]), lane, sn[j]);
#pragma unroll
                for (int j = 0; j < 2; ++j) chain_meta_load(y, b + 2 * stride + j, nb, mn2[j]);
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) finish(c, q);
            if (q + 1 < kChainSyms) issue4(0, q + 1);
#pragma unroll
            for (int c = 4; c < 8; ++c) finish(c, q);
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < 2; ++j)
            if (b + j < nb) chain_store(a, mc[j], lane, pk[j]);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            mc[j] = mn[j];
            mn[j] = mn2[j];
#pragma unroll
            for (int u = 0; u < kStageUnroll; ++u) sc[j][u] = sn[j][u];
        }
    }
}

// Persistent: the block count and the largest block come from the device (k_chain_meta); slots are
// sized in-kernel from the largest block, waves without a slot pair idle (k_decode's rule).
__global__ __launch_bounds__(kDecPipe2Threads) void k_chain_decode(DecArgs a, ChainArgs y) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    copy_lds_table(lds, a.lds_img, a.lds_words);
    const int lane = threadIdx.x & 63;
    const uint32_t wid = wave_id();
    typedef const __attribute__((address_space(4))) unsigned long long* cu64p;
    const uint64_t nb = ((cu64p)y.info)[0];
    if (nb == 0) return;  // no chain has a block (every codeword in heads / tails)
    const uint32_t slot = (uint32_t)__builtin_amdgcn_readfirstlane((int)dec_slot_words(((cu64p)y.info)[1], a.max_len));
    const uint32_t nwave = blockDim.x >> 6;
    uint32_t nw2 = a.region_words / (2 * slot);
    nw2 = nw2 < nwave ? nw2 : nwave;
    if (nw2 == 0) {  // a block larger than the region (cannot happen: the host sizes it for 2048 x max_len)
        if (threadIdx.x == 0) atomicOr(a.err, 128u);
        return;
    }
    if (wid >= nw2) return;
    const uint64_t b = 2 * ((uint64_t)blockIdx.x * nw2 + wid), stride = 2 * (uint64_t)gridDim.x * nw2;
    dec_wave_chain(a, y, nb, lds, lds + a.lds_words + wid * 2 * slot, slot, b, stride, lane);
}

// Codebooks past the pipelined decoder's two table levels (codes longer than chain_k +
// chain_level_bits bits): every record of every block serially, one thread per record of 8 codewords,
// through br_next's multi-level lookup; the block count from the device (k_chain_meta).
__global__ __launch_bounds__(kSyncThreads) void k_chain_decode_serial(DecArgs a, ChainArgs y) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    copy_lds_table(lds, a.lds_img, a.lds_words);
    uint16_t* out16 = reinterpret_cast<uint16_t*>(a.out);
    const uint64_t nrec = y.info[0] * kChainRecs;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nrec; i += stride) {
        const ChainBlk& d = y.blk[i / kChainRecs];
        const uint32_t t = (uint32_t)(i % kChainRecs);
        if (t < d.lo || t >= d.hi) continue;
        const long long o = d.out + 8ll * t;
        const uint32_t cn = t + 1 == d.hi ? d.last : 8u;
        BitReader r;
        br_init(r, a, d.b0 + (uint16_t)(y.rec[d.rec + t] - (uint16_t)d.b0) + a.bit_adj);
        for (uint32_t q = 0; q < cn; ++q) {
            uint32_t sym;
            const uint32_t L = br_next<DEC_LUT>(r, a, lds, sym);
            if (L == 0) { atomicOr(a.err, 2u); break; }
            if (o + q >= 0 && (uint64_t)(o + q) < a.nsym) out16[o + q] = (uint16_t)sym;
        }
    }
}

// One thread per chain: its head (true codewords before its first valid record), the codewords past
// its record capacity, and the end bit of codeword nsym - 1, decoded serially (rare, short).
template <int MODE>
__global__ __launch_bounds__(kSyncThreads) void k_chain_tail(DecArgs a, ChainArgs y) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    copy_lds_table(lds, a.lds_img, a.lds_words);
    uint16_t* out16 = reinterpret_cast<uint16_t*>(a.out);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t last = a.nsym - 1;
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < y.nchains; c += stride) {
        const uint64_t F = y.first[c], T = y.tcnt[c], n = y.cnt[c];
        const uint32_t h = y.hd[c], r0 = y.r0[c], nrec = chain_nrec(n);
        const bool has_end = a.nsym > 0 && F <= last && last < F + T;
        // serial decode of k codewords from stream bit p into output index o, noting the end bit
        auto serial = [&](uint64_t p, uint64_t o, uint64_t k) {
            BitReader r;
            br_init(r, a, p + a.bit_adj);
            for (uint64_t t = 0; t < k; ++t) {
                uint32_t sym;
                const uint32_t L = br_next<MODE>(r, a, lds, sym);
                if (L == 0) { atomicOr(a.err, 2u); return; }
                p += L;
                if (o + t < a.nsym) out16[o + t] = (uint16_t)sym;
                if (o + t == last) y.info[2] = p;
            }
        };
        if (h) serial(c ? y.txit[c - 1] : y.entry0, F, h);
        if (r0 < nrec && nrec > y.cap)      // records past the capacity: the rest of the chain
            serial(y.ckpt[c * (y.bpc + 1) + y.bpc], F + h + 8ull * (y.cap - r0), n - 8ull * y.cap);
        if (has_end && last >= F + h) {     // the end bit inside a piece: walk that piece up to it
            const uint64_t q = last - (F + h);
            const uint64_t m = r0 + q / 8;
            if (m < y.cap) {
                BitReader r;
                uint64_t p = chain_rec_pos(y, c, (uint32_t)m);
                br_init(r, a, p + a.bit_adj);
                for (uint32_t t = 0; t <= (uint32_t)(q % 8); ++t) {
                    uint32_t sym;
                    const uint32_t L = br_next<MODE>(r, a, lds, sym);
                    if (L == 0) { atomicOr(a.err, 2u); break; }
                    p += L;
                }
                y.info[2] = p;
            }
        }
    }
}

// ---- host side -----------------------------------------------------------------------------
// Chain geometry of a part of the payload (bits [pbeg, pend) after start): chains of cbits bits, about
// one per walk lane of the device (16 waves per CU), but at least kChainMinBlocks decode block long;
// each chain's record capacity holds its expected records with 25 % headroom (more go to
// k_chain_tail, serially). avg: expected payload bits per codeword (the lower of the payload's own
// and the codebook's Kraft estimate: more records, more headroom).
// (one: a part of ~2 Gbit -- the CLI's 256 MiB payload windows -- gets 90 K chains instead of 23 K, so
// the walk is not occupancy-starved: 1.85 -> 0.96 ms per window call, 1 GiB 2.50 -> 1.93 ms; 2 blocks:
// 1.21 / 1.94 ms; long parts are lane-limited and unaffected)
constexpr uint64_t kChainMinBlocks = 1;
struct ChainGeom {
    uint64_t nchains = 0, cbits = 0, pbeg = 0, pend = 0;
    uint32_t bpc = 0, cap = 0;
    uint64_t off_rec, off_ckpt, off_arr, off_u32, off_list, off_info, off_tiles, off_blk, words;
};

static ChainGeom chain_geom(uint64_t pbeg, uint64_t pend, double avg, int ncu) {
    ChainGeom g;
    g.pbeg = pbeg;
    g.pend = pend;
    const uint64_t bits = pend > pbeg ? pend - pbeg : 0;
    if (bits == 0) return g;
    if (!(avg >= 1.0)) avg = 1.0;
    const uint64_t lanes = (uint64_t)kChainWalkWaves * 64 * (uint64_t)(ncu > 0 ? ncu : 1);
    const uint64_t minbits = (uint64_t)(kChainMinBlocks * kBlockSyms * avg);
    uint64_t cb = (bits + lanes - 1) / lanes;
    cb = cb > minbits ? cb : minbits;
    cb = (cb + 127) & ~127ull;
    g.cbits = cb;
    g.nchains = (bits + cb - 1) / cb;
    const double recs = (double)cb / avg / 8.0 * 1.25 + 64.0;
    g.bpc = (uint32_t)((recs + kChainRecs - 1) / kChainRecs);
    g.cap = g.bpc * kChainRecs;
    const uint64_t nc = g.nchains;
    const uint64_t ntiles = (nc + kScanTile - 1) / kScanTile;
    uint64_t w = 0;
    g.off_rec = w;   w += (nc * g.cap * 2 + 15) / 16 * 2;       // u16 records (16-byte rows)
    g.off_ckpt = w;  w += nc * (g.bpc + 1);                     // u64 checkpoints
    g.off_arr = w;   w += 8 * nc;                               // ent, xit, txit, cnt, tcnt, nblk, first, bbase
    g.off_u32 = w;   w += nc;                                   // hd, r0 (u32)
    g.off_list = w;  w += nc + 1;                               // list[2] (u32), lcnt
    g.off_info = w;  w += 8;
    g.off_tiles = w; w += ntiles + 2;
    g.off_blk = w;   w += nc * g.bpc * (sizeof(ChainBlk) / 8);
    g.words = w + 8;
    return g;
}

static double chain_avg(const Tables& t, uint64_t bits, uint64_t nsym) {
    double avg = nsym ? (double)bits / (double)nsym : t.dec_avg_bits;
    if (t.dec_avg_bits > 0.5 && t.dec_avg_bits < avg) avg = t.dec_avg_bits;
    return avg;
}

uint64_t chain_scratch_words(uint64_t part_begin, uint64_t part_end, uint64_t nsym, const Tables& t, int ncu) {
    return chain_geom(part_begin, part_end, chain_avg(t, part_end > part_begin ? part_end - part_begin : 0, nsym), ncu)
        .words;
}

bool seg_decode_supported(const Tables& t) {
    return t.dec_mode >= 0 && t.dec_mode != DEC_FIXED16 && t.chain_lds_bytes > 0 && t.walk8_bytes > 0 &&
           t.chain_esc != nullptr;
}

// Codes the pipelined chain decoder resolves (an LDS level, then one global level); longer codebooks
// decode their records serially (k_chain_decode_serial).
static bool chain_pipelined(const Tables& t) { return t.dec_max_len <= t.chain_k + t.chain_level_bits; }

// The decoder arguments of the chain phases: the chain's LUT images (the decode tables' for a LUT
// codebook, the LUT built beside a DENSE one).
static void fill_chain_dec_args(DecArgs& d, const Tables& t, const uint8_t* d_payload, uint64_t payload_bytes,
                                uint64_t nsym) {
    fill_dec_args(d, t, d_payload, payload_bytes, nsym);
    d.lds_img = t.chain_lds;
    d.lds_words = t.chain_lds_bytes / 4;
    d.k = t.chain_k;
    d.level_bits = t.chain_level_bits;
    d.l2 = t.chain_l2;
}

// Payloads under 16 bytes (the walk's 16-byte loads need at least 4 words): one thread decodes the
// codewords serially from start_bit, as Decompressor.cu:259-291 does, stream-ordered; a payload with
// fewer than nsym codewords reports the end bit UINT64_MAX.
__global__ __launch_bounds__(64) void k_decode_tiny(DecArgs a, uint64_t start, uint64_t payload_bits,
                                                    unsigned long long* end) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    copy_lds_table(lds, a.lds_img, a.lds_words);
    if (threadIdx.x) return;
    uint16_t* out16 = reinterpret_cast<uint16_t*>(a.out);
    BitReader r;
    br_init(r, a, start + a.bit_adj);
    uint64_t p = start, i = 0;
    for (; i < a.nsym && p <= payload_bits; ++i) {  // (every code >= 1 bit: at most 128 steps)
        uint32_t sym;
        const uint32_t L = br_next<DEC_LUT>(r, a, lds, sym);
        if (L == 0) { atomicOr(a.err, 2u); break; }
        p += L;
        if (p <= payload_bits) out16[i] = (uint16_t)sym;
    }
    if (end) *end = i == a.nsym && p <= payload_bits ? p : ~0ull;
}

hipError_t chain_decode_tiny(const Tables& t, const uint8_t* d_payload, uint64_t payload_bytes, uint64_t start_bit,
                             uint64_t nsym, uint8_t* d_out, unsigned long long* d_end, uint32_t* d_err, hipStream_t s) {
    if (!seg_decode_supported(t)) return hipErrorInvalidValue;
    DecArgs d;
    fill_chain_dec_args(d, t, d_payload, payload_bytes, nsym);
    d.starts = nullptr; d.subs = nullptr; d.out = d_out; d.err = d_err;
    hipError_t e = ensure_lds_limit((const void*)k_decode_tiny, kLdsBytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_decode_tiny, dim3(1), dim3(64), t.chain_lds_bytes, s, d, start_bit, payload_bytes * 8, d_end);
    return hipGetLastError();
}

// HZ_CAPTURE_DEBUG=1 (debug): the stream's capture status after each step of the launchers.
static void cap_check(hipStream_t s, const char* tag) {
    static const bool on = getenv("HZ_CAPTURE_DEBUG") != nullptr;
    if (!on) return;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    const hipError_t e = hipStreamGetCaptureInfo(s, &st, &id);
    fprintf(stderr, "[hz capture] %-12s status %d (err %d)\n", tag, (int)st, (int)e);
}

static hipError_t scan_u64(const unsigned long long* v, uint64_t n, unsigned long long* tiles, unsigned long long* out,
                           hipStream_t s) {
    const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(k_scan_reduce, dim3(ntiles), dim3(kScanThreads), 0, s, v, n, tiles, ~0ull);
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kScanThreads), 0, s, tiles, ntiles, 0ull);
    hipLaunchKernelGGL(k_scan_apply, dim3(ntiles), dim3(kScanThreads), 0, s, v, n, (const unsigned long long*)tiles,
                       out, ~0ull);
    return hipGetLastError();
}

// The state a chain decode keeps between its phases (scan, refix, decode): geometry, kernel arguments
// (device pointers into the context's scratch and tables), the part's summary in y.info.
struct ChainState {
    ChainGeom g;
    ChainArgs y;
    DecArgs d;
    WalkArgs w;
    unsigned long long* tiles = nullptr;  // scan scratch
    uint64_t base = 0;                     // stream bit of byte 0 of the payload view (hz_indexless_scan)
    bool valid = false;
};
ChainState* chain_state_create() { return new ChainState(); }
void chain_state_destroy(ChainState* st) { delete st; }
const unsigned long long* chain_info(const ChainState* st) { return st->valid ? st->y.info : nullptr; }
void chain_invalidate(ChainState* st) { st->valid = false; }

// The part's summary in stream bits: codewords, true exit, entry in use (view bits + base).
__global__ void k_chain_summary(const unsigned long long* info, unsigned long long* dst, uint64_t base) {
    if (threadIdx.x == 0) {
        dst[0] = info[3];
        dst[1] = info[4] + base;
        dst[2] = info[5] + base;
    }
}
// The end bit in stream bits (all ones: not in this part).
__global__ void k_chain_end(const unsigned long long* info, unsigned long long* dst, uint64_t base) {
    if (threadIdx.x == 0) dst[0] = info[2] == ~0ull ? ~0ull : info[2] + base;
}
__global__ void k_put3(unsigned long long* dst, uint64_t a, uint64_t b, uint64_t c) {
    if (threadIdx.x == 0) {
        dst[0] = a;
        dst[1] = b;
        dst[2] = c;
    }
}
struct StageArgs {
    const uint8_t* src;
    StageSeg seg[kStageMaxSegs];
};
// Segment blockIdx.y of the staging buffer to its table: 16-byte vectors, then the 4-byte tail.
__global__ __launch_bounds__(256) void k_stage_scatter(StageArgs a) {
    const StageSeg g = a.seg[blockIdx.y];
    const uint4* src = reinterpret_cast<const uint4*>(a.src + g.off);
    uint4* dst = reinterpret_cast<uint4*>(g.dst);
    const uint64_t nv = g.bytes / 16;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
    if (blockIdx.x == 0 && threadIdx.x < (g.bytes % 16) / 4) {
        const uint64_t w = nv * 4 + threadIdx.x;
        reinterpret_cast<uint32_t*>(g.dst)[w] = reinterpret_cast<const uint32_t*>(a.src + g.off)[w];
    }
}

hipError_t stage_scatter(const uint8_t* h_src, const StageSeg* segs, int nseg, hipStream_t s) {
    for (int i0 = 0; i0 < nseg; i0 += kStageMaxSegs) {
        StageArgs a;
        a.src = h_src;
        const int n = nseg - i0 < kStageMaxSegs ? nseg - i0 : kStageMaxSegs;
        uint64_t most = 0;
        for (int i = 0; i < n; ++i) {
            a.seg[i] = segs[i0 + i];
            most = a.seg[i].bytes > most ? a.seg[i].bytes : most;
        }
        uint64_t blocks = (most / 16 + 255) / 256;
        blocks = blocks < 1 ? 1 : (blocks > 512 ? 512 : blocks);
        hipLaunchKernelGGL(k_stage_scatter, dim3((uint32_t)blocks, (uint32_t)n), dim3(256), 0, s, a);
    }
    return hipGetLastError();
}

hipError_t put3(unsigned long long* d_dst, uint64_t a, uint64_t b, uint64_t c, hipStream_t s) {
    hipLaunchKernelGGL(k_put3, dim3(1), dim3(64), 0, s, d_dst, a, b, c);
    return hipGetLastError();
}
hipError_t chain_summary(const ChainState* st, unsigned long long* d_dst, hipStream_t s) {
    if (!st->valid) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_chain_summary, dim3(1), dim3(64), 0, s, (const unsigned long long*)st->y.info, d_dst, st->base);
    return hipGetLastError();
}

// fix-ups (every chain once, then the listed ones on one workgroup), the scans and the descriptors
static hipError_t chain_fix_and_meta(ChainState* st, const Tables& t, int ncu, hipStream_t s) {
    ChainArgs& y = st->y;
    hipError_t e;
    if ((e = hipMemsetAsync(y.lcnt, 0, 8, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(y.info, 0, 16, s)) != hipSuccess) return e;  // blocks, largest block (atomicMax)
    if ((e = ensure_lds_limit((const void*)k_chain_fix<DEC_LUT>, kLdsBytes)) != hipSuccess) return e;
    if ((e = ensure_lds_limit((const void*)k_chain_fix_loop<DEC_LUT>, kLdsBytes)) != hipSuccess) return e;
    uint64_t wgs = (y.nchains + kSyncThreads - 1) / kSyncThreads;
    wgs = wgs < (uint64_t)ncu ? (wgs ? wgs : 1) : (uint64_t)ncu;
    hipLaunchKernelGGL(k_chain_fix<DEC_LUT>, dim3(wgs), dim3(kSyncThreads), t.chain_lds_bytes, s, st->d, y);
    hipLaunchKernelGGL(k_chain_fix_loop<DEC_LUT>, dim3(1), dim3(kSyncThreads), t.chain_lds_bytes, s, st->d, y);
    cap_check(s, "fix");
    if ((e = scan_u64(y.tcnt, y.nchains, st->tiles, y.first, s)) != hipSuccess) return e;
    if ((e = scan_u64(y.nblk, y.nchains, st->tiles, y.bbase, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_chain_meta, dim3((y.nchains + 255) / 256), dim3(256), 0, s, y);
    cap_check(s, "scan+meta");
    return hipGetLastError();
}

hipError_t chain_scan(ChainState* st, const Tables& t, const uint8_t* d_payload, uint64_t payload_bytes,
                      uint64_t base, uint64_t start_bit, uint64_t nsym, uint64_t part_begin, uint64_t part_end,
                      uint64_t entry0, unsigned long long* d_scratch, uint32_t* d_err, int ncu, hipStream_t s) {
    st->valid = false;
    // bits of the view from here on: stream bit b is view bit b - base (mod 2^64: start_bit may lie
    // before the view when it begins inside the stream)
    st->base = base;
    start_bit -= base;
    if (entry0 != ~0ull) entry0 -= base;
    if (!seg_decode_supported(t)) return hipErrorInvalidValue;
    DecArgs& d = st->d;
    fill_chain_dec_args(d, t, d_payload, payload_bytes, nsym);
    d.starts = nullptr; d.subs = nullptr; d.out = nullptr; d.err = d_err;
    if (d.nwords < 4) return hipErrorInvalidValue;
    const ChainGeom& g = st->g = chain_geom(part_begin, part_end,
                                             chain_avg(t, part_end > part_begin ? part_end - part_begin : 0, nsym), ncu);
    if (g.nchains == 0 || g.nchains >= (1ull << 32)) return hipErrorInvalidValue;
    ChainArgs& y = st->y;
    y.nchains = g.nchains; y.cbits = g.cbits; y.pbeg = g.pbeg; y.pend = g.pend; y.start = start_bit;
    y.entry0 = entry0;
    y.bpc = g.bpc; y.cap = g.cap;
    unsigned long long* sc = d_scratch;
    y.rec = reinterpret_cast<uint16_t*>(sc + g.off_rec);
    y.ckpt = sc + g.off_ckpt;
    unsigned long long* arr = sc + g.off_arr;
    y.ent = arr; y.xit = arr + g.nchains; y.txit = arr + 2 * g.nchains; y.cnt = arr + 3 * g.nchains;
    y.tcnt = arr + 4 * g.nchains; y.nblk = arr + 5 * g.nchains; y.first = arr + 6 * g.nchains;
    y.bbase = arr + 7 * g.nchains;
    y.hd = reinterpret_cast<uint32_t*>(sc + g.off_u32);
    y.r0 = y.hd + g.nchains;
    y.list[0] = reinterpret_cast<uint32_t*>(sc + g.off_list);
    y.list[1] = y.list[0] + g.nchains;
    y.lcnt = y.list[1] + g.nchains;
    y.info = sc + g.off_info;
    y.blk = reinterpret_cast<ChainBlk*>(sc + g.off_blk);
    y.err = d_err;
    st->tiles = sc + g.off_tiles;
    WalkArgs& w = st->w;
    w.words = d.words; w.nwords = d.nwords; w.bit_adj = d.bit_adj;
    w.start = start_bit; w.nseg = 0;
    w.lds_img = nullptr; w.lds_words = 0; w.k = 0; w.bias = 0;
    w.esc = t.chain_esc; w.m = t.chain_esc_m;
    w.w8_img = t.d_walk8; w.w8_words = t.walk8_bytes / 4; w.k8 = t.walk8_k;
    w.lut1 = t.chain_lds; w.lut2 = t.chain_l2; w.lutk = t.chain_k;
    w.bmp = nullptr; w.cnt = nullptr; w.ent = nullptr; w.dirty = nullptr;
    // test hook: HZ_SEG_LEAD=<bits> (0: no lead-in, so nearly every chain takes the fix-up path)
    static const uint32_t lead = [] { const char* v = getenv("HZ_SEG_LEAD"); return v ? (uint32_t)atoi(v) : kWalkLead; }();
    w.lead = lead;
    hipError_t e;
    // 1. the walk: one chain per lane; small chain counts spread over every CU (fewer waves per workgroup)
    {
        uint64_t wpg = (g.nchains + 64ull * ncu - 1) / (64ull * ncu);
        wpg = wpg < 1 ? 1 : (wpg > (uint64_t)kChainWalkWaves ? (uint64_t)kChainWalkWaves : wpg);
        const uint32_t threads = (uint32_t)(64 * wpg);
        const uint32_t ring_bytes = kSegRing * kRingRow * 4 + threads * 16;  // ring rows (1024 lanes), record buffers
        // DEEP: escapes past the escape table's bits (codes longer than kChainEscMaxBits)
        const bool deep = t.dec_max_len > t.chain_esc_m;
        const void* fn = deep ? (const void*)k_chain_walk<true> : (const void*)k_chain_walk<false>;
        if ((e = ensure_lds_limit(fn, (int)(kChainWalkWaves * 64 * (kSegRing * 4 + 16)))) != hipSuccess) return e;
        const uint64_t wgs = (g.nchains + threads - 1) / threads;
        if (deep) hipLaunchKernelGGL(k_chain_walk<true>, dim3(wgs), dim3(threads), ring_bytes, s, w, y);
        else hipLaunchKernelGGL(k_chain_walk<false>, dim3(wgs), dim3(threads), ring_bytes, s, w, y);
        cap_check(s, "walk");
    }
    // 2.-4. fix-ups, scans, block descriptors and the part's summary
    if ((e = chain_fix_and_meta(st, t, ncu, s)) != hipSuccess) return e;
    st->valid = true;
    return hipSuccess;
}

hipError_t chain_refix(ChainState* st, const Tables& t, uint64_t entry0, int ncu, hipStream_t s) {
    if (!st->valid) return hipErrorInvalidValue;
    st->y.entry0 = entry0 != ~0ull ? entry0 - st->base : entry0;
    return chain_fix_and_meta(st, t, ncu, s);
}

hipError_t chain_decode(ChainState* st, const Tables& t, uint64_t nsym, uint8_t* d_out, unsigned long long* d_end,
                        int ncu, hipStream_t s) {
    if (!st->valid) return hipErrorInvalidValue;
    DecArgs d = st->d;
    const ChainArgs& y = st->y;
    d.out = d_out;
    d.nsym = nsym;
    hipError_t e;
    if ((e = hipMemsetAsync(y.info + 2, 0xff, 8, s)) != hipSuccess) return e;  // end bit: not found
    if (nsym && !chain_pipelined(t)) {
        // 5'. codes past two table levels: the records one thread each
        if ((e = ensure_lds_limit((const void*)k_chain_decode_serial, kLdsBytes)) != hipSuccess) return e;
        hipLaunchKernelGGL(k_chain_decode_serial, dim3(4 * ncu), dim3(kSyncThreads), t.chain_lds_bytes, s, d, y);
    }
    if (nsym && chain_pipelined(t)) {
        // 5. the block decoder: k_decode's slot sizing, two slots per wave, persistent over every CU
        if ((e = ensure_lds_limit((const void*)k_chain_decode, kLdsBytes)) != hipSuccess) return e;
        const uint64_t bits = st->g.pend - st->g.pbeg;
        uint64_t avg = (uint64_t)(chain_avg(t, bits, nsym) * kBlockSyms);  // expected block bits
        avg = avg < (uint64_t)kBlockSyms * (uint32_t)d.max_len ? avg : (uint64_t)kBlockSyms * (uint32_t)d.max_len;
        const uint32_t worst = dec_slot_words_max(d.max_len);
        uint32_t est = dec_slot_words(avg + avg / 16 + 256, d.max_len);
        est = est < worst ? est : worst;
        const uint32_t table = d.lds_words;
        if (table < kDecMinLdsWords || table + worst > kLdsBytes / 4) return hipErrorInvalidValue;  // (biased windows)
        uint32_t nslot = (kLdsBytes / 4 - table) / est;
        nslot = nslot > 2 * kDecPipe2Threads / 64 ? 2 * kDecPipe2Threads / 64 : nslot;
        nslot &= ~1u;
        DecArgs b = d;
        b.region_words = nslot * est;
        if (b.region_words < 2 * worst && table + 2 * worst <= kLdsBytes / 4) b.region_words = 2 * worst;
        const int threads = 64 * (int)((nslot / 2) ? nslot / 2 : 1);
        const uint32_t lds = 4 * (table + b.region_words);
        hipLaunchKernelGGL(k_chain_decode, dim3(ncu), dim3(threads), lds, s, b, y);
        cap_check(s, "decode");
    }
    if (nsym) {
        // 6. heads, records past the capacity, the end bit
        if ((e = ensure_lds_limit((const void*)k_chain_tail<DEC_LUT>, kLdsBytes)) != hipSuccess) return e;
        uint64_t wgs = (y.nchains + kSyncThreads - 1) / kSyncThreads;
        wgs = wgs < (uint64_t)ncu ? (wgs ? wgs : 1) : (uint64_t)ncu;
        hipLaunchKernelGGL(k_chain_tail<DEC_LUT>, dim3(wgs), dim3(kSyncThreads), t.chain_lds_bytes, s, d, y);
    }
    if (d_end) {
        if (st->base == 0) {
            if ((e = hipMemcpyAsync(d_end, y.info + 2, 8, hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
        } else {
            hipLaunchKernelGGL(k_chain_end, dim3(1), dim3(64), 0, s, (const unsigned long long*)y.info, d_end, st->base);
        }
    }
    cap_check(s, "tail+end");
    return hipGetLastError();
}

}  // namespace hz
