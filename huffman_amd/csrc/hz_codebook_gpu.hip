// hz_codebook_gpu.hip -- the codebook and the header on the device (SURVEY.md
// 8f-2, 8f-4): gfx950 kernels with the reference's semantics, so a device
// histogram becomes a codebook and a .compressed header without a host hop.
//
//   k_cb_*          65 536-bin histogram -> codebook (hz_codebook layout):
//                   a 64-tile radix sort of (count << 16 | symbol) keys,
//                   GenerateCL's rounds and GenerateCW in one workgroup over
//                   implicit lists, every leaf's code on all CUs (see the
//                   section).
//   k_hw_*          the header (Compressor.cu:431-487, writers :637-669): 64
//                   workgroups of 1024 entries at scanned bit offsets, each
//                   assembled in LDS and stored as words.
//   k_hdr_*         the header parse (Decompressor.cu:65-103): per-segment
//                   entry-offset maps walked in parallel for every candidate
//                   first-entry offset, composed into the true path, then
//                   every entry decoded at its position (see the section).
#include <stdint.h>

#include "huffman_amd.h"
#include "hz_internal.h"

namespace hz {

#define HZ_DEV __device__ __forceinline__

// ---- codebook -----------------------------------------------------------
// 1. Sort: keys (count << 16 | symbol) in 64 tiles of 1024; an LSD radix sort
//    over the count's six 8-bit digits (key bits 16..63; counts < 2^47). The
//    symbols start in order and every pass is stable, so the result is thrust's
//    (count, symbol) order (Compressor.cu:378-425). Each pass is one launch:
//    per-tile digit offsets from the previous pass's per-tile counts, a stable
//    in-tile rank (ballots over the digit's bits), the scatter, and the next
//    digit's per-tile counts by atomics (three rotating count tables).
// 2. GenerateCL (gpuHuffmanConstruction.h:353-466) without materialising its
//    lists: the round list is always the (freq, id) merge of the unused
//    leaves (a suffix of the sorted keys) and the unused internal nodes (a
//    contiguous range: internal nodes are created in nondecreasing frequency,
//    and the merge puts the older node first on ties). A round is a pivot
//    search in both runs (one wave each, 64-ary), the pair formation of the
//    first `pivot` merged elements in LDS tiles (a merge path: each thread
//    merges an even-length run, so a pair never spans threads), and the new
//    nodes appended.
// 3. GenerateCW top-down by round (h:468-494, first child '1'); then toCpu
//    (h:551-579) for every leaf in a 64-workgroup kernel.
constexpr int kCbTiles = 64, kCbTileKeys = 1024, kCbPasses = 6;
constexpr uint32_t kCgT = 6144;  // merged outputs per LDS tile in a GenerateCL round (even)

struct CbWs {
    unsigned long long* keys[2];  // ping-pong, 65 536 each
    uint32_t* cnt[3];             // [tile][256] digit counts (rotating: read, accumulate, zero)
    uint32_t* ublk;               // [64] nonzero counts per tile
    uint32_t* bad;                // [64] a count >= 2^47 in the tile
    unsigned long long* nf;       // internal node frequencies, in creation order
    uint32_t* par;                // [2U - 1] parent id << 1 | code bit
    unsigned long long* ncode;    // internal node codes
    uint8_t* nlen;                // internal node depths
    uint32_t* rounds;             // first internal node id of each round
};

HZ_DEV CbWs cb_ws(unsigned long long* w) {
    CbWs s;
    s.keys[0] = w; w += 65536;
    s.keys[1] = w; w += 65536;
    for (int i = 0; i < 3; ++i) { s.cnt[i] = reinterpret_cast<uint32_t*>(w); w += kCbTiles * 256 / 2; }
    s.ublk = reinterpret_cast<uint32_t*>(w); w += 32;
    s.bad = reinterpret_cast<uint32_t*>(w); w += 32;
    s.nf = w; w += 65536;
    s.par = reinterpret_cast<uint32_t*>(w); w += 65536;
    s.ncode = w; w += 65536;
    s.nlen = reinterpret_cast<uint8_t*>(w); w += 8192;
    s.rounds = reinterpret_cast<uint32_t*>(w);  // up to U + 1 entries (a round creates at least one node)
    return s;
}

constexpr uint64_t kCbWsWords = 2 * 65536 + 3 * kCbTiles * 128 + 64 + 3 * 65536 + 8192 + 32768 + 64;

__global__ __launch_bounds__(kCbTileKeys) void k_cb_keys(const unsigned long long* __restrict__ hist,
                                                         hz_codebook* __restrict__ cb, unsigned long long* wsp) {
    __shared__ uint32_t dh[256];
    const CbWs w = cb_ws(wsp);
    const uint32_t t = blockIdx.x, tid = threadIdx.x, s = t * kCbTileKeys + tid;
    if (tid < 256) {
        dh[tid] = 0;
        w.cnt[1][t * 256 + tid] = 0;  // pass 0 accumulates pass 1's counts here
    }
    const unsigned long long h = hist[s];
    cb->len[s] = 0;
    cb->code[s] = 0;
    w.keys[0][s] = (h << 16) | s;
    __syncthreads();
    atomicAdd(&dh[(uint32_t)(h & 0xffu)], 1u);  // pass 0's digit: count bits 0..7
    const int nz = __syncthreads_count(h != 0);
    const int bad = __syncthreads_or((h >> 47) != 0);
    if (tid < 256) w.cnt[0][t * 256 + tid] = dh[tid];
    if (tid == 0) {
        w.ublk[t] = (uint32_t)nz;
        w.bad[t] = bad ? 1u : 0u;
    }
}

template <int P>
__global__ __launch_bounds__(kCbTileKeys) void k_cb_scatter(hz_codebook* __restrict__ cb, unsigned long long* wsp) {
    __shared__ uint32_t wc[kCbTileKeys / 64][256];  // per-wave digit counts, then their scatter offsets
    __shared__ uint32_t sc[256], off[256];
    __shared__ uint32_t sh_z;
    const CbWs w = cb_ws(wsp);
    const uint32_t t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const unsigned long long* src = w.keys[P & 1];
    unsigned long long* dst = w.keys[(P + 1) & 1];
    const uint32_t* cur = w.cnt[P % 3];
    uint32_t* nxt = w.cnt[(P + 1) % 3];
    for (uint32_t i = tid; i < (kCbTileKeys / 64) * 256; i += kCbTileKeys) (&wc[0][0])[i] = 0;
    uint32_t pre = 0;
    if (tid < 256) {
        if (P + 2 < kCbPasses) w.cnt[(P + 2) % 3][t * 256 + tid] = 0;  // read by pass P - 1, accumulated by P + 1
        uint32_t tot = 0;
        for (uint32_t u = 0; u < (uint32_t)kCbTiles; ++u) {
            const uint32_t v = cur[u * 256 + tid];
            tot += v;
            pre += u < t ? v : 0u;
        }
        sc[tid] = tot;
    }
    if (P + 1 == kCbPasses && tid < 64) {
        uint32_t u = w.ublk[tid];
        for (int d = 32; d >= 1; d >>= 1) u += __shfl_xor(u, d);
        if (tid == 0) sh_z = 65536 - u;
    }
    __syncthreads();
    if (tid < 64) {  // exclusive scan of the 256 digit totals
        const uint32_t a0 = sc[4 * lane], a1 = sc[4 * lane + 1], a2 = sc[4 * lane + 2], a3 = sc[4 * lane + 3];
        const uint32_t sum = a0 + a1 + a2 + a3;
        uint32_t incl = sum;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t v = __shfl_up(incl, d);
            if ((int)lane >= d) incl += v;
        }
        const uint32_t e = incl - sum;
        sc[4 * lane] = e;
        sc[4 * lane + 1] = e + a0;
        sc[4 * lane + 2] = e + a0 + a1;
        sc[4 * lane + 3] = e + a0 + a1 + a2;
    }
    __syncthreads();
    if (tid < 256) off[tid] = sc[tid] + pre;
    const unsigned long long key = src[t * kCbTileKeys + tid];
    const uint32_t d = (uint32_t)(key >> (16 + 8 * P)) & 0xffu;
    unsigned long long m = ~0ull;
#pragma unroll
    for (int bt = 0; bt < 8; ++bt) {
        const unsigned long long bal = __ballot((d >> bt) & 1u);
        m &= ((d >> bt) & 1u) ? bal : ~bal;
    }
    const uint32_t below = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    if (below == 0) wc[wv][d] = (uint32_t)__popcll(m);
    __syncthreads();
    if (tid < 256) {
        uint32_t run = off[tid];
        for (uint32_t v = 0; v < (uint32_t)(kCbTileKeys / 64); ++v) {
            const uint32_t x = wc[v][tid];
            wc[v][tid] = run;
            run += x;
        }
    }
    __syncthreads();
    const uint32_t pos = wc[wv][d] + below;
    dst[pos] = key;
    if (P + 1 < kCbPasses) {  // next pass's (tile, digit) counts: one atomic per distinct pair in the wave
        const uint32_t slot = (pos / kCbTileKeys) * 256 + ((uint32_t)(key >> (16 + 8 * (P + 1))) & 0xffu);
        unsigned long long ms = ~0ull;
#pragma unroll
        for (int bt = 0; bt < 14; ++bt) {
            const unsigned long long bal = __ballot((slot >> bt) & 1u);
            ms &= ((slot >> bt) & 1u) ? bal : ~bal;
        }
        if ((ms & ((1ull << lane) - 1ull)) == 0) atomicAdd(&nxt[slot], (uint32_t)__popcll(ms));
    } else if (pos >= sh_z) {
        cb->order[pos - sh_z] = (uint16_t)(key & 0xffffu);  // leaves in (count, symbol) order
    }
}

// Number of indices in [lo, hi) with pred true, pred true on a prefix only. One
// full wave; each level is one dependent probe per lane (64-ary).
template <class Pred>
HZ_DEV uint32_t wave_true_prefix(uint32_t lo, uint32_t hi, uint32_t lane, Pred pred) {
    const uint32_t base = lo;
    while (hi - lo > 64) {
        const uint32_t s = (hi - lo + 63) / 64, idx = lo + (lane + 1) * s - 1;
        const bool tr = idx < hi && pred(idx);
        const uint32_t c = (uint32_t)__popcll(__ballot(tr));
        const uint32_t nhi = lo + (c + 1) * s - 1;
        lo += c * s;
        hi = nhi < hi ? nhi : hi;
        if (lo > hi) lo = hi;
    }
    const bool tr = lo + lane < hi && pred(lo + lane);
    return lo + (uint32_t)__popcll(__ballot(tr)) - base;
}

#ifdef HZ_CB_PROF  // phase timestamps (100 MHz) into the spare key buffer: tools/debug/cb_prof.py
#define CG_T(slot) do { if (tid == 0) prof[slot] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define CG_T(slot) do { } while (0)
#endif
constexpr int kCgThreads = 1024;
constexpr uint32_t kCgMaxTiles = (65536 + kCgT - 1) / kCgT;

__global__ __launch_bounds__(kCgThreads) void k_cb_generate(hz_codebook* __restrict__ cb, unsigned long long* wsp,
                                                            uint32_t* err) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long cgl[];  // SL[kCgT] | SI[kCgT]
    __shared__ uint32_t sh_u, sh_bad, sh_max, sh_min, sh_a, sh_b, sh_bnd[kCgMaxTiles + 1];
    __shared__ unsigned long long sh_spec;
    unsigned long long* SL = cgl;
    unsigned long long* SI = cgl + kCgT;
    const CbWs w = cb_ws(wsp);
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#ifdef HZ_CB_PROF
    unsigned long long* prof = w.keys[(kCbPasses + 1) & 1];
#endif
    CG_T(0);
    if (tid < 64) {
        uint32_t u = w.ublk[tid], b = w.bad[tid];
        for (int d = 32; d >= 1; d >>= 1) {
            u += __shfl_xor(u, d);
            b |= __shfl_xor(b, d);
        }
        if (tid == 0) {
            sh_u = u;
            sh_bad = b;
            sh_max = 0;
            sh_min = 255;
        }
    }
    __syncthreads();
    const uint32_t U = sh_u;
    if (sh_bad) {
        if (tid == 0) atomicOr(err, 16u);
        return;
    }
    if (U <= 1) {  // U == 1: code "0" (the reference's defect B4)
        if (tid == 0) {
            cb->nsym = U;
            cb->max_len = cb->min_len = U;
            cb->reserved = 0;
            if (U == 1) { cb->len[cb->order[0]] = 1; cb->code[cb->order[0]] = 0; }
        }
        return;
    }
    const unsigned long long* keys = w.keys[kCbPasses & 1] + (65536 - U);  // sorted leaves; freq = key >> 16
    auto LF = [&](uint32_t i) { return keys[i] >> 16; };
    const unsigned long long* nf = w.nf;
    uint32_t lp = 0, ip = 0, ni = 0, nr = 0;  // next leaf, next internal node, internal nodes, rounds
    CG_T(1);
    for (;;) {
        const uint32_t size = (U - lp) + (ni - ip);
        if (size <= 1) break;
        if (tid == 0) {  // the two smallest of the merged list (the leaf first on ties)
            const unsigned long long l0 = lp < U ? LF(lp) : ~0ull, l1 = lp + 1 < U ? LF(lp + 1) : ~0ull;
            const unsigned long long i0 = ip < ni ? nf[ip] : ~0ull, i1 = ip + 1 < ni ? nf[ip + 1] : ~0ull;
            unsigned long long f0, f1;
            if (l0 <= i0) { f0 = l0; f1 = l1 <= i0 ? l1 : i0; }
            else { f0 = i0; f1 = l0 <= i1 ? l0 : i1; }
            sh_spec = f0 + f1;
            w.rounds[nr] = U + ni;
        }
        __syncthreads();
        const unsigned long long spec = sh_spec;
        // BinarySearch (h:137-151): the first element > f0 + f1 among f[2 .. size - 1), else size - 1
        if (wv == 0) {
            const uint32_t c = wave_true_prefix(lp, U, lane, [&](uint32_t i) { return LF(i) <= spec; });
            if (lane == 0) sh_a = c;
        } else if (wv == 1) {
            const uint32_t c = wave_true_prefix(ip, ni, lane, [&](uint32_t k) { return nf[k] <= spec; });
            if (lane == 0) sh_b = c;
        }
        __syncthreads();
        CG_T(16 + 4 * nr);
        uint32_t a = sh_a, b = sh_b;
        const uint32_t cap = size - 1 > 2 ? size - 1 : 2;
        const uint32_t P = (a + b < cap ? a + b : cap) & ~1u, half = P / 2;
        if (a + b > P) {  // the prefix loses its largest one or two elements (the newer node last on ties)
            __syncthreads();
            if (tid == 0) {
                while (a + b > P) {
                    if (b == 0) --a;
                    else if (a == 0) --b;
                    else if (nf[ip + b - 1] >= LF(lp + a - 1)) --b;
                    else --a;
                }
                sh_a = a;
                sh_b = b;
            }
            __syncthreads();
            a = sh_a;
            b = sh_b;
        }
        // pairs (2i, 2i + 1) of the first P merged elements -> internal nodes U + ni + i, in LDS tiles
        const uint32_t ntile = (P + kCgT - 1) / kCgT;
        for (uint32_t j = wv + 1; j < ntile; j += kCgThreads / 64) {  // tile boundaries: co-rank, one wave each
            const uint32_t q = j * kCgT, xlo = q > b ? q - b : 0, xhi = q < a ? q : a;
            const uint32_t c = wave_true_prefix(xlo + 1, xhi + 1, lane, [&](uint32_t x) {
                return q - x >= b || LF(lp + x - 1) <= nf[ip + q - x];
            });
            if (lane == 0) sh_bnd[j] = xlo + c;
        }
        if (tid == 0) {
            sh_bnd[0] = 0;
            sh_bnd[ntile] = a;
        }
        __syncthreads();
        for (uint32_t j = 0; j < ntile; ++j) {
            const uint32_t q0 = j * kCgT, q1 = q0 + kCgT < P ? q0 + kCgT : P;
            const uint32_t x0 = sh_bnd[j], nl = sh_bnd[j + 1] - x0, y0 = q0 - x0, nI = (q1 - q0) - nl;
            for (uint32_t i = tid; i < nl; i += kCgThreads) SL[i] = LF(lp + x0 + i);
            for (uint32_t i = tid; i < nI; i += kCgThreads) SI[i] = nf[ip + y0 + i];
            __syncthreads();
            // merge path: thread tid takes an even-length run of the tile's merged outputs
            const uint32_t n = q1 - q0, c = ((n + kCgThreads - 1) / kCgThreads + 1) & ~1u;
            const uint32_t k0 = tid * c < n ? tid * c : n, k1 = k0 + c < n ? k0 + c : n;
            if (k0 < k1) {
                uint32_t lo = k0 > nI ? k0 - nI : 0, hi = k0 < nl ? k0 : nl;  // leaves among the first k0
                while (lo < hi) {
                    const uint32_t x = (lo + hi + 1) / 2;
                    if (k0 - x >= nI || SL[x - 1] <= SI[k0 - x]) lo = x;
                    else hi = x - 1;
                }
                uint32_t x = lo, y = k0 - lo;
                unsigned long long even = 0;
                for (uint32_t k = k0; k < k1; ++k) {
                    const bool leaf = y >= nI || (x < nl && SL[x] <= SI[y]);  // the leaf first on ties
                    const unsigned long long f = leaf ? SL[x] : SI[y];
                    const uint32_t id = leaf ? lp + x0 + x : U + ip + y0 + y, node = U + ni + (q0 + k) / 2;
                    w.par[id] = (node << 1) | ((k & 1u) ^ 1u);  // first child '1'
                    if (k & 1u) w.nf[node - U] = even + f;
                    else even = f;
                    x += leaf;
                    y += !leaf;
                }
            }
            __syncthreads();
        }
#ifdef HZ_CB_PROF
        CG_T(17 + 4 * nr);
        if (tid == 0) {
            prof[18 + 4 * nr] = P | (unsigned long long)ntile << 32;
            prof[19 + 4 * nr] = a | (unsigned long long)b << 32;
        }
#endif
        lp += a;
        ip += b;
        ni += half;
        ++nr;
    }
    CG_T(2);
    if (tid == 0) w.rounds[nr] = U + ni;  // == 2U - 1
    __syncthreads();
    // GenerateCW top-down, round by round from the root (the last round's only node)
    for (int r = (int)nr - 1; r >= 0; --r) {
        const uint32_t b0 = w.rounds[r], e0 = w.rounds[r + 1];
        for (uint32_t v = b0 + tid; v < e0; v += kCgThreads) {
            unsigned long long c = 0;
            uint32_t L = 0;
            if (v != 2 * U - 2) {
                const uint32_t pr = w.par[v], pk = (pr >> 1) - U;
                c = (w.ncode[pk] << 1) | (pr & 1u);
                L = w.nlen[pk] + 1u;
            }
            w.ncode[v - U] = c;
            w.nlen[v - U] = (uint8_t)(L < 255 ? L : 255);
        }
        __syncthreads();
    }
    CG_T(3);
    if (tid == 0) {
        cb->nsym = U;
        cb->max_len = 0;
        cb->min_len = 255;
        cb->reserved = 0;
#ifdef HZ_CB_PROF
        prof[5] = nr;
#endif
    }
}

// toCpu (h:551-579): every leaf's code from its parent's, in (count, symbol) order; all CUs.
__global__ __launch_bounds__(kCbTileKeys) void k_cb_leaves(hz_codebook* __restrict__ cb, unsigned long long* wsp,
                                                           uint32_t* err) {
    __shared__ uint32_t sh_u, sh_bad;
    const CbWs w = cb_ws(wsp);
    const uint32_t tid = threadIdx.x;
    if (tid < 64) {
        uint32_t u = w.ublk[tid], b = w.bad[tid];
        for (int d = 32; d >= 1; d >>= 1) {
            u += __shfl_xor(u, d);
            b |= __shfl_xor(b, d);
        }
        if (tid == 0) {
            sh_u = u;
            sh_bad = b;
        }
    }
    __syncthreads();
    const uint32_t U = sh_u, i = blockIdx.x * kCbTileKeys + tid;
    if (sh_bad || U <= 1) return;  // k_cb_generate reported / wrote these
    uint32_t L = 0;
    if (i < U) {
        const uint32_t pr = w.par[i], pk = (pr >> 1) - U;
        const uint32_t L0 = w.nlen[pk] + 1u;
        L = L0 < 255 ? L0 : 255;
        const uint32_t s = (uint32_t)(w.keys[kCbPasses & 1][65536 - U + i] & 0xffffu);
        cb->len[s] = (uint8_t)L;
        cb->code[s] = (w.ncode[pk] << 1) | (pr & 1u);
    }
    uint32_t mx = L, mn = i < U ? L : 255;
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t a = __shfl_xor(mx, d), b = __shfl_xor(mn, d);
        mx = a > mx ? a : mx;
        mn = b < mn ? b : mn;
    }
    if ((tid & 63) == 0 && mx) {
        atomicMax(&cb->max_len, mx);
        atomicMin(&cb->min_len, mn);
        if (mx > HZ_MAXLEN) atomicOr(err, 32u);
    }
}

// ---- header writer ---------------------------------------------------------
// Bit stream MSB first: bit b of the header is bit 7 - b % 8 of byte b / 8.
// 64 workgroups own 1024 entries each (Compressor.cu:454-483: symbol, L, code):
// k_hw_sum sums each workgroup's entry bits, k_hw_prep scans the 64 sums into
// start bits, zeroes the output words two workgroups share and writes the
// info, k_hw_write assembles each workgroup's bits in LDS (prefix :434-443 in
// workgroup 0, N :661-669 in workgroup 63) and stores its words -- the two
// shared ones with atomicOr, the rest with plain stores.
constexpr int kHwGroups = 64, kHwThreads = 1024;
constexpr uint32_t kHwWords = (kHwThreads * (24 + HZ_MAXLEN) + 64 + 32 + 31) / 32 + 2;  // one workgroup's bits

struct HwWs {
    unsigned long long* sum;   // [64] entry bits per workgroup
    unsigned long long* off;   // [65] first bit per workgroup, then the N field's first bit
    unsigned long long* meta;  // [0] total bits, [1] capacity failure
};

HZ_DEV HwWs hw_ws(unsigned long long* w) { return HwWs{w, w + 64, w + 64 + 65}; }

// ORs the low nb (<= 64) bits of v, first bit = bit nb - 1, at bit b of an LDS
// run of big-endian-valued words.
HZ_DEV void hw_put(uint32_t* lw, uint32_t b, uint64_t v, uint32_t nb) {
    while (nb) {
        const uint32_t off = b & 31, take = 32 - off < nb ? 32 - off : nb;
        const uint32_t bits = (uint32_t)(v >> (nb - take)) & (take == 32 ? 0xffffffffu : ((1u << take) - 1u));
        atomicOr(&lw[b >> 5], bits << (32 - off - take));
        b += take;
        nb -= take;
    }
}

__global__ __launch_bounds__(kHwThreads) void k_hw_sum(const hz_codebook* __restrict__ cb, unsigned long long* wsp) {
    __shared__ uint32_t part[kHwThreads / 64];
    const HwWs w = hw_ws(wsp);
    const uint32_t i = blockIdx.x * kHwThreads + threadIdx.x, U = cb->nsym;
    uint32_t v = i < U ? 24u + cb->len[cb->order[i]] : 0u;
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long s = 0;
        for (int k = 0; k < kHwThreads / 64; ++k) s += part[k];
        w.sum[blockIdx.x] = s;
    }
}

// info (device): [0] complete header bytes, [1] pending bits, [2] pending byte (MSB aligned), [3] header bits
__global__ __launch_bounds__(64) void k_hw_prep(const hz_codebook* __restrict__ cb, uint64_t n, uint8_t* out,
                                                uint64_t cap, unsigned long long* info, unsigned long long* wsp,
                                                uint32_t* err) {
    const HwWs w = hw_ws(wsp);
    const uint32_t t = threadIdx.x;
    const unsigned long long v = w.sum[t];
    unsigned long long incl = v;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)incl, d), hi = (uint32_t)__shfl_up((int)(uint32_t)(incl >> 32), d);
        if ((int)t >= d) incl += ((unsigned long long)hi << 32) | lo;
    }
    const uint64_t pre = 8ull * (3 + (n & 1));
    const uint64_t start = pre + incl - v, nstart = pre + (uint64_t)__shfl((int)(uint32_t)incl, 63) +
                                                    ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(incl >> 32), 63) << 32);
    const uint64_t total = nstart + 64, words = (total + 31) / 32;
    const bool fail = words * 4 > cap;
    w.off[t] = start;
    if (t == 0) {
        w.off[64] = nstart;
        w.meta[0] = total;
        w.meta[1] = fail;
        if (fail) atomicOr(err, 4u);
        const uint32_t r = (uint32_t)(total % 8), last = (uint32_t)(n >> 56) & 0xffu;  // N's last byte ends the header
        info[0] = total / 8;
        info[1] = r;
        info[2] = r ? ((last & ((1u << r) - 1u)) << (8 - r)) & 0xffu : 0u;
        info[3] = total;
    }
    if (!fail && t > 0 && (start & 31)) reinterpret_cast<uint32_t*>(out)[start >> 5] = 0;  // shared with group t - 1
}

__global__ __launch_bounds__(kHwThreads) void k_hw_write(const hz_codebook* __restrict__ cb, uint64_t n,
                                                         uint32_t last_byte, uint8_t* out, unsigned long long* wsp) {
    __shared__ uint32_t lw[kHwWords];
    __shared__ uint32_t part[kHwThreads / 64];
    const HwWs w = hw_ws(wsp);
    if (w.meta[1]) return;
    const uint32_t t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, U = cb->nsym;
    const uint64_t s0 = t == 0 ? 0 : w.off[t], s1 = t + 1 < kHwGroups ? w.off[t + 1] : w.meta[0];
    if (s1 <= s0) return;
    const uint64_t base = s0 & ~31ull;
    const uint32_t nw = (uint32_t)((s1 + 31) / 32 - base / 32);
    for (uint32_t k = tid; k < nw; k += kHwThreads) lw[k] = 0;
    const uint32_t i = t * kHwThreads + tid;
    uint32_t sym = 0, L = 0;
    if (i < U) {
        sym = cb->order[i];
        L = cb->len[sym];
    }
    const uint32_t bits = i < U ? 24u + L : 0u;
    uint32_t incl = bits;  // exclusive scan of the entries' bits in the workgroup
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t x = (uint32_t)__shfl_up((int)incl, d);
        if ((int)lane >= d) incl += x;
    }
    if (lane == 63) part[tid >> 6] = incl;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t k = 0; k < (tid >> 6); ++k) before += part[k];
    const uint32_t rel = (uint32_t)(w.off[t] - base) + before + incl - bits;
    if (i < U) {  // writeFromUShort, writeFromUChar, code bits (:454-483)
        hw_put(lw, rel, ((uint64_t)sym << 8) | L, 24);
        hw_put(lw, rel + 24, cb->code[sym], L);
    }
    if (tid == 0 && t == 0) {
        const uint32_t U16 = U & 0xffffu, odd = (uint32_t)(n & 1);
        hw_put(lw, 0, U16 ? ((U16 & 0xffu) << 8) | (U16 >> 8) : 0u, 16);  // u16 LE (:434)
        hw_put(lw, 16, odd, 8);                                           // isOdd (:438)
        if (odd) hw_put(lw, 24, last_byte & 0xffu, 8);                    // lastByte (:439-443)
    }
    if (tid == 0 && t + 1 == kHwGroups) {  // writeFileSize (:661-669): 8 LE bytes, each MSB first
        uint64_t nn = n;
        const uint32_t nb = (uint32_t)(w.off[64] - base);
        for (int k = 0; k < 8; ++k, nn >>= 8) hw_put(lw, nb + 8 * k, nn & 0xffu, 8);
    }
    __syncthreads();
    uint32_t* o32 = reinterpret_cast<uint32_t*>(out) + base / 32;
    const bool shared_first = t > 0 && (s0 & 31), shared_last = t + 1 < kHwGroups && (s1 & 31);
    for (uint32_t k = tid; k < nw; k += kHwThreads) {
        const uint32_t v = __builtin_bswap32(lw[k]);
        if ((k == 0 && shared_first) || (k + 1 == nw && shared_last)) atomicOr(&o32[k], v);
        else o32[k] = v;
    }
}

// ---- header parser: segment-parallel entry positions --------------------
// An entry is `16-bit symbol, 8-bit L, L code bits`, 25..24 + HZ_MAXLEN bits,
// and its position needs every earlier length (Decompressor.cu:78-103). The
// entry stream (from bit P0 = 8 * (3 + odd)) is cut into kHpSeg-bit segments
// of kHpSub sub-segments. An entry that starts before a (sub-)segment ends
// fewer than kHpCand bits into it, so each has kHpCand candidate first-entry
// offsets. k_hdr_seg walks every (sub-segment, candidate) pair -- exit offset
// into the next sub-segment and entry count -- and composes them into
// per-segment maps; k_hdr_chain resolves the true offset of every segment
// (32-segment groups composed in LDS, then the groups, then the segments) and
// numbers the entries; k_hdr_emit re-walks each sub-segment of the true path
// and decodes its entries in parallel; k_hdr_finish reads N and checks the
// whole. Every walk step is one LDS read pair; no step depends on more than
// one sub-segment (512 bits, at most 21 entries).
constexpr uint32_t kHpSeg = 4096, kHpSub = 8, kHpSubBits = kHpSeg / kHpSub;
constexpr uint32_t kHpCand = 24 + HZ_MAXLEN;                          // 80 candidate offsets
constexpr uint32_t kHpMaxSeg = (65536u * kHpCand + kHpSeg - 1) / kHpSeg;  // 1280
constexpr uint32_t kHpGroup = 32, kHpMaxGroup = (kHpMaxSeg + kHpGroup - 1) / kHpGroup;
constexpr uint32_t kHpWords = (kHpSeg + kHpCand + 24 + 32) / 32 + 2;  // segment + the longest entry past it
constexpr uint8_t kHpDead = 0xff;
static_assert(kHpCand < kHpDead && kHpSeg / 25 < 256, "u8 maps");

struct HpWs {            // in the codebook workspace
    uint8_t* exm;        // [seg][cand] exit offset into the next segment (kHpDead: an invalid length)
    uint8_t* cntm;       // [seg][cand] entries that start in the segment (before an invalid one)
    uint8_t* sub;        // [seg][cand][16]: sub-segment entry offsets, then entries before each sub-segment
    uint8_t* segoff;     // [seg] true first-entry offset (kHpDead past an invalid length)
    uint32_t* base;      // [seg] index of the segment's first entry
    uint32_t* seen;      // 65 536-bit symbol bitmap (duplicates)
    unsigned long long* st;  // [0] entries on the true path, [1] end bit of entry U - 1, [2] dup flag, [3] max, [4] min
};

HZ_DEV HpWs hp_ws(unsigned long long* w) {
    HpWs s;
    uint8_t* b = reinterpret_cast<uint8_t*>(w);
    s.exm = b; b += kHpMaxSeg * kHpCand;
    s.cntm = b; b += kHpMaxSeg * kHpCand;
    s.sub = b; b += kHpMaxSeg * kHpCand * 16;
    s.segoff = b; b += kHpMaxSeg + 64;
    s.base = reinterpret_cast<uint32_t*>(b); b += 4 * (kHpMaxSeg + 64);
    s.seen = reinterpret_cast<uint32_t*>(b); b += 4 * 2048;
    s.st = reinterpret_cast<unsigned long long*>(b);
    return s;
}

struct HpGeo {
    uint32_t ok, U, odd, nseg;
    uint64_t p0;  // first entry bit
};

HZ_DEV HpGeo hp_geo(const uint8_t* f, uint64_t len) {
    HpGeo g{};
    if (len < 3) return g;
    g.odd = f[2] != 0;  // Decompressor.cu:76
    if (g.odd && len < 4) return g;
    const uint64_t pre = g.odd ? 4 : 3;
    g.ok = 1;
    g.U = (uint32_t)f[0] | ((uint32_t)f[1] << 8);  // :69-71, U 0 => 65536 (and the empty-file convention)
    if (g.U == 0) g.U = (len == pre + 8) ? 0 : 65536;
    g.p0 = 8 * pre;
    const uint64_t avail = 8 * len - g.p0, need = (uint64_t)g.U * kHpCand;
    const uint64_t bound = need < avail ? need : avail;
    g.nseg = (uint32_t)((bound + kHpSeg - 1) / kHpSeg);
    return g;
}

// The segment's bits (from bit p0 + seg * kHpSeg, byte aligned) as big-endian words in LDS, zeros past len.
HZ_DEV void hp_load(uint32_t* wl, const uint8_t* f, uint64_t len, uint64_t byte0) {
    for (uint32_t i = threadIdx.x; i < kHpWords; i += blockDim.x) {
        uint32_t v = 0;
        for (uint32_t k = 0; k < 4; ++k) {
            const uint64_t b = byte0 + 4 * i + k;
            v = (v << 8) | (b < len ? f[b] : 0u);
        }
        wl[i] = v;
    }
}

HZ_DEV uint32_t hp_bits32(const uint32_t* wl, uint32_t p) {
    const uint32_t i = p >> 5, sh = p & 31;
    return sh ? (wl[i] << sh) | (wl[i + 1] >> (32 - sh)) : wl[i];
}

// Walk from segment bit p while p < end: entries and the first start at or past end (kHpDead on an invalid L).
HZ_DEV uint32_t hp_walk(const uint32_t* wl, uint32_t p, uint32_t end, uint32_t& cnt) {
    uint32_t c = 0;
    while (p < end) {
        const uint32_t L = (hp_bits32(wl, p) >> 8) & 0xffu;  // bits p + 16 .. p + 24: the entry's L
        if (L - 1u >= (uint32_t)HZ_MAXLEN) { cnt = c; return ~0u; }
        p += 24 + L;
        ++c;
    }
    cnt = c;
    return p;
}

constexpr int kHpSegThreads = kHpSub * kHpCand;  // 640: one lane per (sub-segment, candidate)

__global__ __launch_bounds__(kHpSegThreads) void k_hdr_seg(const uint8_t* __restrict__ f, uint64_t len,
                                                            hz_codebook* __restrict__ cb, unsigned long long* wsp) {
    __shared__ uint32_t wl[kHpWords];
    __shared__ uint8_t sx[kHpSub][kHpCand], sc[kHpSub][kHpCand];
    const HpWs w = hp_ws(wsp);
    const uint32_t tid = threadIdx.x;
    // zero the codebook and the duplicate bitmap (grid-stride over every block)
    const uint64_t gt = (uint64_t)blockIdx.x * blockDim.x + tid, gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t s = gt; s < 65536; s += gs) { cb->len[s] = 0; cb->code[s] = 0; }
    for (uint64_t s = gt; s < 2048; s += gs) w.seen[s] = 0;
    if (gt < 8) w.st[gt] = gt == 4 ? 255 : 0;
    const HpGeo g = hp_geo(f, len);
    const uint32_t seg = blockIdx.x;
    if (!g.ok || seg >= g.nseg) return;
    hp_load(wl, f, len, g.p0 / 8 + (uint64_t)seg * (kHpSeg / 8));
    __syncthreads();
    {
        const uint32_t q = tid / kHpCand, o = tid % kHpCand, end = (q + 1) * kHpSubBits;
        uint32_t c;
        const uint32_t p = hp_walk(wl, q * kHpSubBits + o, end, c);
        sx[q][o] = p == ~0u ? kHpDead : (uint8_t)(p - end);
        sc[q][o] = (uint8_t)c;
    }
    __syncthreads();
    if (tid < kHpCand) {  // compose the sub-segment maps for candidate tid
        uint32_t x = tid, cum = 0;
        uint64_t offs = 0, cums = 0;
        for (uint32_t q = 0; q < kHpSub; ++q) {
            offs |= (uint64_t)x << (8 * q);
            cums |= (uint64_t)cum << (8 * q);
            if (x != kHpDead) {
                cum += sc[q][x];
                x = sx[q][x];
            }
        }
        const uint32_t k = seg * kHpCand + tid;
        w.exm[k] = (uint8_t)x;
        w.cntm[k] = (uint8_t)cum;
        uint64_t* sub = reinterpret_cast<uint64_t*>(w.sub + 16ull * k);
        sub[0] = offs;
        sub[1] = cums;
    }
}

constexpr int kHpChainThreads = 1024;

__global__ __launch_bounds__(kHpChainThreads) void k_hdr_chain(const uint8_t* __restrict__ f, uint64_t len,
                                                                unsigned long long* wsp) {
    extern __shared__ __attribute__((aligned(16))) uint8_t xm[];  // [seg][cand] exits
    __shared__ uint8_t gx[kHpMaxGroup * kHpCand], gin[kHpMaxGroup];
    __shared__ uint32_t part[kHpChainThreads / 64];
    const HpWs w = hp_ws(wsp);
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const HpGeo g = hp_geo(f, len);
    const uint32_t nseg = g.ok ? g.nseg : 0, ngr = (nseg + kHpGroup - 1) / kHpGroup;
    const uint32_t nbytes = nseg * kHpCand;  // a multiple of 16
    for (uint32_t i = tid; i < nbytes / 16; i += nt)
        reinterpret_cast<uint4*>(xm)[i] = reinterpret_cast<const uint4*>(w.exm)[i];
    __syncthreads();
    for (uint32_t k = tid; k < ngr * kHpCand; k += nt) {  // a group's exit for each entry offset
        const uint32_t gr = k / kHpCand, s1 = (gr + 1) * kHpGroup < nseg ? (gr + 1) * kHpGroup : nseg;
        uint32_t x = k % kHpCand;
        for (uint32_t s = gr * kHpGroup; s < s1 && x != kHpDead; ++s) x = xm[s * kHpCand + x];
        gx[k] = (uint8_t)x;
    }
    __syncthreads();
    if (tid == 0) {  // the groups, from entry 0 at offset 0
        uint32_t x = 0;
        for (uint32_t gr = 0; gr < ngr; ++gr) {
            gin[gr] = (uint8_t)x;
            if (x != kHpDead) x = gx[gr * kHpCand + x];
        }
    }
    __syncthreads();
    if (tid < ngr) {  // the segments of group tid
        const uint32_t s1 = (tid + 1) * kHpGroup < nseg ? (tid + 1) * kHpGroup : nseg;
        uint32_t x = gin[tid];
        for (uint32_t s = tid * kHpGroup; s < s1; ++s) {
            w.segoff[s] = (uint8_t)x;
            if (x != kHpDead) x = xm[s * kHpCand + x];
        }
    }
    __syncthreads();
    // entries per segment on the true path -> exclusive scan -> first entry index
    constexpr uint32_t kPer = (kHpMaxSeg + kHpChainThreads - 1) / kHpChainThreads;
    uint32_t c[kPer], mine = 0;
    for (uint32_t j = 0; j < kPer; ++j) {
        const uint32_t s = tid * kPer + j;
        const uint32_t x = s < nseg ? w.segoff[s] : kHpDead;
        c[j] = x != kHpDead ? w.cntm[s * kHpCand + x] : 0u;
        mine += c[j];
    }
    uint32_t incl = mine;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t v = __shfl_up(incl, d);
        if ((int)(tid & 63) >= d) incl += v;
    }
    if ((tid & 63) == 63) part[tid >> 6] = incl;
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (uint32_t k = 0; k < nt / 64; ++k) {
        before += k < (tid >> 6) ? part[k] : 0u;
        total += part[k];
    }
    uint32_t run = before + incl - mine;
    for (uint32_t j = 0; j < kPer; ++j) {
        const uint32_t s = tid * kPer + j;
        if (s < nseg) w.base[s] = run;
        run += c[j];
    }
    if (tid == 0) w.st[0] = total;
}

constexpr int kHpEmitThreads = 64;

__global__ __launch_bounds__(kHpEmitThreads) void k_hdr_emit(const uint8_t* __restrict__ f, uint64_t len,
                                                              hz_codebook* __restrict__ cb, unsigned long long* wsp) {
    __shared__ uint32_t wl[kHpWords];
    __shared__ uint16_t pos[kHpSeg / 25 + 8];
    const HpWs w = hp_ws(wsp);
    const uint32_t lane = threadIdx.x, seg = blockIdx.x;
    const HpGeo g = hp_geo(f, len);
    if (!g.ok || seg >= g.nseg) return;
    const uint32_t o = w.segoff[seg], base = w.base[seg];
    if (o == kHpDead || base >= g.U) return;
    const uint32_t k = seg * kHpCand + o;
    const uint32_t cnt = w.cntm[k], n = cnt < g.U - base ? cnt : g.U - base;
    hp_load(wl, f, len, g.p0 / 8 + (uint64_t)seg * (kHpSeg / 8));
    __syncthreads();
    if (lane < kHpSub) {  // the sub-segments of the true path, each from its known offset and entry number
        const uint32_t x = w.sub[16ull * k + lane], cum = w.sub[16ull * k + 8 + lane];
        if (x != kHpDead) {
            uint32_t p = lane * kHpSubBits + x, j = cum;
            const uint32_t end = (lane + 1) * kHpSubBits;
            while (p < end) {
                const uint32_t L = (hp_bits32(wl, p) >> 8) & 0xffu;
                if (L - 1u >= (uint32_t)HZ_MAXLEN) break;
                pos[j++] = (uint16_t)p;
                p += 24 + L;
            }
        }
    }
    __syncthreads();
    uint32_t mx = 0, mn = 255;
    for (uint32_t e = lane; e < n; e += kHpEmitThreads) {
        const uint32_t p = pos[e], head = hp_bits32(wl, p) >> 8, sym = head >> 8, L = head & 0xffu;
        const uint64_t hi = hp_bits32(wl, p + 24), lo = hp_bits32(wl, p + 56);
        const uint64_t code = ((hi << 32) | lo) >> (64 - L);  // 1 <= L <= 56
        const uint32_t i = base + e;
        if (atomicOr(&w.seen[sym >> 5], 1u << (sym & 31)) & (1u << (sym & 31))) atomicOr(&w.st[2], 1ull);
        cb->order[i] = (uint16_t)sym;
        cb->len[sym] = (uint8_t)L;
        cb->code[sym] = code;
        mx = L > mx ? L : mx;
        mn = L < mn ? L : mn;
        if (i == g.U - 1) w.st[1] = (uint64_t)seg * kHpSeg + p + 24 + L;
    }
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t a = __shfl_xor(mx, d), b = __shfl_xor(mn, d);
        mx = a > mx ? a : mx;
        mn = b < mn ? b : mn;
    }
    if (lane == 0) {
        atomicMax(&w.st[3], (unsigned long long)mx);
        atomicMin(&w.st[4], (unsigned long long)mn);
    }
}

// Bits [p, p + nb) of the file, nb <= 56, read byte-wise (zeros past len).
HZ_DEV uint64_t file_bits(const uint8_t* f, uint64_t len, uint64_t p, uint32_t nb) {
    const uint64_t b0 = p >> 3;
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) v = (v << 8) | (b0 + k < len ? f[b0 + k] : 0u);
    return (v << (p & 7)) >> (64 - nb);
}

// info (device): [0] n, [1] payload byte, [2] payload bit, [3] is_odd, [4] last byte, [5] nsym
__global__ __launch_bounds__(64) void k_hdr_finish(const uint8_t* __restrict__ f, uint64_t len,
                                                   hz_codebook* __restrict__ cb, unsigned long long* info,
                                                   unsigned long long* wsp, uint32_t* err) {
    if (threadIdx.x) return;
    const HpWs w = hp_ws(wsp);
    const HpGeo g = hp_geo(f, len);
    if (!g.ok || w.st[0] < g.U || w.st[2]) {  // short file, an invalid length or a truncation before entry U, a duplicate
        atomicOr(err, 2u);
        return;
    }
    uint64_t p = g.p0 + (g.U ? w.st[1] : 0);
    if ((p + 64 + 7) / 8 > len) {
        atomicOr(err, 2u);
        return;
    }
    const uint64_t n = file_bits(f, len, p, 32) << 32 | file_bits(f, len, p + 32, 32);  // N, stream order
    uint64_t nn = 0;  // 8 LE bytes, each MSB first
    for (int b = 0; b < 8; ++b) nn |= ((n >> (56 - 8 * b)) & 0xffu) << (8 * b);
    p += 64;
    if (nn / 2 > 0 && g.U == 0) {
        atomicOr(err, 2u);
        return;
    }
    cb->nsym = g.U;
    cb->max_len = g.U ? (uint32_t)w.st[3] : 0;
    cb->min_len = g.U ? (uint32_t)w.st[4] : 0;
    cb->reserved = 0;
    info[0] = nn;
    info[1] = p >> 3;
    info[2] = p & 7;
    info[3] = g.odd;
    info[4] = g.odd ? f[3] : 0;
    info[5] = g.U;
}

hipError_t launch_header_write(const hz_codebook* d_cb, uint64_t n, uint32_t last_byte, uint8_t* d_out, uint64_t cap,
                               unsigned long long* d_info, unsigned long long* d_ws, uint32_t* d_err, hipStream_t s) {
    unsigned long long* w = d_ws + codebook_ws_words() - 256;  // the workspace's last 256 words
    hipLaunchKernelGGL(k_hw_sum, dim3(kHwGroups), dim3(kHwThreads), 0, s, d_cb, w);
    hipLaunchKernelGGL(k_hw_prep, dim3(1), dim3(64), 0, s, d_cb, n, d_out, cap, d_info, w, d_err);
    hipLaunchKernelGGL(k_hw_write, dim3(kHwGroups), dim3(kHwThreads), 0, s, d_cb, n, last_byte, d_out, w);
    return hipGetLastError();
}

hipError_t launch_header_parse(const uint8_t* d_file, uint64_t len, hz_codebook* d_cb, unsigned long long* d_info,
                               unsigned long long* d_ws, uint32_t* d_err, hipStream_t s) {
    // grid: the most segments `len` bytes can hold (the kernels take the true count from the header)
    const uint64_t avail = len > 3 ? 8 * (len - 3) : 0, bound = avail < 65536ull * kHpCand ? avail : 65536ull * kHpCand;
    const uint32_t nseg = (uint32_t)((bound + kHpSeg - 1) / kHpSeg);
    const uint32_t grid = nseg > 128 ? nseg : 128;  // at least enough blocks to zero the codebook quickly
    hipLaunchKernelGGL(k_hdr_seg, dim3(grid), dim3(kHpSegThreads), 0, s, d_file, len, d_cb, d_ws);
    const int lds = (int)(kHpMaxSeg * kHpCand);
    hipError_t e = hipFuncSetAttribute((const void*)k_hdr_chain, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_hdr_chain, dim3(1), dim3(kHpChainThreads), lds, s, d_file, len, d_ws);
    if (nseg) hipLaunchKernelGGL(k_hdr_emit, dim3(nseg), dim3(kHpEmitThreads), 0, s, d_file, len, d_cb, d_ws);
    hipLaunchKernelGGL(k_hdr_finish, dim3(1), dim3(64), 0, s, d_file, len, d_cb, d_info, d_ws, d_err);
    return hipGetLastError();
}

hipError_t launch_codebook(const unsigned long long* d_hist, hz_codebook* d_cb, unsigned long long* d_ws,
                           uint32_t* d_err, hipStream_t s) {
    static_assert(kCbPasses == 6, "one launch per pass");
    hipLaunchKernelGGL(k_cb_keys, dim3(kCbTiles), dim3(kCbTileKeys), 0, s, d_hist, d_cb, d_ws);
    hipLaunchKernelGGL(k_cb_scatter<0>, dim3(kCbTiles), dim3(kCbTileKeys), 0, s, d_cb, d_ws);
    hipLaunchKernelGGL(k_cb_scatter<1>, dim3(kCbTiles), dim3(kCbTileKeys), 0, s, d_cb, d_ws);
    hipLaunchKernelGGL(k_cb_scatter<2>, dim3(kCbTiles), dim3(kCbTileKeys), 0, s, d_cb, d_ws);
    hipLaunchKernelGGL(k_cb_scatter<3>, dim3(kCbTiles), dim3(kCbTileKeys), 0, s, d_cb, d_ws);
    hipLaunchKernelGGL(k_cb_scatter<4>, dim3(kCbTiles), dim3(kCbTileKeys), 0, s, d_cb, d_ws);
    hipLaunchKernelGGL(k_cb_scatter<5>, dim3(kCbTiles), dim3(kCbTileKeys), 0, s, d_cb, d_ws);
    const int lds = (int)((2 * kCgT + kCgT / 2) * sizeof(unsigned long long));
    hipError_t e = hipFuncSetAttribute((const void*)k_cb_generate, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_cb_generate, dim3(1), dim3(kCgThreads), lds, s, d_cb, d_ws, d_err);
    hipLaunchKernelGGL(k_cb_leaves, dim3(kCbTiles), dim3(kCbTileKeys), 0, s, d_cb, d_ws, d_err);
    return hipGetLastError();
}

// Workspace (u64 words) shared by the codebook build and the header parse.
uint64_t codebook_ws_words() {
    const uint64_t hp = (18ull * kHpMaxSeg * kHpCand + 5ull * (kHpMaxSeg + 64) + 4 * 2048 + 64) / 8 + 8;
    return (kCbWsWords > hp ? kCbWsWords : hp) + 256;  // + the header writer's scan
}

}  // namespace hz
