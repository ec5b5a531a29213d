// hz_codebook_gpu.hip -- the codebook and the header on the device (SURVEY.md
// 8f-2, 8f-4): gfx950 kernels with the reference's semantics, so a device
// histogram becomes a codebook and a .compressed header without a host hop.
//
//   k_codebook      65 536-bin histogram -> codebook (hz_codebook layout) in
//                   ONE workgroup: bitonic sort of (count << 16 | symbol)
//                   keys (thrust's stable order, Compressor.cu:378-425), then
//                   GenerateCL's rounds (gpuHuffmanConstruction.h:353-466:
//                   pivot by binary search, pairs (2i, 2i + 1) of the sorted
//                   list become internal nodes, a stable merge of the rest with
//                   the new nodes, older nodes first on ties), then GenerateCW
//                   top-down by round (h:468-494, first child '1',
//                   toCpu h:551-579). No grid barrier: every round is one
//                   workgroup barrier.
//   k_header_write  the header (Compressor.cu:431-487, writers :637-669): one
//                   thread per codebook entry at its scanned bit offset,
//                   words ORed together.
//   k_header_parse  the header (Decompressor.cu:65-103): one wave finds the
//                   entry positions (each needs the previous length; 256
//                   header bytes at a time in registers, read by lane reads),
//                   then the workgroup decodes every entry at its position.
#include <stdint.h>

#include "huffman_amd.h"
#include "hz_internal.h"

namespace hz {

#define HZ_DEV __device__ __forceinline__

constexpr int kCbThreads = 1024;
constexpr uint32_t kCbTile = 16384;  // bitonic passes with j < kCbTile run in LDS, a tile at a time

// Workspace of k_codebook in device memory (u64 words): keys, two node lists
// (freq + id), the new nodes of a round, children, per-node code and length,
// round starts.
uint64_t codebook_ws_words() { return 65536 + 2 * (65536 + 32768) + (65536 + 32768) + 65536 + 2 * 65536 + 16384 + 32768 + 64; }

struct CbWs {
    unsigned long long* keys;  // 65536
    unsigned long long* fa;    // list A freq
    uint32_t* ia;              // list A id
    unsigned long long* fb;
    uint32_t* ib;
    unsigned long long* fr;    // new nodes of the round (freq)
    uint32_t* ir;              // and id
    uint32_t* child;           // 2 per internal node
    unsigned long long* ncode; // per node (2U - 1)
    uint8_t* nlen;
    uint32_t* rounds;          // first internal node id of each round
};

HZ_DEV CbWs cb_ws(unsigned long long* w) {
    CbWs s;
    s.keys = w; w += 65536;
    s.fa = w; w += 65536;
    s.ia = reinterpret_cast<uint32_t*>(w); w += 32768;
    s.fb = w; w += 65536;
    s.ib = reinterpret_cast<uint32_t*>(w); w += 32768;
    s.fr = w; w += 65536;
    s.ir = reinterpret_cast<uint32_t*>(w); w += 32768;
    s.child = reinterpret_cast<uint32_t*>(w); w += 65536;
    s.ncode = w; w += 2 * 65536;
    s.nlen = reinterpret_cast<uint8_t*>(w); w += 16384;
    s.rounds = reinterpret_cast<uint32_t*>(w);  // up to U rounds (a degenerate histogram pairs two nodes a round)
    return s;
}

HZ_DEV void cmp_swap(unsigned long long& a, unsigned long long& b, bool up) {
    const unsigned long long lo = a < b ? a : b, hi = a < b ? b : a;
    a = up ? lo : hi;
    b = up ? hi : lo;
}

// Bitonic passes j = j_hi .. 1 of stage k on one kCbTile-key tile in LDS.
HZ_DEV void tile_passes(unsigned long long* t, uint32_t base, uint32_t k, uint32_t j_hi) {
    for (uint32_t j = j_hi; j >= 1; j >>= 1) {
        for (uint32_t p = threadIdx.x; p < kCbTile / 2; p += blockDim.x) {
            const uint32_t i = (p / j) * 2 * j + (p % j);  // first of the pair (bit j clear)
            unsigned long long a = t[i], b = t[i + j];
            cmp_swap(a, b, ((base + i) & k) == 0);
            t[i] = a;
            t[i + j] = b;
        }
        __syncthreads();
    }
}

// Stable-merge co-rank (left wins ties): how many of the first q outputs come from L.
HZ_DEV uint32_t co_rank(const unsigned long long* L, uint32_t nl, const unsigned long long* R, uint32_t nr,
                        uint32_t q) {
    uint32_t lo = q > nr ? q - nr : 0, hi = q < nl ? q : nl;
    while (lo < hi) {
        const uint32_t x = (lo + hi + 1) / 2;  // try taking x from L
        // x feasible iff L[x-1] <= R[q-x] (L's x-th comes before R's (q-x+1)-th)
        if (q - x >= nr || L[x - 1] <= R[q - x]) lo = x;
        else hi = x - 1;
    }
    return lo;
}

__global__ __launch_bounds__(kCbThreads) void k_codebook(const unsigned long long* __restrict__ hist,
                                                         hz_codebook* __restrict__ cb, unsigned long long* wsp,
                                                         uint32_t* err) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lds64[];
    __shared__ uint32_t sh_u, sh_pivot, sh_bad, sh_max, sh_min;
    const CbWs w = cb_ws(wsp);
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    if (tid == 0) { sh_u = 0; sh_bad = 0; sh_max = 0; sh_min = 255; }
    __syncthreads();
    // keys in symbol order; a sort of unique (count, symbol) keys is thrust's stable order
    uint32_t u = 0;
    for (uint32_t s = tid; s < 65536; s += nt) {
        const unsigned long long h = hist[s];
        if (h >> 47) atomicOr(&sh_bad, 1u);
        w.keys[s] = (h << 16) | s;
        u += h != 0;
    }
    atomicAdd(&sh_u, u);
    __syncthreads();
    const uint32_t U = sh_u;
    if (sh_bad) {
        if (tid == 0) atomicOr(err, 16u);
        return;
    }
    // ---- bitonic sort of the 65 536 keys: stages up to kCbTile in LDS, then global passes + LDS tails
    for (uint32_t tb = 0; tb < 65536; tb += kCbTile) {
        for (uint32_t i = tid; i < kCbTile; i += nt) lds64[i] = w.keys[tb + i];
        __syncthreads();
        for (uint32_t k = 2; k <= kCbTile; k <<= 1) tile_passes(lds64, tb, k, k / 2);
        for (uint32_t i = tid; i < kCbTile; i += nt) w.keys[tb + i] = lds64[i];
        __syncthreads();
    }
    for (uint32_t k = 2 * kCbTile; k <= 65536; k <<= 1) {
        for (uint32_t j = k / 2; j >= kCbTile; j >>= 1) {
            for (uint32_t p = tid; p < 32768; p += nt) {
                const uint32_t i = (p / j) * 2 * j + (p % j);
                unsigned long long a = w.keys[i], b = w.keys[i + j];
                cmp_swap(a, b, (i & k) == 0);
                w.keys[i] = a;
                w.keys[i + j] = b;
            }
            __syncthreads();
        }
        for (uint32_t tb = 0; tb < 65536; tb += kCbTile) {
            for (uint32_t i = tid; i < kCbTile; i += nt) lds64[i] = w.keys[tb + i];
            __syncthreads();
            tile_passes(lds64, tb, k, kCbTile / 2);
            for (uint32_t i = tid; i < kCbTile; i += nt) w.keys[tb + i] = lds64[i];
            __syncthreads();
        }
    }
    // ---- leaves: the nonzero tail of the sorted keys (Compressor.cu:414,419-425)
    const uint32_t z = 65536 - U;
    for (uint32_t i = tid; i < U; i += nt) {
        const unsigned long long key = w.keys[z + i];
        w.fa[i] = key >> 16;
        w.ia[i] = i;
        cb->order[i] = (uint16_t)(key & 0xffff);
    }
    for (uint32_t s = tid; s < 65536; s += nt) {
        cb->len[s] = 0;
        cb->code[s] = 0;
    }
    __syncthreads();
    if (U <= 1) {  // U == 1: code "0" (the reference's defect B4)
        if (tid == 0) {
            cb->nsym = U;
            cb->max_len = cb->min_len = U;
            cb->reserved = 0;
            if (U == 1) { cb->len[cb->order[0]] = 1; cb->code[cb->order[0]] = 0; }
        }
        return;
    }
    // ---- GenerateCL rounds
    unsigned long long* fa = w.fa;
    uint32_t* ia = w.ia;
    unsigned long long* fb = w.fb;
    uint32_t* ib = w.ib;
    uint32_t size = U, cur = U, nr = 0;
    while (size > 1) {
        if (tid == 0) {  // BinarySearch (h:137-151) over f[2..size): first > f0 + f1, capped
            const unsigned long long spec = fa[0] + fa[1];
            uint32_t l = 0, r = size > 2 ? size - 3 : 0;
            while (l < r) {
                const uint32_t m = l + (r - l) / 2;
                if (fa[2 + m] <= spec) l = m + 1;
                else r = m;
            }
            const uint32_t pv = l + 2;
            sh_pivot = pv - (pv & 1);
            w.rounds[nr] = cur;
        }
        __syncthreads();
        const uint32_t pivot = sh_pivot, half = pivot >> 1, nl = size - pivot, out = nl + half;
        for (uint32_t i = tid; i < half; i += nt) {  // pairs (2i, 2i + 1) -> node cur + i
            w.fr[i] = fa[2 * i] + fa[2 * i + 1];
            w.ir[i] = cur + i;
            w.child[2 * (cur + i - U)] = ia[2 * i];
            w.child[2 * (cur + i - U) + 1] = ia[2 * i + 1];
        }
        __syncthreads();
        // stable merge of the rest [pivot, size) with the new nodes (ParallelMerge h:263-351)
        const uint32_t per = (out + nt - 1) / nt;
        const uint32_t q0 = tid * per < out ? tid * per : out, q1 = q0 + per < out ? q0 + per : out;
        if (q0 < q1) {
            const unsigned long long* L = fa + pivot;
            const uint32_t* Li = ia + pivot;
            uint32_t x = co_rank(L, nl, w.fr, half, q0), y = q0 - x;
            for (uint32_t q = q0; q < q1; ++q) {
                const bool left = y >= half || (x < nl && L[x] <= w.fr[y]);
                fb[q] = left ? L[x] : w.fr[y];
                ib[q] = left ? Li[x] : w.ir[y];
                x += left;
                y += !left;
            }
        }
        __syncthreads();
        cur += half;
        size = out;
        ++nr;
        unsigned long long* tf = fa; fa = fb; fb = tf;
        uint32_t* ti = ia; ia = ib; ib = ti;
    }
    if (tid == 0) w.rounds[nr] = cur;  // cur == 2U - 1
    // ---- GenerateCW top-down, round by round from the root
    if (tid == 0) { w.ncode[2 * U - 2] = 0; w.nlen[2 * U - 2] = 0; }
    __syncthreads();
    for (int r = (int)nr - 1; r >= 0; --r) {
        const uint32_t b = w.rounds[r], e = w.rounds[r + 1];
        for (uint32_t p = b + tid; p < e; p += nt) {
            const unsigned long long c = w.ncode[p];
            const uint32_t L = w.nlen[p] + 1u;
            const uint32_t c0 = w.child[2 * (p - U)], c1 = w.child[2 * (p - U) + 1];
            w.ncode[c0] = (c << 1) | 1u;  // first child '1'
            w.ncode[c1] = c << 1;         // second child '0'
            w.nlen[c0] = (uint8_t)(L < 255 ? L : 255);
            w.nlen[c1] = (uint8_t)(L < 255 ? L : 255);
        }
        __syncthreads();
    }
    uint32_t mx = 0, mn = 255;
    for (uint32_t i = tid; i < U; i += nt) {
        const uint32_t s = cb->order[i], L = w.nlen[i];
        cb->len[s] = (uint8_t)L;
        cb->code[s] = w.ncode[i];
        mx = L > mx ? L : mx;
        mn = L < mn ? L : mn;
    }
    atomicMax(&sh_max, mx);
    atomicMin(&sh_min, mn);
    __syncthreads();
    if (tid == 0) {
        cb->nsym = U;
        cb->max_len = sh_max;
        cb->min_len = sh_min;
        cb->reserved = 0;
        if (sh_max > HZ_MAXLEN) atomicOr(err, 32u);
    }
}

// ---- header writer ---------------------------------------------------------
// Bit stream MSB first: bit b of the header is bit 7 - b % 8 of byte b / 8.
// `put` ORs the low `nb` (<= 64) bits of v, first bit = bit nb - 1, at bit b.
HZ_DEV void hdr_put(uint32_t* w32, uint64_t b, uint64_t v, uint32_t nb) {
    while (nb) {
        const uint32_t off = (uint32_t)(b & 31), take = 32 - off < nb ? 32 - off : nb;
        const uint32_t bits = (uint32_t)(v >> (nb - take)) & (take == 32 ? 0xffffffffu : ((1u << take) - 1u));
        const uint32_t be = bits << (32 - off - take);  // big-endian word value
        atomicOr(&w32[b >> 5], __builtin_bswap32(be));
        b += take;
        nb -= take;
    }
}

constexpr int kHdrThreads = 1024;

// info (device): [0] complete header bytes, [1] pending bits, [2] pending byte (MSB aligned), [3] header bits
__global__ __launch_bounds__(kHdrThreads) void k_header_write(const hz_codebook* __restrict__ cb, uint64_t n,
                                                              uint32_t last_byte, uint8_t* out, uint64_t cap,
                                                              unsigned long long* info, uint32_t* err) {
    __shared__ unsigned long long part[kHdrThreads + 1];
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint32_t U = cb->nsym;
    const uint32_t odd = (uint32_t)(n & 1);
    const uint32_t per = (U + nt - 1) / nt, i0 = tid * per < U ? tid * per : U, i1 = i0 + per < U ? i0 + per : U;
    unsigned long long mine = 0;
    for (uint32_t i = i0; i < i1; ++i) mine += 24u + cb->len[cb->order[i]];
    part[tid] = mine;
    __syncthreads();
    if (tid == 0) {  // exclusive scan of the per-thread sums (1024 values)
        unsigned long long acc = 8ull * (3 + odd);
        for (uint32_t t = 0; t < nt; ++t) { const unsigned long long v = part[t]; part[t] = acc; acc += v; }
        part[nt] = acc + 64;  // + N
    }
    __syncthreads();
    const unsigned long long total = part[nt];
    const uint64_t words = (total + 31) / 32;
    if (words * 4 > cap) {
        if (tid == 0) atomicOr(err, 4u);
        return;
    }
    uint32_t* w32 = reinterpret_cast<uint32_t*>(out);
    for (uint64_t k = tid; k < words; k += nt) w32[k] = 0;
    __syncthreads();
    if (tid == 0) {
        hdr_put(w32, 0, U & 0xffffu ? ((U & 0xffu) << 8) | ((U >> 8) & 0xffu) : 0u, 16);  // u16 LE (:434)
        hdr_put(w32, 16, odd, 8);                                                          // isOdd (:438)
        if (odd) hdr_put(w32, 24, last_byte & 0xffu, 8);                                   // lastByte (:439-443)
        uint64_t nn = n;                                                                   // writeFileSize (:661-669)
        for (int k = 0; k < 8; ++k, nn >>= 8) hdr_put(w32, total - 64 + 8 * k, nn & 0xff, 8);
    }
    unsigned long long b = part[tid];
    for (uint32_t i = i0; i < i1; ++i) {  // writeFromUShort, writeFromUChar, code bits (:454-483)
        const uint32_t sym = cb->order[i], L = cb->len[sym];
        hdr_put(w32, b, ((uint64_t)sym << 8) | L, 24);
        hdr_put(w32, b + 24, cb->code[sym], L);
        b += 24 + L;
    }
    __syncthreads();
    if (tid == 0) {
        // the words were built by atomics at L2: read the pending byte the same way
        const uint32_t wv = atomicOr(&w32[(total / 8) / 4], 0u);
        info[0] = total / 8;
        info[1] = total % 8;
        info[2] = (total % 8) ? (wv >> (8 * ((total / 8) % 4))) & 0xffu : 0;
        info[3] = total;
    }
}

// ---- header parser: one wave walks the entries over a 256-byte register window
// info (device): [0] n, [1] payload byte, [2] payload bit, [3] is_odd, [4] last byte, [5] nsym
struct HdrWin {
    uint32_t w;        // this lane's big-endian word of the window
    uint64_t base;     // bit of the window's first bit
};

HZ_DEV uint32_t hdr_word_be(const uint8_t* f, uint64_t len, uint64_t byte) {
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) v = (v << 8) | (byte + k < len ? f[byte + k] : 0u);
    return v;
}

// 32 bits at bit p (p - base < 2016): two lane reads and a funnel shift (uniform values: scalar registers)
HZ_DEV uint32_t hdr_bits32(const HdrWin& win, uint64_t p) {
    const uint32_t d = (uint32_t)(p - win.base), wi = d >> 5, sh = d & 31;
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)win.w, (int)wi);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)win.w, (int)(wi + 1 < 64 ? wi + 1 : 63));
    return sh ? (hi << sh) | (lo >> (32 - sh)) : hi;
}

// Bits [p, p + nb) of the file, nb <= 56, read byte-wise (zeros past len).
HZ_DEV uint64_t file_bits(const uint8_t* f, uint64_t len, uint64_t p, uint32_t nb) {
    const uint64_t b0 = p >> 3;
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) v = (v << 8) | (b0 + k < len ? f[b0 + k] : 0u);
    return (v << (p & 7)) >> (64 - nb);
}

constexpr int kParseThreads = 1024;

// Phase A, one wave: the entry positions (each needs the previous length),
// 2048 header bits at a time in registers, read by lane reads. Phase B, the
// whole workgroup: every entry decoded at its position, duplicates caught by a
// symbol bitmap.
__global__ __launch_bounds__(kParseThreads) void k_header_parse(const uint8_t* __restrict__ f, uint64_t len,
                                                                hz_codebook* __restrict__ cb, unsigned long long* info,
                                                                uint32_t* ws, uint32_t* err) {
    __shared__ uint32_t seen[2048];  // 65 536-symbol bitmap
    __shared__ uint32_t sh_bad, sh_max, sh_min;
    __shared__ unsigned long long sh_end;
    const uint32_t tid = threadIdx.x, nt = blockDim.x, lane = tid & 63;
    for (uint32_t s = tid; s < 65536; s += nt) { cb->len[s] = 0; cb->code[s] = 0; }
    for (uint32_t i = tid; i < 2048; i += nt) seen[i] = 0;
    if (tid == 0) { sh_bad = 0; sh_max = 0; sh_min = 255; sh_end = 0; }
    __syncthreads();
    if (len < 3 || (f[2] != 0 && len < 4)) {
        if (tid == 0) atomicOr(err, 2u);
        return;
    }
    uint32_t U = (uint32_t)f[0] | ((uint32_t)f[1] << 8);  // Decompressor.cu:69-71
    const uint32_t odd = f[2] != 0;                        // :76
    const uint64_t pre = odd ? 4 : 3;
    if (U == 0) U = (len == pre + 8) ? 0 : 65536;          // U 0 => 65536 (and the empty-file convention)
    if (tid < 64) {
        HdrWin win;
        auto load = [&](uint64_t bit) {
            win.base = bit & ~31ull;
            win.w = hdr_word_be(f, len, win.base / 8 + 4ull * lane);
        };
        uint64_t p = 8 * pre;
        load(p);
        uint32_t bad = 0;
        for (uint32_t i = 0; i < U; ++i) {
            if (p - win.base > 2048 - 128) load(p);
            const uint32_t L = (hdr_bits32(win, p) >> 8) & 0xffu;
            if (L == 0 || L > HZ_MAXLEN || (p + 24 + L + 64 + 7) / 8 > len) { bad = 1; break; }
            if (lane == 0) ws[i] = (uint32_t)p;  // header < 2^32 bits
            p += 24 + L;
        }
        if (lane == 0) {
            sh_bad = bad;
            sh_end = p;
        }
    }
    __syncthreads();
    if (sh_bad) {
        if (tid == 0) atomicOr(err, 2u);
        return;
    }
    uint32_t mx = 0, mn = 255;
    for (uint32_t i = tid; i < U; i += nt) {
        const uint64_t p = ws[i];
        const uint32_t head = (uint32_t)file_bits(f, len, p, 24);
        const uint32_t sym = head >> 8, L = head & 0xffu;
        if (atomicOr(&seen[sym >> 5], 1u << (sym & 31)) & (1u << (sym & 31))) atomicOr(&sh_bad, 1u);  // duplicate
        cb->order[i] = (uint16_t)sym;
        cb->len[sym] = (uint8_t)L;
        cb->code[sym] = file_bits(f, len, p + 24, L);
        mx = L > mx ? L : mx;
        mn = L < mn ? L : mn;
    }
    atomicMax(&sh_max, mx);
    atomicMin(&sh_min, mn);
    __syncthreads();
    if (tid == 0) {
        uint64_t p = sh_end;
        const uint64_t n = file_bits(f, len, p, 32) << 32 | file_bits(f, len, p + 32, 32);  // N, stream order
        uint64_t nn = 0;  // 8 LE bytes, each MSB first
        for (int b = 0; b < 8; ++b) nn |= ((n >> (56 - 8 * b)) & 0xffu) << (8 * b);
        p += 64;
        if ((p + 7) / 8 > len || (nn / 2 > 0 && U == 0) || sh_bad) {
            atomicOr(err, 2u);
        } else {
            cb->nsym = U;
            cb->max_len = U ? sh_max : 0;
            cb->min_len = U ? sh_min : 0;
            cb->reserved = 0;
            info[0] = nn;
            info[1] = p >> 3;
            info[2] = p & 7;
            info[3] = odd;
            info[4] = odd ? f[3] : 0;
            info[5] = U;
        }
    }
}

hipError_t launch_header_write(const hz_codebook* d_cb, uint64_t n, uint32_t last_byte, uint8_t* d_out, uint64_t cap,
                               unsigned long long* d_info, uint32_t* d_err, hipStream_t s) {
    hipLaunchKernelGGL(k_header_write, dim3(1), dim3(kHdrThreads), 0, s, d_cb, n, last_byte, d_out, cap, d_info, d_err);
    return hipGetLastError();
}

hipError_t launch_header_parse(const uint8_t* d_file, uint64_t len, hz_codebook* d_cb, unsigned long long* d_info,
                               unsigned long long* d_ws, uint32_t* d_err, hipStream_t s) {
    hipLaunchKernelGGL(k_header_parse, dim3(1), dim3(kParseThreads), 0, s, d_file, len, d_cb, d_info,
                       reinterpret_cast<uint32_t*>(d_ws), d_err);
    return hipGetLastError();
}

hipError_t launch_codebook(const unsigned long long* d_hist, hz_codebook* d_cb, unsigned long long* d_ws,
                           uint32_t* d_err, hipStream_t s) {
    const int lds = (int)(kCbTile * sizeof(unsigned long long));
    hipError_t e = hipFuncSetAttribute((const void*)k_codebook, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_codebook, dim3(1), dim3(kCbThreads), lds, s, d_hist, d_cb, d_ws, d_err);
    return hipGetLastError();
}

}  // namespace hz
