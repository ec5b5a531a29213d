// hz_codebook.cpp -- host codebook, header bit-writer / parser and the device
// table images (encode and decode) built from a codebook.
//
// The codebook follows the reference GPU encoder exactly:
//   order : thrust::sequence + stable sort_by_key of (count, symbol)
//           (Compressor.cu:387-393,414,419-425)  -> (count asc, symbol asc)
//   tree  : GenerateCL (gpuHuffmanConstruction.h:353-466) == sequential
//           Huffman whose picks are the two smallest (count, age) nodes, leaves
//           older than internals; pinned by oracle/generatecl_literal.py
//   bits  : first child '1', second '0', root first (GenerateCW h:468-494 +
//           toCpu h:562-574)
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <queue>
#include <vector>

#include "huffman_amd.h"
#include "hz_internal.h"

namespace {

// LSD radix sort of u64 keys, 11-bit digits (a 2048-entry count table stays
// in L1) over bits [lo, highest set bit]; a digit every key shares is skipped.
// `tmp` is scratch of k's size. Stable.
void radix_sort_u64(uint64_t* k, uint64_t* tmp, uint32_t n, int lo) {
    if (n < 2) return;
    uint64_t mx = 0;
    for (uint32_t i = 0; i < n; ++i) mx |= k[i];
    const int bits = 64 - __builtin_clzll(mx | 1);
    uint32_t cnt[2048];
    uint64_t* const out = k;
    for (int sh = lo; sh < bits; sh += 11) {
        memset(cnt, 0, sizeof(cnt));
        for (uint32_t i = 0; i < n; ++i) cnt[(k[i] >> sh) & 2047]++;
        if (cnt[(k[0] >> sh) & 2047] == n) continue;  // one digit value: already in order
        uint32_t sum = 0;
        for (auto& c : cnt) { const uint32_t t = c; c = sum; sum += t; }
        for (uint32_t i = 0; i < n; ++i) tmp[cnt[(k[i] >> sh) & 2047]++] = k[i];
        std::swap(k, tmp);
    }
    if (k != out) memcpy(out, k, (size_t)n * sizeof(uint64_t));  // the result is in the scratch
}

// Per-thread scratch of the codebook builder (no zero-fill per call).
struct CbScratch {
    std::unique_ptr<uint64_t[]> keys{new uint64_t[HZ_NSYM]}, tmp{new uint64_t[HZ_NSYM]};
    std::unique_ptr<uint64_t[]> f{new uint64_t[2 * HZ_NSYM]}, cw{new uint64_t[2 * HZ_NSYM]};
    std::unique_ptr<uint32_t[]> up{new uint32_t[2 * HZ_NSYM]};
    std::unique_ptr<uint8_t[]> dep{new uint8_t[2 * HZ_NSYM]};
};

struct BitWriter {
    uint8_t* p;
    uint64_t cap, pos = 0;
    uint64_t acc = 0;
    int nacc = 0;
    bool overflow = false;
    void put(uint64_t v, int nbits) {
        while (nbits > 0) {
            int take = nbits > 32 ? 32 : nbits;
            uint64_t part = (v >> (nbits - take)) & ((1ull << take) - 1);
            acc = (acc << take) | part;
            nacc += take;
            nbits -= take;
            while (nacc >= 8) {
                nacc -= 8;
                if (pos < cap) p[pos] = (uint8_t)(acc >> nacc);
                else overflow = true;
                pos++;
            }
        }
    }
};

struct BitReader {
    const uint8_t* p;
    uint64_t len, bit = 0;
    bool eof = false;
    uint64_t get(int n) {
        uint64_t v = 0;
        for (int i = 0; i < n; ++i) {
            if ((bit >> 3) >= len) { eof = true; return 0; }
            v = (v << 1) | ((p[bit >> 3] >> (7 - (bit & 7))) & 1);
            bit++;
        }
        return v;
    }
};

}  // namespace

extern "C" int hz_codebook_build(const uint64_t* hist, hz_codebook* cb) {
    if (!hist || !cb) return HZ_EINVAL;
    memset(cb->len, 0, sizeof(cb->len));
    memset(cb->code, 0, sizeof(cb->code));
    cb->nsym = cb->max_len = cb->min_len = 0;
    thread_local CbScratch sc;
    uint64_t* keys = sc.keys.get();
    uint32_t U = 0;
    for (uint32_t s = 0; s < HZ_NSYM; ++s) {
        if (hist[s]) {
            if (hist[s] >> 47) return HZ_EINVAL;  // > 2^47 symbols: out of range
            keys[U++] = (hist[s] << 16) | s;
        }
    }
    cb->nsym = U;
    if (U == 0) return HZ_OK;
    // keys were built in symbol order: a stable sort by count == (count, symbol) order (thrust's)
    radix_sort_u64(keys, sc.tmp.get(), U, 16);
    for (uint32_t i = 0; i < U; ++i) cb->order[i] = (uint16_t)(keys[i] & 0xffff);
    if (U == 1) {  // reference defect B4: its code would be empty; use "0"
        cb->len[cb->order[0]] = 1;
        cb->code[cb->order[0]] = 0;
        cb->max_len = cb->min_len = 1;
        return HZ_OK;
    }
    // Merge with two FIFO queues (leaves by (count, symbol), then merged nodes in creation
    // order); the leaf head wins a tie. Each node records its parent and the branch bit it
    // hangs on, and the codes are then assigned top-down in reverse creation order.
    const uint32_t nn = 2 * U - 1;
    uint64_t* f = sc.f.get();
    uint32_t* up = sc.up.get();  // parent << 1 | branch bit ('1' for the first child)
    for (uint32_t i = 0; i < U; ++i) f[i] = keys[i] >> 16;
    uint32_t li = 0, qi = U;
    for (uint32_t nx = U; nx < nn; ++nx) {
        auto take = [&]() -> uint32_t {
            const bool leaf = li < U && (qi == nx || f[li] <= f[qi]);
            return leaf ? li++ : qi++;
        };
        const uint32_t a = take(), b = take();
        f[nx] = f[a] + f[b];
        up[a] = nx << 1 | 1u;
        up[b] = nx << 1;
    }
    uint8_t* dep = sc.dep.get();
    uint64_t* cw = sc.cw.get();
    dep[nn - 1] = 0;
    cw[nn - 1] = 0;
    for (uint32_t i = nn - 1; i-- > 0;) {  // a parent is always created after its children
        const uint32_t p = up[i] >> 1, d = dep[p] + 1u;
        if (d > HZ_MAXLEN) return HZ_ETOOLONG;
        dep[i] = (uint8_t)d;
        cw[i] = cw[p] << 1 | (up[i] & 1u);
    }
    uint32_t mx = 0, mn = 255;
    for (uint32_t i = 0; i < U; ++i) {
        const uint32_t s = cb->order[i], d = dep[i];
        cb->len[s] = (uint8_t)d;
        cb->code[s] = cw[i];
        mx = std::max(mx, d);
        mn = std::min(mn, d);
    }
    cb->max_len = mx;
    cb->min_len = mn;
    return HZ_OK;
}

extern "C" int hz_header_bits(const hz_codebook* cb, uint64_t n, uint64_t* bits) {
    if (!cb || !bits) return HZ_EINVAL;
    uint64_t b = 8ull * (3 + (n & 1)) + 64;
    for (uint32_t i = 0; i < cb->nsym; ++i) b += 24 + cb->len[cb->order[i]];
    *bits = b;
    return HZ_OK;
}

extern "C" int hz_payload_bits(const hz_codebook* cb, const uint64_t* hist, uint64_t* bits) {
    if (!cb || !hist || !bits) return HZ_EINVAL;
    uint64_t b = 0;
    for (uint32_t s = 0; s < HZ_NSYM; ++s) b += hist[s] * cb->len[s];
    *bits = b;
    return HZ_OK;
}

// Compressor.cu:431-487 with the writer semantics of :637-669,692-700.
extern "C" int hz_header_write(const hz_codebook* cb, uint64_t n, uint8_t last_byte, uint8_t* out, uint64_t cap,
                               uint64_t* bytes, uint32_t* pending_bits, uint8_t* pending) {
    if (!cb || !out || !bytes || !pending_bits || !pending) return HZ_EINVAL;
    BitWriter w{out, cap};
    w.put(cb->nsym & 0xff, 8);            // fwrite(&uniqueSymbolCount, 2, ...) LE   :434
    w.put((cb->nsym >> 8) & 0xff, 8);
    w.put(n & 1, 8);                      // isOdd                                   :438
    if (n & 1) w.put(last_byte, 8);       // lastByte                                :439-443
    for (uint32_t i = 0; i < cb->nsym; ++i) {
        const uint32_t s = cb->order[i];
        w.put(s, 16);                     // writeFromUShort, high byte first        :463,648-656
        w.put(cb->len[s] & 0xff, 8);      // writeFromUChar(L)                        :465
        w.put(cb->code[s], cb->len[s]);   // code string, first char first           :470-481
    }
    for (int b = 0; b < 8; ++b) w.put((n >> (8 * b)) & 0xff, 8);  // writeFileSize    :487,661-669
    if (w.overflow) return HZ_ECAP;
    *bytes = w.pos;
    *pending_bits = (uint32_t)w.nacc;
    *pending = w.nacc ? (uint8_t)((w.acc << (8 - w.nacc)) & 0xff) : 0;
    return HZ_OK;
}

// Decompressor.cu:65-103 (+ the build's U == 0 convention).
extern "C" int hz_header_parse(const uint8_t* f, uint64_t len, hz_codebook* cb, hz_header_info* info) {
    if (!f || !cb || !info) return HZ_EINVAL;
    if (len < 3) return HZ_EFORMAT;
    uint32_t U = (uint32_t)f[0] | ((uint32_t)f[1] << 8);
    const int odd = f[2] != 0;
    uint64_t pre = 3;
    uint8_t last = 0;
    if (odd) {
        if (len < 4) return HZ_EFORMAT;
        last = f[3];
        pre = 4;
    }
    if (U == 0) U = (len == pre + 8) ? 0 : 65536;
    memset(cb->len, 0, sizeof(cb->len));
    memset(cb->code, 0, sizeof(cb->code));
    cb->nsym = U;
    BitReader r{f, len, pre * 8};
    uint32_t mx = 0, mn = 255;
    for (uint32_t i = 0; i < U; ++i) {
        const uint32_t s = (uint32_t)r.get(16);
        const uint32_t L = (uint32_t)r.get(8);
        if (r.eof) return HZ_EFORMAT;
        if (L == 0 || L > HZ_MAXLEN) return HZ_EFORMAT;  // reference reads 0 as 65536 (:94-95)
        if (cb->len[s]) return HZ_EFORMAT;               // duplicate symbol
        cb->order[i] = (uint16_t)s;
        cb->len[s] = (uint8_t)L;
        cb->code[s] = r.get((int)L);
        mx = std::max(mx, L);
        mn = std::min(mn, L);
    }
    uint64_t n = 0;
    for (int b = 0; b < 8; ++b) n |= r.get(8) << (8 * b);
    if (r.eof) return HZ_EFORMAT;
    cb->max_len = U ? mx : 0;
    cb->min_len = U ? mn : 0;
    info->n = n;
    info->payload_byte = r.bit >> 3;
    info->payload_bit = (uint32_t)(r.bit & 7);
    info->is_odd = (uint32_t)odd;
    info->last_byte = last;
    info->nsym = U;
    if (n / 2 > 0 && U == 0) return HZ_EFORMAT;
    return HZ_OK;
}

// ---------------------------------------------------------------------------
// Device table images.
// ---------------------------------------------------------------------------
namespace hz {

int select_enc_mode(const hz_codebook* cb) {
    if (cb->min_len == 16 && cb->max_len == 16) return ENC_FIXED16;  // U = 65 536, a complete 16-bit code
    if (cb->max_len <= 16) return ENC_DENSE;
    if (cb->max_len <= kHotMaxLen) return ENC_HOT;  // every code fits a slot: a miss is a taken slot
    return ENC_WIDE;
}

// FIXED16: u16 code per symbol.
std::vector<uint32_t> build_enc_fixed16(const hz_codebook* cb) {
    std::vector<uint32_t> img(kFixed16LdsBytes / 4, 0u);
    uint16_t* c16 = reinterpret_cast<uint16_t*>(img.data());
    for (uint32_t s = 0; s < HZ_NSYM; ++s) c16[s] = (uint16_t)cb->code[s];
    return img;
}

// DENSE: entry s = (code << 1 | 1) << (16 - L), 17 bits at bit 17*s (LE bit order).
std::vector<uint32_t> build_enc_dense(const hz_codebook* cb) {
    std::vector<uint32_t> img((kDenseLdsBytes + 16) / 4, 0u);
    for (uint32_t s = 0; s < HZ_NSYM; ++s) {
        const uint32_t L = cb->len[s];
        if (!L) continue;
        const uint64_t f = ((cb->code[s] << 1) | 1u) << (16 - L);
        const uint64_t bit = (uint64_t)s * 17;
        const uint64_t w = bit >> 5, sh = bit & 31;
        const uint64_t v = f << sh;
        img[w] |= (uint32_t)v;
        img[w + 1] |= (uint32_t)(v >> 32);
    }
    return img;
}

// HOT: 32768 slots; symbols s and s ^ m share slot hot_slot(s, m). The slot
// holds the shorter-coded (more frequent) of the pair when its code fits 25
// bits: (s >> 15) << 31 | L << 26 | code (L = 0: empty). m is chosen per
// codebook to minimise the escaped probability mass (weight 2^-L).
uint32_t choose_hot_mask(const hz_codebook* cb) {
    static const uint32_t cand[] = {0x8000, 0xffff, 0x8080, 0xc0c0, 0x80ff, 0xff80, 0xa0a0, 0xf0f0,
                                    0x8888, 0xcccc, 0xaaaa, 0x8001, 0xff00, 0x80c0, 0xe0e0, 0x9999};
    // weight 2^-L in fixed point (2^-25 units, fits u32); ineligible (absent or > 25
    // bits) symbols escape whatever the pairing, so they do not rank the masks
    static_assert(kHotMaxLen <= 25, "u32 weights");
    thread_local std::unique_ptr<uint32_t[]> wbuf(new uint32_t[HZ_NSYM]);
    uint32_t* w = wbuf.get();
    for (uint32_t s = 0; s < HZ_NSYM; ++s) {
        const uint32_t L = cb->len[s];
        w[s] = (L && L <= (uint32_t)kHotMaxLen) ? (1u << (kHotMaxLen - L)) : 0u;
    }
    uint32_t best = 0x8000;
    uint64_t best_miss = ~0ull;
    for (uint32_t m : cand) {
        // s ^ m for s in an 8-aligned run is an 8-aligned run permuted by m & 7
        const uint32_t hi = m & ~7u, lo = m & 7u;
        uint64_t miss = 0;
        for (uint32_t s0 = 0; s0 < 32768; s0 += 8) {
            const uint32_t* a = w + s0;
            const uint32_t* b = w + (s0 ^ hi);
            uint32_t part = 0;  // <= 8 * 2^24
            for (uint32_t j = 0; j < 8; ++j) {
                const uint32_t wa = a[j], wb = b[j ^ lo];  // the partner with bit 15 set
                part += wa < wb ? wa : wb;                 // the slot keeps the heavier one
            }
            miss += part;
        }
        if (miss < best_miss) { best_miss = miss; best = m; }
    }
    return best;
}

std::vector<uint32_t> build_enc_hot(const hz_codebook* cb, uint32_t m) {
    std::vector<uint32_t> img(kHotLdsBytes / 4, 0u);
    for (uint32_t slot = 0; slot < 32768; ++slot) {
        const uint32_t cands[2] = {slot, slot ^ (m & 0x7fffu) ^ 0x8000u};
        int best = -1;
        for (uint32_t s : cands) {
            const uint32_t L = cb->len[s];
            if (!L || L > (uint32_t)kHotMaxLen) continue;
            if (best < 0 || L < cb->len[best]) best = (int)s;
        }
        if (best >= 0) {
            const uint32_t s = (uint32_t)best;
            img[hot_word(slot)] = ((s >> 15) << 31) | ((uint32_t)cb->len[s] << 26) | (uint32_t)cb->code[s];
        }
    }
    return img;
}

// HOT escapes: for every slot, the entry (len << 26 | code) of the symbol that does NOT own it, at
// the slot's LDS word index hot_word(slot): a miss reads it at the byte offset of its slot's load.
std::vector<uint32_t> build_enc_esc(const hz_codebook* cb, uint32_t m) {
    std::vector<uint32_t> t(32768, 0u);
    for (uint32_t slot = 0; slot < 32768; ++slot) {
        const uint32_t cands[2] = {slot, slot ^ (m & 0x7fffu) ^ 0x8000u};
        int best = -1;
        for (uint32_t s : cands) {
            const uint32_t L = cb->len[s];
            if (!L || L > (uint32_t)kHotMaxLen) continue;
            if (best < 0 || L < cb->len[best]) best = (int)s;
        }
        for (uint32_t s : cands)
            if ((int)s != best && cb->len[s] && cb->len[s] <= (uint32_t)kNarrowMaxLen)
                t[hot_word(slot)] = ((uint32_t)cb->len[s] << 26) | (uint32_t)cb->code[s];
    }
    return t;
}

std::vector<uint32_t> build_len8(const hz_codebook* cb) {
    std::vector<uint32_t> img(kLen8LdsBytes / 4, 0u);
    uint8_t* b = reinterpret_cast<uint8_t*>(img.data());
    for (uint32_t s = 0; s < HZ_NSYM; ++s) b[len8_index(s)] = cb->len[s];
    return img;
}

// Range plan (k_range_dot): the code lengths of both symbols a histogram LDS word counts,
// in hist_word order: u16 = len[2 s'] | len[2 s' + 1] << 8, two per u32.
std::vector<uint32_t> build_lenpair(const hz_codebook* cb) {
    std::vector<uint32_t> img(16384, 0u);
    uint16_t* lp = reinterpret_cast<uint16_t*>(img.data());
    for (uint32_t w = 0; w < 32768; ++w) {
        const uint32_t s2 = hist_word_inv(w) << 1;
        lp[w] = (uint16_t)(cb->len[s2] | ((uint32_t)cb->len[s2 + 1] << 8));
    }
    return img;
}

std::vector<uint64_t> build_enc_wide(const hz_codebook* cb) {
    std::vector<uint64_t> t(HZ_NSYM, 0ull);
    for (uint32_t s = 0; s < HZ_NSYM; ++s)
        if (cb->len[s]) t[s] = ((uint64_t)cb->len[s] << 56) | cb->code[s];
    return t;
}

static uint32_t dense_dec_bytes(uint32_t K) {
    const uint32_t ent = 1u << K;
    const uint32_t words = (ent / 2 ? ent / 2 : 1) + (ent / 16 ? ent / 16 : 1);
    return 4 * ((words + 3) & ~3u);
}

// FIXED16 when every code is 16 bits; DENSE when the lengths span <= 4 values
// and the table leaves room for kDecMinWaves staging slots; LUT otherwise.
int select_dec_mode(const hz_codebook* cb) {
    if (cb->min_len == 16 && cb->max_len == 16) return DEC_FIXED16;
    if (cb->max_len <= 16 && cb->max_len - cb->min_len <= 3 &&
        dense_dec_bytes(cb->max_len) + 4 * kDecMinWaves * dec_slot_words_max((int)cb->max_len) <= kLdsBytes)
        return DEC_DENSE;
    return DEC_LUT;
}

// FIXED16 decode: u16 symbol per 16-bit code.
std::vector<uint32_t> build_dec_fixed16(const hz_codebook* cb) {
    std::vector<uint32_t> img(kFixed16LdsBytes / 4, 0u);
    uint16_t* t16 = reinterpret_cast<uint16_t*>(img.data());
    for (uint32_t s = 0; s < HZ_NSYM; ++s) t16[cb->code[s] & 0xffffu] = (uint16_t)s;
    return img;
}

// DENSE decode: u16 symbol per K-bit window, then 2-bit (L - min_len) per window.
int build_dec_dense(const hz_codebook* cb, std::vector<uint32_t>& img, int& K) {
    K = (int)cb->max_len;
    const uint32_t ent = 1u << K;
    const uint32_t symwords = ent / 2 ? ent / 2 : 1;
    const uint32_t lenwords = ent / 16 ? ent / 16 : 1;
    uint32_t words = symwords + lenwords;
    words = (words + 3) & ~3u;
    img.assign(words, 0u);
    std::vector<uint8_t> seen(ent, 0);
    for (uint32_t s = 0; s < HZ_NSYM; ++s) {
        const uint32_t L = cb->len[s];
        if (!L) continue;
        const uint32_t lo = (uint32_t)cb->code[s] << (K - L), hi = ((uint32_t)cb->code[s] + 1) << (K - L);
        for (uint32_t i = lo; i < hi; ++i) {
            if (seen[i]) return HZ_EFORMAT;  // not a prefix code
            seen[i] = 1;
            img[i >> 1] |= s << (16 * (i & 1));
            img[symwords + (i >> 4)] |= (L - cb->min_len) << ((i & 15) * 2);
        }
    }
    return HZ_OK;
}

namespace {
constexpr uint32_t kLeafBit = 1u << 31;
inline uint32_t leaf(uint32_t L, uint32_t sym) { return lut_leaf_entry(L, sym); }
}  // namespace

// Fill one table level. `syms` are the symbols whose codes pass through this
// table: their first D bits are consumed, the table is (1 << nb) entries at
// tab[base...]. Codes ending within nb bits fill their ranges with leaves;
// longer ones are grouped by their next nb bits (counting sort) and each
// group gets a subtable of its own, appended to l2, at most kDecLevelBits wide.
static int fill_level(const hz_codebook* cb, std::vector<uint32_t>& tab, size_t base, uint32_t nb, uint32_t D,
                      const uint32_t* syms, size_t nsyms, std::vector<uint32_t>& l2, uint32_t lvl) {
    const uint32_t E = 1u << nb;
    std::vector<uint32_t> cnt(E + 1, 0u), maxd(E, 0u);
    size_t ndeep = 0;
    for (size_t i = 0; i < nsyms; ++i) {
        const uint32_t s = syms[i];
        const uint32_t rem = cb->len[s] - D;
        const uint64_t bits = cb->code[s] & ((1ull << rem) - 1);
        if (rem <= nb) {
            const uint64_t lo = bits << (nb - rem), hi = (bits + 1) << (nb - rem);
            uint32_t* t = tab.data() + base;
            for (uint64_t k = lo; k < hi; ++k) {
                if (t[k]) return HZ_EFORMAT;
                t[k] = leaf(cb->len[s], s);
            }
        } else {
            const uint32_t q = (uint32_t)(bits >> (rem - nb));
            cnt[q + 1]++;
            maxd[q] = std::max(maxd[q], rem - nb);
            ++ndeep;
        }
    }
    if (!ndeep) return HZ_OK;
    for (uint32_t q = 0; q < E; ++q) cnt[q + 1] += cnt[q];
    std::vector<uint32_t> order(ndeep);
    {
        std::vector<uint32_t> pos(cnt.begin(), cnt.end() - 1);
        for (size_t i = 0; i < nsyms; ++i) {
            const uint32_t s = syms[i];
            const uint32_t rem = cb->len[s] - D;
            if (rem <= nb) continue;
            const uint64_t bits = cb->code[s] & ((1ull << rem) - 1);
            order[pos[(uint32_t)(bits >> (rem - nb))]++] = s;
        }
    }
    for (uint32_t q = 0; q < E; ++q) {
        if (cnt[q + 1] == cnt[q]) continue;
        if (tab[base + q]) return HZ_EFORMAT;
        const uint32_t nb2 = std::min<uint32_t>(maxd[q], lvl);
        const size_t off = l2.size();
        if (off + (1ull << nb2) > kLutMaxL2) return HZ_ENOMEM;
        l2.resize(off + (1ull << nb2), 0u);
        // (tab may alias l2: index, not pointer)
        tab[base + q] = lut_link((uint32_t)off + kLutGlobal, nb2, D + nb);
        const int rc = fill_level(cb, l2, off, nb2, D + nb, order.data() + cnt[q], cnt[q + 1] - cnt[q], l2, lvl);
        if (rc) return rc;
    }
    return HZ_OK;
}

// Hot second level in the LDS image. `budget` LDS words (what the kernel's
// staging leaves beside level 1) hold c-bit heads of the most used global subtables: entry j
// of a head is the leaf its range resolves to, or a link to the rest of the
// global subtable. Choice: greedy by decoded-mass per LDS word; the Kraft
// weight 2^-L of a code stands in for its frequency, so each global entry of
// an nb-bit subtable under level 1 carries mass 2^-(K1+nb).
static void add_lds_level(const hz_codebook* cb, std::vector<uint32_t>& img, const std::vector<uint32_t>& l2, int K1,
                          long budget) {
    if (budget < 64) return;
    struct Head { uint32_t q, nb, off, c; };
    std::vector<Head> heads;
    std::vector<std::vector<uint32_t>> resolved;  // per head: entries resolved within c bits, c = 1..nb
    for (uint32_t q = 0; q < img.size(); ++q) {
        const uint32_t e = img[q];
        if (e & kLeafBit) continue;
        const uint32_t nb = (e >> 5) & 15u, off = (e >> 10) - kLutGlobal;
        std::vector<uint32_t> r(nb + 1, 0u);
        for (uint32_t t = 0; t < (1u << nb); ++t) {
            const uint32_t x = l2[off + t];
            if (!(x & kLeafBit)) continue;
            const uint32_t rem = lut_leaf_len(x) - (uint32_t)K1;
            for (uint32_t c = rem; c <= nb; ++c) r[c]++;
        }
        heads.push_back({q, nb, off, 0});
        resolved.push_back(std::move(r));
    }
    // marginal greedy: mass gain (in units of 2^-(K1+nb) per entry) per added LDS word
    struct Cand { double rate; uint32_t h, c; bool operator<(const Cand& o) const { return rate < o.rate; } };
    std::priority_queue<Cand> pq;
    auto push = [&](uint32_t h) {
        const Head& hd = heads[h];
        const double unit = ldexp(1.0, -(K1 + (int)hd.nb));
        const uint32_t cs = hd.c ? (1u << hd.c) : 0u, cr = hd.c ? resolved[h][hd.c] : 0u;
        Cand best{0.0, h, 0};
        for (uint32_t c = hd.c + 1; c <= hd.nb; ++c) {
            const double rate = unit * (double)(resolved[h][c] - cr) / (double)((1u << c) - cs);
            if (rate > best.rate) best = {rate, h, c};
        }
        if (best.c) pq.push(best);
    };
    for (uint32_t h = 0; h < heads.size(); ++h) push(h);
    long used = 0;
    while (!pq.empty()) {
        const Cand cd = pq.top();
        pq.pop();
        Head& hd = heads[cd.h];
        if (cd.c <= hd.c) continue;
        const long add = (long)(1u << cd.c) - (hd.c ? (long)(1u << hd.c) : 0);
        if (used + add > budget) continue;
        used += add;
        hd.c = cd.c;
        push(cd.h);
    }
    for (const Head& hd : heads) {
        if (!hd.c) continue;
        const uint32_t o = (uint32_t)img.size(), rest = hd.nb - hd.c;
        for (uint32_t j = 0; j < (1u << hd.c); ++j) {
            const uint32_t t0 = hd.off + (j << rest);
            const uint32_t x = l2[t0];
            const bool done = (x & kLeafBit) && lut_leaf_len(x) - (uint32_t)K1 <= hd.c;
            img.push_back(done ? x : (rest ? lut_link(t0 + kLutGlobal, rest, (uint32_t)K1 + hd.c) : x));
        }
        img[hd.q] = lut_link(o, hd.c, (uint32_t)K1);
    }
    while (img.size() & 3) img.push_back(leaf(1, 0));
}

// LUT decode: level 1 (2^K1 u32) for the LDS, deeper levels (u32) for global
// memory.
int build_dec_lut(const hz_codebook* cb, std::vector<uint32_t>& img, std::vector<uint32_t>& l2, int& K1, int& lvl) {
    K1 = std::min<int>((int)cb->max_len, kDecLutMaxK1);
    if (K1 < 1) K1 = 1;
    std::vector<uint32_t> syms;
    syms.reserve(HZ_NSYM);
    for (uint32_t s = 0; s < HZ_NSYM; ++s)
        if (cb->len[s]) syms.push_back(s);
    // Global subtables of kDecLevelBits index bits; narrower (more levels, fewer entries) for a
    // codebook whose global table would not fit the link's 21-bit raw field.
    int rc = HZ_ENOMEM;
    for (lvl = kDecLevelBits; lvl >= 4 && rc == HZ_ENOMEM; --lvl) {
        img.assign(1u << K1, 0u);
        l2.clear();
        l2.reserve(1u << 19);
        rc = fill_level(cb, img, 0, (uint32_t)K1, 0, syms.data(), syms.size(), l2, (uint32_t)lvl);
    }
    ++lvl;
    if (rc) return rc;
    // Unused windows (incomplete codes) decode as a 1-bit filler so a lane
    // that runs past its unit's end never stalls.
    for (auto& e : img) if (!e) e = leaf(1, 0);
    for (auto& e : l2) if (!e) e = leaf(1, 0);
    if (l2.empty()) l2.push_back(leaf(1, 0));
    // heads fill what the decoder's staging slots (16 waves, sized from the
    // Kraft-weighted mean code length) leave
    double kbits = 0.0;
    for (uint32_t s = 0; s < HZ_NSYM; ++s)
        if (cb->len[s]) kbits += ldexp((double)cb->len[s], -(int)cb->len[s]);
    const uint64_t est_bits = (uint64_t)(kbits * kBlockSyms * 1.0625) + 256;
    add_lds_level(cb, img, l2, K1,
                  (long)(kLdsBytes / 4) - (long)img.size() - (long)kDecMaxWaves * (long)dec_slot_words(est_bits, (int)cb->max_len) - 64);
    while (img.size() < kDecMinLdsWords) img.push_back(leaf(1, 0));  // unused words: the slots start past LDS bit 1024
    return HZ_OK;
}

// Index walker tables (hz_kernels.hip k_idx_walk): a walk needs code LENGTHS
// only. img: one nibble per K-bit window (window w in byte w / 2, the high
// nibble for odd w), K = max(2, min(max_len, kWalkK, min_len + 14)): the length
// of the code the window starts with, minus bias = min_len - 1; for a window that
// starts a code longer than K bits, that length when every code under the window's
// prefix has it (and it fits), else 0. esc (max_len > K): one byte per max_len-bit window, the
// true length, filled under the escape prefixes. Windows no code starts
// (incomplete code spaces) read min_len, so a walk past the stream's end keeps
// moving. Byte i of a table is byte i of its u32 vector (little-endian).
void build_walk_len(const hz_codebook* cb, std::vector<uint32_t>& img, std::vector<uint32_t>& esc, int& K, int& M,
                    int& bias) {
    M = (int)cb->max_len;
    const int lmin = (int)cb->min_len;
    K = std::max(2, std::min(std::min(M, kWalkK), lmin + 14));
    bias = lmin - 1;
    img.assign(std::max<size_t>((size_t)1 << (K - 1), 16) / 4, 0x11111111u);
    uint8_t* t1 = reinterpret_cast<uint8_t*>(img.data());
    auto put = [&](uint64_t w, uint32_t v) {
        uint8_t& b = t1[w >> 1];
        b = (w & 1) ? (uint8_t)((b & 0x0f) | (v << 4)) : (uint8_t)((b & 0xf0) | v);
    };
    esc.clear();
    // esc holds every code longer than KE = min(K, 16) bits: k_idx_walk escapes only codes longer than
    // K, the chain walker's byte table (build_walk8, 16-bit windows) codes longer than 16
    const int KE = std::min(K, 16);
    if (M > KE) esc.assign(((size_t)1 << M) / 4, 0x01010101u);
    uint8_t* t2 = reinterpret_cast<uint8_t*>(esc.data());
    // a K-bit prefix shared only by codes of ONE length L > K still tells the length:
    // such windows read L - bias when it fits the nibble, and only the rest escape
    // (16 GiB Zipf(1.1), K = 17: 9 596 long prefixes, 420 ambiguous; escaped
    // codewords 7.4 % -> 2.3 %, the lengths past min_len + 14 included)
    std::vector<uint8_t> plen;
    if (M > K) plen.assign((size_t)1 << K, 0);
    for (uint32_t s = 0; s < HZ_NSYM; ++s) {
        const int L = cb->len[s];
        if (!L) continue;
        const uint64_t c = cb->code[s];
        if (L > KE) memset(t2 + (c << (M - L)), L, (size_t)1 << (M - L));
        if (L <= K) {
            const uint64_t w0 = c << (K - L), n = (uint64_t)1 << (K - L);
            for (uint64_t w = w0; w < w0 + n; ++w) put(w, (uint32_t)(L - bias));
        } else {
            uint8_t& pl = plen[c >> (L - K)];
            pl = pl == 0 || pl == (uint8_t)L ? (uint8_t)L : (uint8_t)255;
        }
    }
    for (size_t p = 0; p < plen.size(); ++p)
        if (plen[p]) put(p, plen[p] != 255 && plen[p] - bias <= 15 ? (uint32_t)(plen[p] - bias) : 0u);
}

}  // namespace hz

// The chain walker's length table (hz_kernels.hip k_chain_walk): one BYTE per K-bit window, K =
// min(max_len, 16) (2^16 bytes, the same 64 KiB of LDS as the 17-bit nibble table): the length of the
// code the window starts with when that code is at most K bits, or when every code under the
// window's prefix has one length; 0 (escape: the walker reads esc, build_walk_len's 2^max_len table)
// for prefixes shared by codes of different lengths. No bias and no nibble select per step, and
// long lengths need no escape (16 GiB Zipf(1.1): escaped codewords 2.4 % -> 1.4 %). Windows no code
// starts read min_len, so a walk past the stream's end keeps moving.
namespace hz {
void build_walk8(const hz_codebook* cb, std::vector<uint32_t>& img, int& K) {
    const int M = (int)cb->max_len;
    K = std::max(1, std::min(M, 16));
    std::vector<uint8_t> t((size_t)1 << K, (uint8_t)cb->min_len);
    std::vector<uint8_t> plen((size_t)1 << K, 0);
    for (uint32_t s = 0; s < HZ_NSYM; ++s) {
        const int L = cb->len[s];
        if (!L) continue;
        const uint64_t c = cb->code[s];
        if (L <= K) {
            const uint64_t w0 = c << (K - L), n = (uint64_t)1 << (K - L);
            memset(t.data() + w0, L, (size_t)n);
        } else {
            uint8_t& pl = plen[c >> (L - K)];
            pl = pl == 0 || pl == (uint8_t)L ? (uint8_t)L : (uint8_t)255;
        }
    }
    for (size_t p = 0; p < plen.size(); ++p)
        if (plen[p]) t[p] = plen[p] != 255 ? plen[p] : 0;
    while (t.size() % 16) t.push_back(0);
    img.assign(t.size() / 4, 0);
    memcpy(img.data(), t.data(), t.size());
}
}  // namespace hz

// The chain walker's escape table for codebooks whose codes exceed kWalkMaxLen bits (build_walk_len's
// 2^max_len table would not fit): one byte per M = kChainEscMaxBits window, the length of every code
// longer than 16 bits (the byte table's escapes) that is at most M bits, or shared by every code under
// the window when they are longer; 0 (a DEEP escape, resolved through the decode LUT) for M-bit
// prefixes of codes of different lengths. Windows no code starts read 1.
namespace hz {
void build_chain_esc(const hz_codebook* cb, std::vector<uint32_t>& img, int& M) {
    M = std::min((int)cb->max_len, kChainEscMaxBits);
    std::vector<uint8_t> t((size_t)1 << M, (uint8_t)1);
    std::vector<uint8_t> plen((size_t)1 << M, 0);
    for (uint32_t s = 0; s < HZ_NSYM; ++s) {
        const int L = cb->len[s];
        if (L <= 16) continue;
        const uint64_t c = cb->code[s];
        if (L <= M) {
            memset(t.data() + (c << (M - L)), L, (size_t)1 << (M - L));
        } else {
            uint8_t& pl = plen[c >> (L - M)];
            pl = pl == 0 || pl == (uint8_t)L ? (uint8_t)L : (uint8_t)255;
        }
    }
    for (size_t p = 0; p < plen.size(); ++p)
        if (plen[p]) t[p] = plen[p] != 255 ? plen[p] : 0;
    while (t.size() % 16) t.push_back(1);
    img.assign(t.size() / 4, 0);
    memcpy(img.data(), t.data(), t.size());
}
}  // namespace hz
