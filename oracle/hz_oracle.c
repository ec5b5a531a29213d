/*
 * hz_oracle.c -- CPU restatement of the reference Huffman path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker. The product
 * (huffman_amd/) never links or calls it.
 *
 * Parity pins (see DESIGN.md section "Oracle"):
 *   - files written by hzo_encode decode bit-exactly with the reference's own
 *     Decompressor.cu compiled from /root/reference (oracle/Makefile -> _ref/extract);
 *   - hzo_decode decodes the reference baseline encoder's output (tests/golden/);
 *   - hzo_codebook matches the literal round-by-round restatement of GenerateCL
 *     (oracle/generatecl_literal.py) and the hand-derived KAT of SURVEY.md 8(a4).
 *
 * Every function cites the reference file:line it restates. Reference paths are
 * relative to the yechuan51/huffman tree.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

#define HZO_NSYM 65536
#define HZO_MAXLEN 56

/* ------------------------------------------------------------------------ */
/* a1/a2: symbolisation + histogram.                                          */
/* Compressor.cu:38-48 (calculateFrequency): symbol i = data[2i] | data[2i+1]<<8,
 * one count per symbol, i < size/2. The odd tail byte is not a symbol
 * (Compressor.cu:339-351). Counts are u64 here (reference: u32 bins, identical
 * below 2^32 counts per bin). */
void hzo_hist16(const uint8_t *data, uint64_t n, uint64_t *hist)
{
    memset(hist, 0, sizeof(uint64_t) * HZO_NSYM);
    uint64_t s = n / 2;
    for (uint64_t i = 0; i < s; ++i)
        hist[(uint32_t)data[2 * i] | ((uint32_t)data[2 * i + 1] << 8)]++;
}

/* ------------------------------------------------------------------------ */
/* a3/a4: codebook.                                                          */
typedef struct { uint64_t f; uint32_t s; } hzo_leaf;

static int leaf_cmp(const void *a, const void *b)
{
    const hzo_leaf *x = (const hzo_leaf *)a, *y = (const hzo_leaf *)b;
    if (x->f != y->f) return x->f < y->f ? -1 : 1;
    return x->s < y->s ? -1 : (x->s > y->s);
}

/*
 * Build the codebook exactly as Compressor.cu + gpuHuffmanConstruction.h do.
 *
 *  order  : the U nonzero symbols in header order. thrust::sequence +
 *           sort_by_key over all 65536 (freq, index) pairs, then the nonzero tail
 *           (Compressor.cu:387-393, 414, 419-425). The radix sort is stable and
 *           the initial order is the symbol value, so order = (freq asc, sym asc).
 *  len,code: per symbol value (65536 entries), code right-aligned, first code
 *           bit = MSB of the len-bit value.
 *
 * Tree: GenerateCL (gpuHuffmanConstruction.h:353-466) pairs nodes (2i,2i+1) of a
 * list kept sorted by (freq, age) -- leftovers merge before new internals on
 * ties (KthElement h:193-206) -- in rounds bounded by the pivot of h:381-387.
 * Every round is a batch of consecutive steps of sequential Huffman whose two
 * picks are the smallest (freq, id) nodes, id = leaf rank for leaves and
 * U + creation index for internals (leaves are always older than internals).
 * That is the two-queue merge below with ties going to the leaf queue. The
 * literal round simulation in oracle/generatecl_literal.py pins this.
 *
 * Bits: GenerateCW (h:468-494) writes 0 for the left (first) child and 1 for
 * the right one, leaf to root; GpuCodewords::toCpu (h:562-574) maps 0->'1',
 * 1->'0' and reverses. So the first child of every pair carries '1', the second
 * '0', root first.
 *
 * Degenerate inputs (reference defect B4): U == 1 gives the reference
 * a 0-length code the decoder reads as 65536; here the single symbol gets code
 * "0" (len 1), which the reference decoder accepts. U == 0 builds nothing.
 *
 * Returns U (0..65536) or -1 on allocation failure, -2 if a code exceeds
 * HZO_MAXLEN bits (needs > ~5e11 symbols; unreachable at the configs).
 */
int hzo_codebook(const uint64_t *hist, uint16_t *order, uint8_t *len, uint64_t *code)
{
    memset(len, 0, HZO_NSYM);
    memset(code, 0, sizeof(uint64_t) * HZO_NSYM);
    uint32_t U = 0;
    for (uint32_t s = 0; s < HZO_NSYM; ++s) U += hist[s] != 0;
    if (U == 0) return 0;
    hzo_leaf *leaves = (hzo_leaf *)malloc(sizeof(hzo_leaf) * U);
    if (!leaves) return -1;
    uint32_t k = 0;
    for (uint32_t s = 0; s < HZO_NSYM; ++s)
        if (hist[s]) { leaves[k].f = hist[s]; leaves[k].s = s; ++k; }
    qsort(leaves, U, sizeof(hzo_leaf), leaf_cmp);
    for (uint32_t i = 0; i < U; ++i) order[i] = (uint16_t)leaves[i].s;
    if (U == 1) {
        len[leaves[0].s] = 1;
        code[leaves[0].s] = 0;
        free(leaves);
        return 1;
    }
    uint32_t nn = 2 * U - 1;
    uint64_t *f = (uint64_t *)malloc(sizeof(uint64_t) * nn);
    int32_t *lc = (int32_t *)malloc(sizeof(int32_t) * nn);
    int32_t *rc = (int32_t *)malloc(sizeof(int32_t) * nn);
    uint32_t *dep = (uint32_t *)malloc(sizeof(uint32_t) * nn);
    uint64_t *cw = (uint64_t *)malloc(sizeof(uint64_t) * nn);
    if (!f || !lc || !rc || !dep || !cw) {
        free(leaves); free(f); free(lc); free(rc); free(dep); free(cw);
        return -1;
    }
    for (uint32_t i = 0; i < U; ++i) { f[i] = leaves[i].f; lc[i] = rc[i] = -1; }
    uint32_t li = 0, qi = U, next = U;
    for (; next < nn; ++next) {
        uint32_t pick[2];
        for (int j = 0; j < 2; ++j) {
            /* smallest (freq, id): leaf wins ties (older). */
            if (li < U && (qi >= next || f[li] <= f[qi])) pick[j] = li++;
            else pick[j] = qi++;
        }
        f[next] = f[pick[0]] + f[pick[1]];
        lc[next] = (int32_t)pick[0];
        rc[next] = (int32_t)pick[1];
    }
    int rc_ok = (int)U;
    dep[nn - 1] = 0;
    cw[nn - 1] = 0;
    for (int32_t v = (int32_t)nn - 1; v >= (int32_t)U; --v) {
        dep[lc[v]] = dep[v] + 1; cw[lc[v]] = (cw[v] << 1) | 1u;  /* first child: '1' */
        dep[rc[v]] = dep[v] + 1; cw[rc[v]] = (cw[v] << 1);       /* second child: '0' */
    }
    for (uint32_t i = 0; i < U; ++i) {
        if (dep[i] > HZO_MAXLEN) { rc_ok = -2; break; }
        len[leaves[i].s] = (uint8_t)dep[i];
        code[leaves[i].s] = cw[i];
    }
    free(leaves); free(f); free(lc); free(rc); free(dep); free(cw);
    return rc_ok;
}

/* ------------------------------------------------------------------------ */
/* MSB-first bit writer: the semantics of writeFromUChar / writeFromUShort /    */
/* writeIfFullBuffer / writeFileSize (Compressor.cu:637-669,692-700). Those     */
/* helpers keep `bitCounter` pending bits and emit whole bytes MSB first, so   */
/* the header + payload is one continuous MSB-first bit stream.                */
typedef struct { uint8_t *p; uint64_t cap, pos; uint64_t acc; int nacc; int overflow; } hzo_bw;

static void bw_put(hzo_bw *w, uint64_t v, int nbits)
{
    while (nbits > 0) {
        int take = nbits > 32 ? 32 : nbits;
        uint64_t part = (v >> (nbits - take)) & ((1ull << take) - 1);
        w->acc = (w->acc << take) | part;
        w->nacc += take;
        nbits -= take;
        while (w->nacc >= 8) {
            w->nacc -= 8;
            if (w->pos < w->cap) w->p[w->pos] = (uint8_t)(w->acc >> w->nacc);
            else w->overflow = 1;
            w->pos++;
        }
    }
}

static void bw_flush(hzo_bw *w)
{
    /* Compressor.cu:597-601: bufferByte <<= (8 - bitCounter); zero padded. */
    if (w->nacc > 0) bw_put(w, 0, 8 - w->nacc);
}

/* Header of Compressor.cu:431-487. Returns header bit length (bytes*8 incl. the
 * 3-4 byte-aligned prefix); the payload starts at that bit. */
static uint64_t write_header(hzo_bw *w, uint64_t n, uint32_t U, const uint16_t *order,
                             const uint8_t *len, const uint64_t *code)
{
    uint8_t pre[4];
    int np = 0;
    pre[np++] = (uint8_t)(U & 0xff);          /* fwrite(&U, 2, ...) little endian :434 */
    pre[np++] = (uint8_t)((U >> 8) & 0xff);
    pre[np++] = (uint8_t)(n & 1);             /* isOdd :438 */
    if (n & 1) pre[np++] = 0;                 /* lastByte placeholder, set by caller :439-443 */
    for (int i = 0; i < np; ++i) bw_put(w, pre[i], 8);
    for (uint32_t i = 0; i < U; ++i) {        /* :454-483 */
        uint32_t s = order[i];
        bw_put(w, s, 16);                     /* writeFromUShort: high byte first :648-656 */
        bw_put(w, len[s] & 0xff, 8);          /* writeFromUChar(L) :465 */
        bw_put(w, code[s], len[s]);           /* code string, first char first :470-481 */
    }
    for (int b = 0; b < 8; ++b) bw_put(w, (n >> (8 * b)) & 0xff, 8);  /* writeFileSize :661-669 */
    return (uint64_t)np * 8;  /* caller recomputes exact bit position */
}

/* Exact size of the encoded file for a codebook (header + payload, padded). */
uint64_t hzo_encoded_bits(uint64_t n, uint32_t U, const uint64_t *hist, const uint8_t *len,
                          uint64_t *header_bits)
{
    uint64_t hb = (uint64_t)(3 + (n & 1)) * 8;
    uint64_t pb = 0;
    for (uint32_t s = 0; s < HZO_NSYM; ++s) {
        if (hist[s]) { hb += 24 + len[s]; pb += hist[s] * len[s]; }
    }
    (void)U;
    hb += 64;
    if (header_bits) *header_bits = hb;
    return hb + pb;
}

/*
 * Whole-file encode: the byte stream `archive <file>` writes to <file>.compressed,
 * with the reference's packing semantics (Compressor.cu:541-601: payload bit k of
 * symbol j sits at b + sum_{i<j} L(s_i) + k after the header's pending bits) and
 * without its B1/B2 packing defects.
 * Returns 0, or -1 alloc / -2 code too long / -3 capacity too small.
 */
int hzo_encode(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len)
{
    uint64_t *hist = (uint64_t *)malloc(sizeof(uint64_t) * HZO_NSYM);
    uint16_t *order = (uint16_t *)malloc(sizeof(uint16_t) * HZO_NSYM);
    uint8_t *len = (uint8_t *)malloc(HZO_NSYM);
    uint64_t *code = (uint64_t *)malloc(sizeof(uint64_t) * HZO_NSYM);
    if (!hist || !order || !len || !code) { free(hist); free(order); free(len); free(code); return -1; }
    hzo_hist16(in, n, hist);
    int U = hzo_codebook(hist, order, len, code);
    if (U < 0) { free(hist); free(order); free(len); free(code); return U; }
    hzo_bw w = {out, cap, 0, 0, 0, 0};
    write_header(&w, n, (uint32_t)U, order, len, code);
    if ((n & 1) && cap > 3) out[3] = in[n - 1];
    uint64_t S = n / 2;
    for (uint64_t i = 0; i < S; ++i) {
        uint32_t s = (uint32_t)in[2 * i] | ((uint32_t)in[2 * i + 1] << 8);
        bw_put(&w, code[s], len[s]);
    }
    bw_flush(&w);
    *out_len = w.pos;
    free(hist); free(order); free(len); free(code);
    return w.overflow ? -3 : 0;
}

/*
 * Pack symbols [sym0, sym0+count) of `in` with a given code table into a
 * zero-initialised buffer at absolute bit offset `bit0` (MSB-first), OR-ing.
 * Restates the payload placement of Compressor.cu:541-576 for an arbitrary
 * slice; used to check GPU output at sizes where a whole-file oracle is slow.
 */
void hzo_pack_range(const uint8_t *in, uint64_t sym0, uint64_t count, const uint8_t *len,
                    const uint64_t *code, uint64_t bit0, uint8_t *out)
{
    uint64_t pos = bit0;
    for (uint64_t i = sym0; i < sym0 + count; ++i) {
        uint32_t s = (uint32_t)in[2 * i] | ((uint32_t)in[2 * i + 1] << 8);
        uint32_t L = len[s];
        uint64_t c = code[s];
        for (int b = (int)L - 1; b >= 0; --b, ++pos)
            if ((c >> b) & 1) out[pos >> 3] |= (uint8_t)(0x80u >> (pos & 7));
    }
}

/* ------------------------------------------------------------------------ */
/* a9: decode (Decompressor.cu:47-291).                                      */
typedef struct { const uint8_t *p; uint64_t len, bit; int eof; } hzo_br;

static uint32_t br_bit(hzo_br *r)
{
    if ((r->bit >> 3) >= r->len) { r->eof = 1; return 0; }
    uint32_t v = (r->p[r->bit >> 3] >> (7 - (r->bit & 7))) & 1;
    r->bit++;
    return v;
}

static uint32_t br_bits(hzo_br *r, int n)
{
    uint32_t v = 0;
    for (int i = 0; i < n; ++i) v = (v << 1) | br_bit(r);
    return v;
}

/*
 * Parse the header (Decompressor.cu:65-103) into a code table and decode.
 * U field 0 means 65536 (:69-71) -- except that this build's encoder writes
 * U = 0 for inputs of fewer than 2 bytes, recognisable because the file then
 * ends right after the 8-byte size (a 65536-entry codebook is >= 196 KiB).
 * L field 0 means 65536 (:94-95), unsupported here (returns -4).
 * Output: floor(N/2) symbols as 2 bytes LE (:283) then lastByte if isOdd (:286-289).
 * Returns 0, or -3 output capacity, -4 malformed/truncated stream, -1 alloc.
 */
int hzo_decode(const uint8_t *f, uint64_t flen, uint8_t *out, uint64_t cap, uint64_t *out_n)
{
    if (flen < 3) return -4;
    uint32_t U = (uint32_t)f[0] | ((uint32_t)f[1] << 8);
    int odd = f[2] != 0;
    uint8_t last = 0;
    uint64_t pre = 3;
    if (odd) { if (flen < 4) return -4; last = f[3]; pre = 4; }
    if (U == 0) U = (flen == pre + 8) ? 0 : 65536;
    /* trie: node 0 = root; child[2*v + bit]; sym for leaves */
    uint64_t maxn = 1 + (uint64_t)U * HZO_MAXLEN + 2;
    int32_t *child = (int32_t *)malloc(sizeof(int32_t) * 2 * maxn);
    int32_t *sym = (int32_t *)malloc(sizeof(int32_t) * maxn);
    if (!child || !sym) { free(child); free(sym); return -1; }
    memset(child, 0xff, sizeof(int32_t) * 2 * maxn);
    memset(sym, 0xff, sizeof(int32_t) * maxn);
    uint64_t nn = 1;
    hzo_br r = {f, flen, pre * 8, 0};
    int rc = 0;
    for (uint32_t i = 0; i < U && !rc; ++i) {
        uint32_t s = br_bits(&r, 16);           /* process_16_bits_DATA :92 */
        uint32_t L = br_bits(&r, 8);            /* process_8_bits_NUMBER :93 */
        if (L == 0 || L > HZO_MAXLEN) { rc = -4; break; }
        uint64_t v = 0;
        for (uint32_t b = 0; b < L; ++b) {      /* process_n_bits_TO_STRING :129-163 */
            uint32_t bit = br_bit(&r);
            if (child[2 * v + bit] < 0) { child[2 * v + bit] = (int32_t)nn; nn++; }
            v = (uint64_t)child[2 * v + bit];
        }
        sym[v] = (int32_t)s;                    /* :162 */
    }
    uint64_t n = 0;
    for (int b = 0; b < 8 && !rc; ++b) n |= (uint64_t)br_bits(&r, 8) << (8 * b);   /* readFileSize :243-255 */
    if (r.eof) rc = -4;
    uint64_t S = n / 2;
    uint64_t need = 2 * S + (odd ? 1 : 0);
    if (!rc && need > cap) rc = -3;
    for (uint64_t i = 0; i < S && !rc; ++i) {   /* translateFile :262-284 */
        uint64_t v = 0;
        while (child[2 * v] >= 0 || child[2 * v + 1] >= 0) {
            uint32_t bit = br_bit(&r);
            if (r.eof || child[2 * v + bit] < 0) { rc = -4; break; }
            v = (uint64_t)child[2 * v + bit];
        }
        if (rc) break;
        out[2 * i] = (uint8_t)(sym[v] & 0xff);
        out[2 * i + 1] = (uint8_t)((sym[v] >> 8) & 0xff);
    }
    if (!rc && odd) out[2 * S] = last;
    if (!rc) *out_n = need;
    free(child); free(sym);
    return rc;
}

/*
 * Header alone (Decompressor.cu:65-103, read :69-71, :74-80, :90-96,
 * readFileSize :243-255): entry i of the file -> order[i] = symbol,
 * len[symbol] = L, code[symbol] = its L bits right aligned. info[6] = N, the
 * payload's first byte and bit (MSB = 0), isOdd, lastByte, U. The checker of
 * the product's header parsers (host and device). Returns 0 or -4 (malformed
 * or truncated: L == 0 / > HZO_MAXLEN, a duplicate symbol, EOF in the header).
 */
int hzo_parse_header(const uint8_t *f, uint64_t flen, uint16_t *order, uint8_t *len, uint64_t *code,
                     uint64_t *info)
{
    if (flen < 3) return -4;
    uint32_t U = (uint32_t)f[0] | ((uint32_t)f[1] << 8);
    int odd = f[2] != 0;
    uint8_t last = 0;
    uint64_t pre = 3;
    if (odd) { if (flen < 4) return -4; last = f[3]; pre = 4; }
    if (U == 0) U = (flen == pre + 8) ? 0 : 65536;
    memset(len, 0, HZO_NSYM);
    memset(code, 0, sizeof(uint64_t) * HZO_NSYM);
    hzo_br r = {f, flen, pre * 8, 0};
    for (uint32_t i = 0; i < U; ++i) {
        uint32_t s = br_bits(&r, 16);
        uint32_t L = br_bits(&r, 8);
        if (r.eof || L == 0 || L > HZO_MAXLEN || len[s]) return -4;
        uint64_t c = 0;
        for (uint32_t b = 0; b < L; ++b) c = (c << 1) | br_bit(&r);
        order[i] = (uint16_t)s;
        len[s] = (uint8_t)L;
        code[s] = c;
    }
    uint64_t n = 0;
    for (int b = 0; b < 8; ++b) n |= (uint64_t)br_bits(&r, 8) << (8 * b);
    if (r.eof) return -4;
    info[0] = n;
    info[1] = r.bit >> 3;
    info[2] = r.bit & 7;
    info[3] = (uint64_t)odd;
    info[4] = last;
    info[5] = U;
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Synthetic inputs (this build's generator, not a reference function;      */
/* DESIGN.md "Synthetic inputs"). byte i of the stream, i counted from 0:    */
/*   zipf   : smallest r-1 with u < thr[r-1], u = splitmix64(seed ^ i)       */
/*   uniform: low 8 bits of splitmix64(seed ^ i)                             */
static uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

void hzo_zipf_thresholds(double alpha, uint64_t *thr)
{
    double H = 0.0;
    for (int r = 1; r <= 256; ++r) H += pow((double)r, -alpha);
    double c = 0.0;
    for (int r = 1; r <= 256; ++r) {
        c += pow((double)r, -alpha);
        double x = c / H;
        thr[r - 1] = (r == 256 || x >= 1.0) ? UINT64_MAX : (uint64_t)ldexp(x, 64);
    }
}

void hzo_gen(uint8_t *out, uint64_t n, uint64_t offset, int kind, uint64_t seed, const uint64_t *thr)
{
    for (uint64_t j = 0; j < n; ++j) {
        uint64_t u = splitmix64(seed ^ (offset + j));
        if (kind == 0) { out[j] = (uint8_t)u; continue; }
        int lo = 0, hi = 255;
        while (lo < hi) { int m = (lo + hi) >> 1; if (u < thr[m]) hi = m; else lo = m + 1; }
        out[j] = (uint8_t)lo;
    }
}

/* ------------------------------------------------------------------------ */
/* The serial codeword walk of translateFile (Decompressor.cu:262-284) over a bare payload, started at
 * any stream bit: codewords are decoded from bit `pos` (a trie of the codebook, MSB-first bits of
 * payload byte 0 onwards) while the position is below `end` and fewer than max_count were taken;
 * symbols go to out (2 bytes LE each) when out is not NULL. Returns the number of codewords and sets
 * *exit to the bit after the last one (a walk started mid-codeword follows whatever path the bits
 * give: Huffman codes resynchronise). The checker of the per-part index-less decode
 * (huffman_amd/dist.py decode_indexless_split, tests/test_dist.py). -1: allocation failed or a code
 * the trie does not hold. */
int64_t hzo_walk(const uint8_t *payload, uint64_t nbytes, const uint8_t *len, const uint64_t *code, uint64_t pos,
                 uint64_t end, uint64_t max_count, uint8_t *out, uint64_t *exit)
{
    uint64_t maxn = 1 + 65536ull * HZO_MAXLEN;
    int32_t *child = (int32_t *)malloc(sizeof(int32_t) * 2 * maxn);
    int32_t *sym = (int32_t *)malloc(sizeof(int32_t) * maxn);
    if (!child || !sym) { free(child); free(sym); return -1; }
    memset(child, 0xff, sizeof(int32_t) * 2 * maxn);
    uint64_t nn = 1;
    for (uint32_t s = 0; s < 65536; ++s) {
        if (!len[s]) continue;
        uint64_t v = 0;
        for (int b = len[s] - 1; b >= 0; --b) {
            uint32_t bit = (uint32_t)((code[s] >> b) & 1);
            if (child[2 * v + bit] < 0) { child[2 * v + bit] = (int32_t)nn; nn++; }
            v = (uint64_t)child[2 * v + bit];
        }
        sym[v] = (int32_t)s;
    }
    hzo_br r = {payload, nbytes, pos, 0};
    int64_t n = 0;
    while (r.bit < end && (uint64_t)n < max_count) {
        uint64_t v = 0;
        while (child[2 * v] >= 0 || child[2 * v + 1] >= 0) {
            uint32_t bit = br_bit(&r);             /* past the payload: zeros */
            if (child[2 * v + bit] < 0) { free(child); free(sym); return -1; }
            v = (uint64_t)child[2 * v + bit];
        }
        if (out) { out[2 * n] = (uint8_t)(sym[v] & 0xff); out[2 * n + 1] = (uint8_t)((sym[v] >> 8) & 0xff); }
        ++n;
    }
    *exit = r.bit;
    free(child); free(sym);
    return n;
}
