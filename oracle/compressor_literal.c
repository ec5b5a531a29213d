/*
 * compressor_literal.c -- literal restatement of the reference GPU encoder's
 * file writer, Compressor.cu main() from the header onwards, defects included.
 *
 * TEST INFRASTRUCTURE ONLY (see hz_oracle.c header). Nothing under huffman_amd/
 * links or calls it. It exists to show, byte by byte, where this build's
 * stream equals what Compressor.cu writes and where it does not (the
 * reference's packing defects B1/B2). Compressor.cu itself
 * needs nvcc, CUDA thrust and inline PTX and cannot be built here (SURVEY.md
 * 8c), so this file re-expresses its host writers and its encodeFromCW kernel
 * serially: every output byte is computed by the same arithmetic the kernel's
 * thread for that byte runs (threads are independent; the order is free).
 *
 * Input: the codebook as the reference host sees it after
 * gpuCodebookConstruction (header order, code length and code per symbol
 * value), the file bytes, and N. Output: the complete .compressed image, plus
 * a flag per byte that says the reference's value for that byte is undefined
 * (it reads memory past the input or past the code pool; B2, and B1 at the
 * pool's end). Undefined reads return 0 here.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define HZL_NSYM 65536

typedef struct {
    uint8_t *out;
    uint64_t cap, n;
    int overflow;
} hzl_file;

static void put(hzl_file *f, uint8_t b)
{
    if (f->n < f->cap) f->out[f->n] = b;
    else f->overflow = 1;
    f->n++;
}

/* Compressor.cu:637-646 writeFromUChar: emits the pending bitCounter bits and
 * the top 8-bitCounter bits of the byte; the byte itself becomes the buffer
 * (its low bitCounter bits are the new pending bits). */
static void write_uchar(hzl_file *f, uint8_t byte, uint8_t *buffer, int bit_counter)
{
    *buffer = (uint8_t)(*buffer << (8 - bit_counter));
    *buffer |= (uint8_t)(byte >> bit_counter);
    put(f, *buffer);
    *buffer = byte;
}

/* Compressor.cu:648-656 writeFromUShort: high byte, then low byte. */
static void write_ushort(hzl_file *f, uint16_t v, uint8_t *buffer, int bit_counter)
{
    write_uchar(f, (uint8_t)(v >> 8), buffer, bit_counter);
    write_uchar(f, (uint8_t)(v & 0xff), buffer, bit_counter);
}

/* Compressor.cu:152-180 binarySearch: the index of target, else the largest
 * index with offsets[i] < target, else -1. */
static int64_t binary_search(const int64_t *offsets, int64_t num, int64_t target)
{
    int64_t low = 0, high = num - 1, left = -1;
    while (low <= high) {
        const int64_t mid = low + (high - low) / 2;
        if (offsets[mid] == target) return mid;
        if (offsets[mid] < target) { left = mid; low = mid + 1; }
        else high = mid - 1;
    }
    return left;
}

typedef struct {
    const uint8_t *data;
    int64_t size;          /* originalFileSize */
    const char *pool;      /* transformationStringsPool ('0'/'1', symbol value order) */
    int64_t pool_chars;
    const int *len;        /* transformationLengths[65536] */
    const int *pool_off;   /* transformationStringsOffset[65536] */
    const int64_t *off;    /* CW_offsets[S + 1] */
} hzl_kernel;

/* Reads that the reference makes past its buffers are undefined: 0 here, flagged. */
static uint8_t rd_data(const hzl_kernel *k, int64_t i, int *undef)
{
    if (i < 0 || i >= k->size) { *undef = 1; return 0; }
    return k->data[i];
}

static int bit_of(const hzl_kernel *k, int64_t i, int *undef)
{
    if (i < 0 || i >= k->pool_chars) { *undef = 1; return 0; }
    return k->pool[i] == '1';
}

/* Compressor.cu:182-313 encodeFromCW, the work of the thread for output byte
 * `index`. *b2 is set when the byte takes bits of symbols past the last one
 * (the loop at :227-246 walks off the input). */
static uint8_t encode_byte(const hzl_kernel *k, int64_t index, uint8_t buffer_byte, int *undef, int *b2)
{
    const int64_t S = k->size / 2;
    uint8_t out = 0;
    const int64_t left = binary_search(k->off, S + 1, index * 8);
    int64_t right = left + 1;
    if (left >= 0) {
        const uint16_t sl = (uint16_t)((rd_data(k, left * 2 + 1, undef) << 8) | rd_data(k, left * 2, undef));
        const int lo = k->pool_off[sl], ll = k->len[sl];
        if (right < S) {
            uint16_t sr = (uint16_t)((rd_data(k, right * 2 + 1, undef) << 8) | rd_data(k, right * 2, undef));
            int ro = k->pool_off[sr], rl = k->len[sr];
            const int64_t n = k->off[right] - index * 8;
            if (n <= 8) {
                int take = 8;
                for (int64_t i = n - 1; i >= 0; i--) {
                    out = (uint8_t)(out << 1);
                    if (bit_of(k, lo + ll - 1 - i, undef)) out |= 1;
                    take -= 1;
                }
                int guard = 0;
                while (take > 0) {
                    const int64_t rs = take <= rl ? take : rl;
                    for (int64_t i = 0; i < rs; i++) {
                        out = (uint8_t)(out << 1);
                        if (bit_of(k, ro + i, undef)) out |= 1;
                        take -= 1;
                    }
                    if (take > 0) {
                        right += 1;
                        if (right >= S) *b2 = 1;   /* past the last symbol: input overrun */
                        sr = (uint16_t)((rd_data(k, right * 2 + 1, undef) << 8) | rd_data(k, right * 2, undef));
                        ro = k->pool_off[sr];
                        rl = k->len[sr];
                        if (++guard > 64) { *undef = 1; break; }   /* a zero-length garbage symbol spins */
                    }
                }
            } else {
                const int64_t sh = index * 8 - k->off[left];
                for (int64_t i = 0; i < 8; i++) {
                    out = (uint8_t)(out << 1);
                    if (bit_of(k, lo + sh + i, undef)) out |= 1;
                }
            }
        } else {  /* the last codeword (:262-292) */
            const int64_t n = k->off[left] + k->len[sl] - index * 8;
            if (n <= 8) {
                for (int64_t i = n - 1; i >= 0; i--) {
                    out = (uint8_t)(out << 1);
                    if (bit_of(k, lo + ll - 1 - i, undef)) out |= 1;
                }
            } else {
                const int64_t sh = index * 8 - k->off[left];
                for (int64_t i = 0; i < 8; i++) {
                    out = (uint8_t)(out << 1);
                    if (bit_of(k, lo + sh + i, undef)) out |= 1;
                }
            }
        }
    } else {  /* byte 0 with CW_offsets[0] > 0 (:294-310): 8 - b bits of symbol 0's string only (B1) */
        const uint16_t sr = (uint16_t)((rd_data(k, 1, undef) << 8) | rd_data(k, 0, undef));
        const int ro = k->pool_off[sr];
        out = (uint8_t)(out | buffer_byte);
        for (int64_t i = 0; i < 8 - k->off[0]; i++) {
            out = (uint8_t)(out << 1);
            if (bit_of(k, ro + i, undef)) out |= 1;
        }
    }
    return out;
}

/* Compressor.cu:431-487 (writers :637-669): the header of a file of n bytes,
 * returned as its complete bytes; the bitCounter pending bits (the payload's
 * first byte opens with them) come back MSB-aligned in *pending and their
 * count in *pending_bits. Returns the byte count, or -2 when cap is short. */
static int64_t header_literal(hzl_file *f, uint64_t n, uint8_t last_byte, const uint16_t *order, uint32_t U,
                              const uint8_t *len8, const uint64_t *code, uint8_t *buffer_out, int *bit_counter_out)
{
    const int64_t size = (int64_t)n;
    const int is_odd = size % 2 == 1;
    /* :434 fwrite(&uniqueSymbolCount, 2, 1): low two bytes, little endian */
    put(f, (uint8_t)(U & 0xff));
    put(f, (uint8_t)((U >> 8) & 0xff));
    put(f, (uint8_t)is_odd);                      /* :438 */
    if (is_odd) put(f, last_byte);                /* :439-443 */
    int bit_counter = 0;
    uint8_t buffer = 0;
    for (uint32_t i = 0; i < U; ++i) {            /* :454-483 */
        const uint16_t ch = order[i];
        const int L = len8[ch];
        write_ushort(f, ch, &buffer, bit_counter);
        write_uchar(f, (uint8_t)L, &buffer, bit_counter);
        for (int b = L - 1; b >= 0; --b) {
            buffer = (uint8_t)(buffer << 1);
            if ((code[ch] >> b) & 1) buffer |= 1;
            bit_counter++;
            if (bit_counter == 8) { put(f, buffer); bit_counter = 0; }   /* writeIfFullBuffer :692-700 */
        }
    }
    int64_t fs = size;                            /* writeFileSize :661-669 */
    for (int i = 0; i < 8; i++) { write_uchar(f, (uint8_t)(fs % 256), &buffer, bit_counter); fs /= 256; }
    *buffer_out = buffer;
    *bit_counter_out = bit_counter;
    return f->overflow ? -2 : (int64_t)f->n;
}

int64_t hzl_header(uint64_t n, uint8_t last_byte, const uint16_t *order, uint32_t U, const uint8_t *len8,
                   const uint64_t *code, uint8_t *out, uint64_t cap, uint32_t *pending_bits, uint8_t *pending)
{
    hzl_file f = {out, cap, 0, 0};
    uint8_t buffer;
    int bc;
    const int64_t r = header_literal(&f, n, last_byte, order, U, len8, code, &buffer, &bc);
    *pending_bits = (uint32_t)bc;
    *pending = bc ? (uint8_t)(buffer << (8 - bc)) : 0;
    return r;
}

/*
 * The whole of Compressor.cu main() from the header on (:431-601, writers
 * :637-684). order[U]: header order; len/code: per symbol value (code right
 * aligned, first code bit = MSB). Writes the file image into out (cap bytes)
 * and a 0/1 flag per byte into undef_flags (cap bytes, may be NULL): 1 when
 * the reference's byte is undefined (reads past its buffers). *b1_byte and
 * *b2_byte receive the file offsets of the bytes the B1 path and the B2 path
 * produced (-1 when the path was not taken). Returns the file size, or -1
 * (U < 2 or N < 2: the reference's defect B4, not restated).
 */
int64_t hzl_archive(const uint8_t *data, uint64_t n, const uint16_t *order, uint32_t U, const uint8_t *len8,
                    const uint64_t *code, uint8_t *out, uint64_t cap, uint8_t *undef_flags,
                    int64_t *b1_byte, int64_t *b2_byte)
{
    *b1_byte = -1;
    *b2_byte = -1;
    if (U < 2 || n < 2) return -1;
    hzl_file f = {out, cap, 0, 0};
    const int64_t size = (int64_t)n;
    uint8_t buffer;
    int bit_counter;
    if (header_literal(&f, n, size % 2 ? data[size - 1] : 0, order, U, len8, code, &buffer, &bit_counter) < 0)
        return -2;
    const uint64_t head = f.n;
    /* :495-539 lengths, pool and pool offsets, in symbol value order */
    int *lens = (int *)calloc(HZL_NSYM, sizeof(int));
    int *poff = (int *)calloc(HZL_NSYM, sizeof(int));
    int64_t total = 0;
    for (int s = 0; s < HZL_NSYM; ++s) { lens[s] = len8[s]; poff[s] = (int)total; total += lens[s]; }
    char *pool = (char *)malloc(total ? (size_t)total : 1);
    for (int s = 0; s < HZL_NSYM; ++s)
        for (int b = 0; b < lens[s]; ++b) pool[poff[s] + b] = ((code[s] >> (lens[s] - 1 - b)) & 1) ? '1' : '0';
    /* :541-553 populateCWLength with CW_lengths[0] = bitCounter, inclusive scan */
    const int64_t S = size / 2;
    int64_t *off = (int64_t *)malloc((size_t)(S + 1) * sizeof(int64_t));
    off[0] = bit_counter;
    for (int64_t i = 0; i < S; ++i) {
        const uint16_t sym = (uint16_t)((data[2 * i + 1] << 8) | data[2 * i]);
        off[i + 1] = off[i] + lens[sym];
    }
    const int64_t content = off[S];                              /* :556-561 */
    int64_t alloc = content;
    if (alloc % 8 != 0) alloc += 8 - alloc % 8;                  /* :564-567 */
    const int64_t nbytes = alloc / 8;
    uint8_t *buf = (uint8_t *)malloc(nbytes ? (size_t)nbytes : 1);
    uint8_t *bad = (uint8_t *)calloc(nbytes ? (size_t)nbytes : 1, 1);
    hzl_kernel k = {data, size, pool, total, lens, poff, off};
    int64_t b2_index = -1;
    for (int64_t index = 0; index * 8 < alloc; ++index) {        /* :573-576 grid-stride loop */
        int undef = 0, b2 = 0;
        buf[index] = encode_byte(&k, index, buffer, &undef, &b2);
        bad[index] = (uint8_t)(undef || b2);
        if (b2) b2_index = index;
    }
    /* :588 writeFileContent (:673-684) */
    const uint8_t last = nbytes ? buf[nbytes - 1] : 0;
    const int64_t extra = alloc - content;
    const int64_t to_write = extra == 0 ? nbytes : nbytes - 1;
    bit_counter = extra == 0 ? 0 : (int)(8 - extra);
    buffer = last;
    for (int64_t i = 0; i < to_write; ++i) {
        if (undef_flags && f.n < cap) undef_flags[f.n] = bad[i];
        put(&f, buf[i]);
    }
    if (bit_counter > 0) {                                       /* :597-601 */
        buffer = (uint8_t)(buffer << (8 - bit_counter));
        if (undef_flags && f.n < cap) undef_flags[f.n] = bad[nbytes - 1];
        put(&f, buffer);
    }
    if (off[0] > 0 && 8 - off[0] > 0) *b1_byte = (int64_t)head;  /* byte 0 took the :294-310 path */
    if (b2_index >= 0) *b2_byte = (int64_t)head + b2_index;
    if (undef_flags)
        for (uint64_t i = 0; i < head && i < cap; ++i) undef_flags[i] = 0;
    free(lens); free(poff); free(pool); free(off); free(buf); free(bad);
    return f.overflow ? -2 : (int64_t)f.n;
}
