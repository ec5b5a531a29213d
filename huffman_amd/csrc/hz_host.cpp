// hz_host.cpp -- C ABI implementation: contexts, stage wrappers, and the
// file-level `archive` / `extract` flow (Compressor.cu:315-632,
// Decompressor.cu:47-114). Device work always runs through the gfx950 kernels
// of hz_kernels.hip; there is no CPU fallback for any stage.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <iostream>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "huffman_amd.h"
#include "hz_internal.h"

namespace hz {
int select_enc_mode(const hz_codebook* cb);
std::vector<uint32_t> build_enc_dense(const hz_codebook* cb);
std::vector<uint32_t> build_enc_fixed16(const hz_codebook* cb);
std::vector<uint32_t> build_dec_fixed16(const hz_codebook* cb);
std::vector<uint32_t> build_enc_hot(const hz_codebook* cb, uint32_t m);
uint32_t choose_hot_mask(const hz_codebook* cb);
std::vector<uint32_t> build_enc_esc(const hz_codebook* cb, uint32_t m);
std::vector<uint32_t> build_len8(const hz_codebook* cb);
std::vector<uint32_t> build_lenpair(const hz_codebook* cb);
std::vector<uint64_t> build_enc_wide(const hz_codebook* cb);
int select_dec_mode(const hz_codebook* cb);
int build_dec_dense(const hz_codebook* cb, std::vector<uint32_t>& img, int& K);
int build_dec_lut(const hz_codebook* cb, std::vector<uint32_t>& img, std::vector<uint32_t>& l2, int& K1, int& lvl);
void build_walk_len(const hz_codebook* cb, std::vector<uint32_t>& img, std::vector<uint32_t>& esc, int& K, int& M,
                    int& bias);
void build_walk8(const hz_codebook* cb, std::vector<uint32_t>& img, int& K);
void build_chain_esc(const hz_codebook* cb, std::vector<uint32_t>& img, int& M);
}  // namespace hz

using namespace hz;

// HZ_DEBUG=1: a failing HIP call is named on stderr (file line, call, HIP's message) before HZ_EHIP.
static int hz_hip_fail(hipError_t e, const char* what, int line) {
    static const bool dbg = getenv("HZ_DEBUG") != nullptr;
    if (dbg) fprintf(stderr, "[huffman_amd] hz_host.cpp:%d %s: %s\n", line, what, hipGetErrorString(e));
    return HZ_EHIP;
}
#define HZ_TRY(x) do { hipError_t _e = (x); if (_e != hipSuccess) return hz_hip_fail(_e, #x, __LINE__); } while (0)

// No C++ exception crosses the C ABI: entry points that allocate host
// containers run their body through this guard.
template <typename F>
static int guarded(F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return HZ_ENOMEM;
    } catch (...) {
        return HZ_EINVAL;
    }
}

// Pinned host staging for table uploads (see hz_codebook_upload_encode).
struct Staging {
    uint8_t* p = nullptr;
    size_t cap = 0, used = 0;
    hipEvent_t done = nullptr;
    std::vector<StageSeg> pend;  // staged, not yet copied (staging_flush)
};

struct hz_ctx {
    int device = 0;
    int ncu = 0;
    ChainState* chain = nullptr;    // the index-less decoder's phases (hz_decode_indexless, hz_indexless_*)
    hipStream_t stream = nullptr;
    bool own_stream = false;
    Tables t;
    unsigned long long* d_desc = nullptr;  // pack scratch: block counts, starts, tile sums
    uint64_t desc_cap = 0;          // u64 words
    uint32_t* d_err = nullptr;
    uint32_t* h_err = nullptr;      // pinned
    unsigned long long* d_thr = nullptr;
    unsigned long long* d_cbws = nullptr;  // hz_codebook_build_device workspace
    double thr_alpha = -1.0;
    hipEvent_t ev[5][2] = {};
    bool ev_used[5] = {false, false, false, false, false};
    // encode tables, decode tables, and the index-less decoder's tables (walk length and escape tables,
    // a DENSE codebook's chain LUT): built with the decode tables, copied by the first call that needs
    // them (hz_decode_indexless, hz_indexless_scan, hz_index_build) -- a decode with a block index never
    // uploads them
    Staging stage_enc, stage_dec, stage_walk;
    size_t cap_enc_lds = 0, cap_enc_esc = 0, cap_enc_wide = 0, cap_len8 = 0, cap_lenpair = 0, cap_dec_lds = 0,
           cap_dec_l2 = 0, cap_walk_lds = 0, cap_walk_esc = 0, cap_walk8 = 0, cap_chain_lds = 0, cap_chain_l2 = 0,
           cap_chain_esc = 0;
    int last_pack_ranges = 0;       // the last hz_pack_ranges call took the range plan
    // a FIXED16 part of hz_indexless_scan (every code 16 bits: positions are arithmetic, no chains)
    struct {
        bool on = false;
        const uint8_t* payload = nullptr;
        uint64_t bytes = 0, base = 0, start = 0, entry = 0, xit = 0;
    } fx;
};

extern "C" const char* hz_strerror(int st) {
    switch (st) {
        case HZ_OK: return "ok";
        case HZ_EINVAL: return "invalid argument";
        case HZ_ENOMEM: return "out of memory";
        case HZ_EHIP: return "HIP runtime error";
        case HZ_ETOOLONG: return "code longer than supported";
        case HZ_EFORMAT: return "malformed compressed stream";
        case HZ_ECAP: return "output capacity too small";
        case HZ_ETIMEOUT: return "device wait timed out";
        case HZ_EIO: return "file I/O error";
        case HZ_ENODEV: return "no usable gfx950 device";
        case HZ_ENOENT: return "input file does not exist";
        default: return "unknown error";
    }
}

extern "C" int hz_version(void) { return 1; }

static void free_tables(Tables& t) {
    (void)hipFree(t.d_enc_lds);
    (void)hipFree(t.d_enc_wide);
    (void)hipFree(t.d_enc_esc);
    (void)hipFree(t.d_len8);
    (void)hipFree(t.d_lenpair);
    (void)hipFree(t.d_dec_lds);
    (void)hipFree(t.d_dec_l2);
    (void)hipFree(t.d_walk_lds);
    (void)hipFree(t.d_walk_esc);
    (void)hipFree(t.d_walk8);
    (void)hipFree(t.d_chain_lds);
    (void)hipFree(t.d_chain_l2);
    (void)hipFree(t.d_chain_esc);
    t = Tables();
}

extern "C" int hz_ctx_create(int device, void* stream, hz_ctx** out) {
    if (!out) return HZ_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) return HZ_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return HZ_ENODEV;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return HZ_ENODEV;
    std::unique_ptr<hz_ctx> c(new hz_ctx());
    c->device = device;
    c->ncu = prop.multiProcessorCount;
    c->chain = chain_state_create();
    HZ_TRY(hipSetDevice(device));
    if (stream) {
        c->stream = (hipStream_t)stream;
    } else {
        HZ_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        c->own_stream = true;
    }
    HZ_TRY(hipMalloc(&c->d_err, 16));
    HZ_TRY(hipMemset(c->d_err, 0, 16));
    HZ_TRY(hipHostMalloc(&c->h_err, 16, hipHostMallocDefault));
    *c->h_err = 0;
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 2; ++j) HZ_TRY(hipEventCreate(&c->ev[i][j]));
    *out = c.release();
    return HZ_OK;
}

extern "C" int hz_ctx_destroy(hz_ctx* c) {
    if (!c) return HZ_EINVAL;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    free_tables(c->t);
    for (Staging* st : {&c->stage_enc, &c->stage_dec, &c->stage_walk}) {
        if (st->done) (void)hipEventDestroy(st->done);
        (void)hipHostFree(st->p);
    }
    chain_state_destroy(c->chain);
    (void)hipFree(c->d_desc);
    (void)hipFree(c->d_err);
    (void)hipFree(c->d_thr);
    (void)hipFree(c->d_cbws);
    (void)hipHostFree(c->h_err);
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 2; ++j) (void)hipEventDestroy(c->ev[i][j]);
    if (c->own_stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return HZ_OK;
}

extern "C" int hz_ctx_set_stream(hz_ctx* c, void* stream) {
    if (!c || !stream) return HZ_EINVAL;
    if (c->own_stream) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamDestroy(c->stream);
        c->own_stream = false;
    }
    c->stream = (hipStream_t)stream;
    return HZ_OK;
}

extern "C" int hz_ctx_sync(hz_ctx* c) {
    if (!c) return HZ_EINVAL;
    (void)hipSetDevice(c->device);
    HZ_TRY(hipStreamSynchronize(c->stream));
    if (*c->h_err) {
        const uint32_t e = *c->h_err;
        *c->h_err = 0;
        HZ_TRY(hipMemset(c->d_err, 0, 16));
        return (e & 4u) ? HZ_ECAP : (e & 8u) ? HZ_ETIMEOUT : (e & 16u) ? HZ_EINVAL : (e & 32u) ? HZ_ETOOLONG : HZ_EFORMAT;
    }
    return HZ_OK;
}

// Stage timing events: skipped while the stream is being captured into a graph (the stage calls
// themselves are stream-ordered and capturable; hz_last_kernel_ms then reports the last eager call).
static hipError_t stage_event(hz_ctx* c, int stage, int which) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    hipError_t e = hipStreamIsCapturing(c->stream, &st);
    if (e != hipSuccess) return e;
    if (st != hipStreamCaptureStatusNone) return hipSuccess;
    return hipEventRecord(c->ev[stage][which], c->stream);
}

static int arm_err_check(hz_ctx* c) {
    HZ_TRY(hipMemcpyAsync(c->h_err, c->d_err, 4, hipMemcpyDeviceToHost, c->stream));
    return HZ_OK;
}

extern "C" int hz_last_kernel_ms(hz_ctx* c, int stage, float* ms) {
    if (!c || !ms || stage < 0 || stage > 4) return HZ_EINVAL;
    if (!c->ev_used[stage]) { *ms = 0.f; return HZ_OK; }
    HZ_TRY(hipEventElapsedTime(ms, c->ev[stage][0], c->ev[stage][1]));
    return HZ_OK;
}

extern "C" int hz_hist16(hz_ctx* c, const uint8_t* d_in, uint64_t n, uint64_t* d_hist, int accumulate) {
    if (!c || !d_hist || (n && !d_in)) return HZ_EINVAL;
    HZ_TRY(hipSetDevice(c->device));
    if (!accumulate) HZ_TRY(hipMemsetAsync(d_hist, 0, HZ_NSYM * sizeof(uint64_t), c->stream));
    HZ_TRY(stage_event(c, HZ_STAGE_HIST, 0));
    HZ_TRY(launch_hist16(d_in, n, reinterpret_cast<unsigned long long*>(d_hist), c->ncu, c->stream));
    HZ_TRY(stage_event(c, HZ_STAGE_HIST, 1));
    c->ev_used[HZ_STAGE_HIST] = true;
    return HZ_OK;
}

extern "C" uint64_t hz_ranges_bytes(uint64_t n) { return range_geom(n / 2).bytes; }

extern "C" int hz_hist16_ranges(hz_ctx* c, const uint8_t* d_in, uint64_t n, uint64_t* d_hist, int accumulate,
                                void* d_ranges) {
    if (!c || !d_hist || (n && !d_in)) return HZ_EINVAL;
    if (!range_geom(n / 2).bytes) return hz_hist16(c, d_in, n, d_hist, accumulate);  // too small for a plan
    if (!d_ranges || (((uintptr_t)d_in) & 15) || (((uintptr_t)d_ranges) & 15)) return HZ_EINVAL;
    HZ_TRY(hipSetDevice(c->device));
    if (!accumulate) HZ_TRY(hipMemsetAsync(d_hist, 0, HZ_NSYM * sizeof(uint64_t), c->stream));
    HZ_TRY(stage_event(c, HZ_STAGE_HIST, 0));
    HZ_TRY(launch_hist16_ranges(d_in, n, reinterpret_cast<unsigned long long*>(d_hist), d_ranges, c->d_err,
                                c->stream));
    HZ_TRY(stage_event(c, HZ_STAGE_HIST, 1));
    c->ev_used[HZ_STAGE_HIST] = true;
    return arm_err_check(c);
}

extern "C" int hz_codebook_build_device(hz_ctx* c, const uint64_t* d_hist, hz_codebook* d_cb) {
    if (!c || !d_hist || !d_cb) return HZ_EINVAL;
    HZ_TRY(hipSetDevice(c->device));
    if (!c->d_cbws) HZ_TRY(hipMalloc(&c->d_cbws, codebook_ws_words() * sizeof(unsigned long long)));
    HZ_TRY(launch_codebook(reinterpret_cast<const unsigned long long*>(d_hist), d_cb, c->d_cbws, c->d_err, c->stream));
    return arm_err_check(c);
}

#ifdef HZ_CB_PROF  // variant builds only: k_cb_generate's phase timestamps (tools/debug/cb_prof.py)
extern "C" int hz_debug_cb_prof(hz_ctx* c, uint64_t* out) {
    HZ_TRY(hipStreamSynchronize(c->stream));
    HZ_TRY(hipMemcpy(out, c->d_cbws + 65536, 512 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return HZ_OK;
}
#endif

extern "C" int hz_header_write_device(hz_ctx* c, const hz_codebook* d_cb, uint64_t n, uint8_t last_byte,
                                      uint8_t* d_out, uint64_t cap, uint64_t* d_info) {
    if (!c || !d_cb || !d_out || !d_info || (((uintptr_t)d_out) & 3)) return HZ_EINVAL;
    HZ_TRY(hipSetDevice(c->device));
    if (!c->d_cbws) HZ_TRY(hipMalloc(&c->d_cbws, codebook_ws_words() * sizeof(unsigned long long)));
    HZ_TRY(launch_header_write(d_cb, n, last_byte, d_out, cap, reinterpret_cast<unsigned long long*>(d_info), c->d_cbws,
                               c->d_err, c->stream));
    return arm_err_check(c);
}

extern "C" int hz_header_parse_device(hz_ctx* c, const uint8_t* d_file, uint64_t len, hz_codebook* d_cb,
                                      uint64_t* d_info) {
    if (!c || !d_file || !d_cb || !d_info) return HZ_EINVAL;
    HZ_TRY(hipSetDevice(c->device));
    if (!c->d_cbws) HZ_TRY(hipMalloc(&c->d_cbws, codebook_ws_words() * sizeof(unsigned long long)));
    HZ_TRY(launch_header_parse(d_file, len, d_cb, reinterpret_cast<unsigned long long*>(d_info), c->d_cbws, c->d_err,
                               c->stream));
    return arm_err_check(c);
}

// Device tables live in per-context buffers that only grow; host images are
// staged in pinned memory and copied asynchronously on the context stream (one
// scatter kernel per set), so an upload never synchronises and the decode tables
// can be built on the host while the pack kernel runs (bench step: upload_encode
// -> pack -> upload_decode -> decode). Stream order keeps in-flight kernels on the
// previous tables; a staging buffer is reused only after its last copy's event.
static int staging_begin(Staging& st) {
    if (!st.done) HZ_TRY(hipEventCreateWithFlags(&st.done, hipEventDisableTiming));
    else HZ_TRY(hipEventSynchronize(st.done));
    st.used = 0;
    st.pend.clear();  // (a set never flushed is dropped)
    return HZ_OK;
}

// The staged segments to their tables, stream-ordered. Under stream capture the copy is captured and
// the segments stay pending, so a later uncaptured call copies them again.
static int staging_flush(hz_ctx* c, Staging& st) {
    if (st.pend.empty()) return HZ_OK;
    HZ_TRY(stage_scatter(st.p, st.pend.data(), (int)st.pend.size(), c->stream));
    HZ_TRY(hipEventRecord(st.done, c->stream));
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HZ_TRY(hipStreamIsCapturing(c->stream, &cs));
    if (cs == hipStreamCaptureStatusNone) st.pend.clear();
    return HZ_OK;
}

template <typename T>
static int stage_copy(hz_ctx* c, Staging& st, T** dptr, size_t* dcap, const std::vector<T>& v) {
    const size_t bytes = v.size() * sizeof(T);
    if (*dcap < bytes) {
        HZ_TRY(hipStreamSynchronize(c->stream));
        (void)hipFree(*dptr);
        *dptr = nullptr;
        HZ_TRY(hipMalloc(dptr, bytes));
        *dcap = bytes;
    }
    if (st.used + bytes > st.cap) {
        // grow (rare): the segments staged so far move along (no copy of this staging is in flight:
        // staging_begin waited for the last one)
        uint8_t* np = nullptr;
        const size_t ncap = std::max(st.cap * 2, st.used + bytes + (1u << 20));
        HZ_TRY(hipHostMalloc(&np, ncap, hipHostMallocDefault));
        if (st.used) memcpy(np, st.p, st.used);
        (void)hipHostFree(st.p);
        st.p = np;
        st.cap = ncap;
    }
    static_assert(sizeof(T) % 4 == 0, "tables of 4-byte words (k_stage_scatter)");
    memcpy(st.p + st.used, v.data(), bytes);
    if (bytes) st.pend.push_back(StageSeg{(void*)*dptr, (uint64_t)st.used, (uint64_t)bytes});
    st.used += (bytes + 255) & ~(size_t)255;
    return HZ_OK;
}

static int hz_codebook_upload_encode_impl(hz_ctx* c, const hz_codebook* cb) {
    if (!c || !cb) return HZ_EINVAL;
    if (cb->max_len > HZ_MAXLEN) return HZ_ETOOLONG;
    HZ_TRY(hipSetDevice(c->device));
    Tables& t = c->t;
    t.enc_mode = -1;
    if (cb->nsym == 0) return HZ_OK;
    int rc;
    if ((rc = staging_begin(c->stage_enc))) return rc;
    t.max_len = (int)cb->max_len;
    t.min_len = (int)cb->min_len;
    const int mode = select_enc_mode(cb);
    {
        // expected bits per symbol under the code's own distribution (Kraft weights 2^-L)
        uint64_t nl[HZ_MAXLEN + 1] = {0};
        for (uint32_t s = 0; s < HZ_NSYM; ++s) nl[cb->len[s]]++;
        double avg = 0.0;
        for (int L = 1; L <= HZ_MAXLEN; ++L) avg += ldexp((double)nl[L], -L) * L;
        t.enc_avg_bits = avg > 0.0 ? avg : 1.0;
    }
    if (mode == ENC_FIXED16) {
        std::vector<uint32_t> img = build_enc_fixed16(cb);
        t.enc_lds_bytes = (uint32_t)(img.size() * 4);
        if ((rc = stage_copy(c, c->stage_enc, &t.d_enc_lds, &c->cap_enc_lds, img))) return rc;
    } else if (mode == ENC_DENSE) {
        std::vector<uint32_t> img = build_enc_dense(cb);
        t.enc_lds_bytes = (uint32_t)(img.size() * 4);
        if ((rc = stage_copy(c, c->stage_enc, &t.d_enc_lds, &c->cap_enc_lds, img))) return rc;
    } else if (mode == ENC_HOT) {
        t.hot_mask = choose_hot_mask(cb);
        std::vector<uint32_t> img = build_enc_hot(cb, t.hot_mask);
        t.enc_lds_bytes = (uint32_t)(img.size() * 4);
        if ((rc = stage_copy(c, c->stage_enc, &t.d_enc_lds, &c->cap_enc_lds, img))) return rc;
        if ((rc = stage_copy(c, c->stage_enc, &t.d_enc_esc, &c->cap_enc_esc, build_enc_esc(cb, t.hot_mask)))) return rc;
    }
    if (mode == ENC_WIDE &&
        (rc = stage_copy(c, c->stage_enc, &t.d_enc_wide, &c->cap_enc_wide, build_enc_wide(cb))))
        return rc;
    if (mode != ENC_FIXED16 && (rc = stage_copy(c, c->stage_enc, &t.d_len8, &c->cap_len8, build_len8(cb))))
        return rc;
    if (mode != ENC_FIXED16 &&
        (rc = stage_copy(c, c->stage_enc, &t.d_lenpair, &c->cap_lenpair, build_lenpair(cb))))
        return rc;
    if ((rc = staging_flush(c, c->stage_enc))) return rc;
    t.enc_mode = mode;
    return HZ_OK;
}

extern "C" int hz_codebook_upload_encode(hz_ctx* c, const hz_codebook* cb) {
    return guarded([&] { return hz_codebook_upload_encode_impl(c, cb); });
}

static int hz_codebook_upload_decode_impl(hz_ctx* c, const hz_codebook* cb) {
    if (!c || !cb) return HZ_EINVAL;
    if (cb->max_len > HZ_MAXLEN) return HZ_ETOOLONG;
    HZ_TRY(hipSetDevice(c->device));
    Tables& t = c->t;
    t.dec_mode = -1;
    chain_invalidate(c->chain);  // its arguments point at the tables replaced here
    c->fx.on = false;
    if (cb->nsym == 0) return HZ_OK;
    int rc;
    if ((rc = staging_begin(c->stage_dec))) return rc;
    t.dec_max_len = (int)cb->max_len;
    t.dec_min_len = (int)cb->min_len;
    const int mode = select_dec_mode(cb);
    std::vector<uint32_t> dimg, l2, wimg, wesc;
    if (mode == DEC_FIXED16) { dimg = build_dec_fixed16(cb); t.dec_k = 16; rc = HZ_OK; }
    else if (mode == DEC_DENSE) rc = build_dec_dense(cb, dimg, t.dec_k);
    else rc = build_dec_lut(cb, dimg, l2, t.dec_k, t.dec_level_bits);
    if (rc) return rc;
    t.dec_avg_bits = 0.0;  // Kraft estimate of bits per codeword (sizes the index-less decoder's records)
    for (uint32_t s = 0; s < HZ_NSYM; ++s)
        if (cb->len[s]) t.dec_avg_bits += ldexp((double)cb->len[s], -(int)cb->len[s]);
    while (dimg.size() % 4) dimg.push_back(0);
    t.dec_lds_bytes = (uint32_t)(dimg.size() * 4);
    if (mode != DEC_FIXED16 && t.dec_lds_bytes + 4 * dec_slot_words_max(t.dec_max_len) > kLdsBytes)
        return HZ_ENOMEM;  // cannot happen for K1 <= 14 and codes <= 56 bits
    if ((rc = stage_copy(c, c->stage_dec, &t.d_dec_lds, &c->cap_dec_lds, dimg))) return rc;
    if (l2.empty()) l2.push_back(lut_leaf_entry(1, 0));
    t.dec_l2_entries = l2.size();
    if ((rc = stage_copy(c, c->stage_dec, &t.d_dec_l2, &c->cap_dec_l2, l2))) return rc;
    if ((rc = staging_flush(c, c->stage_dec))) return rc;
    // the index-less tables, staged now and copied by the first call that needs them (staging_flush
    // from hz_decode_indexless, hz_indexless_scan or hz_index_build)
    if ((rc = staging_begin(c->stage_walk))) return rc;
    // the index walker's length tables (FIXED16 streams have an arithmetic index)
    t.walk_lds_bytes = 0;
    t.walk8_bytes = 0;
    t.chain_lds_bytes = 0;
    if (mode != DEC_FIXED16 && cb->max_len >= 1 && cb->max_len <= kWalkMaxLen) {
        build_walk_len(cb, wimg, wesc, t.walk_k, t.walk_m, t.walk_bias);
        if (wimg.size() * 4 <= (1u << kWalkK) / 2) {  // k_idx_walk's static table
            if ((rc = stage_copy(c, c->stage_walk, &t.d_walk_lds, &c->cap_walk_lds, wimg))) return rc;
            if (wesc.empty()) wesc.push_back(0x01010101u);
            if ((rc = stage_copy(c, c->stage_walk, &t.d_walk_esc, &c->cap_walk_esc, wesc))) return rc;
            t.walk_lds_bytes = (uint32_t)(wimg.size() * 4);
        }
    }
    // the index-less chain decoder's tables (every codebook but FIXED16): the byte length table, the
    // escape table (the index walker's when it has one: codes <= kWalkMaxLen bits), LUT decode images
    if (mode != DEC_FIXED16 && cb->max_len >= 1) {
        std::vector<uint32_t> w8;
        build_walk8(cb, w8, t.walk8_k);
        if ((rc = stage_copy(c, c->stage_walk, &t.d_walk8, &c->cap_walk8, w8))) return rc;
        t.walk8_bytes = (uint32_t)(w8.size() * 4);
        if (t.walk_lds_bytes > 0) {
            t.chain_esc = reinterpret_cast<const uint8_t*>(t.d_walk_esc);
            t.chain_esc_m = t.walk_m;
        } else {
            std::vector<uint32_t> cesc;
            build_chain_esc(cb, cesc, t.chain_esc_m);
            if ((rc = stage_copy(c, c->stage_walk, &t.d_chain_esc, &c->cap_chain_esc, cesc))) return rc;
            t.chain_esc = reinterpret_cast<const uint8_t*>(t.d_chain_esc);
        }
        if (mode == DEC_LUT) {
            t.chain_lds = t.d_dec_lds;
            t.chain_l2 = t.d_dec_l2;
            t.chain_lds_bytes = t.dec_lds_bytes;
            t.chain_k = t.dec_k;
            t.chain_level_bits = t.dec_level_bits;
        } else {  // DENSE: a LUT image beside the DENSE decoder's
            std::vector<uint32_t> cimg, cl2;
            if ((rc = build_dec_lut(cb, cimg, cl2, t.chain_k, t.chain_level_bits))) return rc;
            while (cimg.size() % 4) cimg.push_back(0);
            if (cl2.empty()) cl2.push_back(lut_leaf_entry(1, 0));
            if ((rc = stage_copy(c, c->stage_walk, &t.d_chain_lds, &c->cap_chain_lds, cimg))) return rc;
            if ((rc = stage_copy(c, c->stage_walk, &t.d_chain_l2, &c->cap_chain_l2, cl2))) return rc;
            t.chain_lds = t.d_chain_lds;
            t.chain_l2 = t.d_chain_l2;
            t.chain_lds_bytes = (uint32_t)(cimg.size() * 4);
        }
    }
    t.dec_mode = mode;
    return HZ_OK;
}

extern "C" int hz_codebook_upload_decode(hz_ctx* c, const hz_codebook* cb) {
    return guarded([&] { return hz_codebook_upload_decode_impl(c, cb); });
}

extern "C" int hz_codebook_upload(hz_ctx* c, const hz_codebook* cb) {
    int rc = hz_codebook_upload_encode(c, cb);
    return rc ? rc : hz_codebook_upload_decode(c, cb);
}

extern "C" int hz_index_format(void) { return HZ_INDEX_FORMAT; }
extern "C" uint64_t hz_index_stride(void) { return kBlockSyms; }
extern "C" uint64_t hz_index_bytes(uint64_t nsym) { return index_bytes(nsym); }
extern "C" uint64_t hz_scratch_bytes(uint64_t nsym) { return pack_scratch_words(nsym) * sizeof(uint64_t); }

// Every call that writes the context's scratch (or reallocates it, or replaces the decode tables) ends
// a pending index-less part (hz_indexless_scan ... hz_indexless_decode): its chain state points there.
static int ensure_scratch(hz_ctx* c, uint64_t words) {
    chain_invalidate(c->chain);
    c->fx.on = false;
    if (c->desc_cap >= words) return HZ_OK;
    HZ_TRY(hipStreamSynchronize(c->stream));
    (void)hipFree(c->d_desc);
    c->d_desc = nullptr;
    c->desc_cap = 0;
    HZ_TRY(hipMalloc(&c->d_desc, words * sizeof(unsigned long long)));
    c->desc_cap = words;
    return HZ_OK;
}

static int pack_impl(hz_ctx* c, const uint8_t* d_in, uint64_t n, uint64_t start_bit, uint32_t lead, uint8_t* d_out,
                     uint64_t out_cap, uint64_t* d_index, void* d_ranges) {
    if (!c || !d_out) return HZ_EINVAL;
    if (((uintptr_t)d_out) & 3) return HZ_EINVAL;
    const uint64_t nsym = n / 2;
    if (nsym == 0) return HZ_OK;
    if (!d_in || (((uintptr_t)d_in) & 15)) return HZ_EINVAL;
    if (c->t.enc_mode < 0) return HZ_EINVAL;
    // d_out must hold ceil((start_bit + payload_bits) / 32) words; the kernel
    // drops (and flags HZ_ECAP) any block that would write past out_cap.
    if (out_cap < 4) return HZ_ECAP;
    HZ_TRY(hipSetDevice(c->device));
    int rc = ensure_scratch(c, pack_scratch_words(nsym));
    if (rc) return rc;
    HZ_TRY(stage_event(c, HZ_STAGE_PACK, 0));
    HZ_TRY(launch_pack(c->t, d_in, nsym, start_bit, lead, reinterpret_cast<uint32_t*>(d_out), out_cap / 4, c->d_desc,
                       reinterpret_cast<unsigned long long*>(d_index), c->d_err, c->ncu, c->stream, d_ranges,
                       &c->last_pack_ranges));
    HZ_TRY(stage_event(c, HZ_STAGE_PACK, 1));
    c->ev_used[HZ_STAGE_PACK] = true;
    return arm_err_check(c);
}

extern "C" int hz_pack(hz_ctx* c, const uint8_t* d_in, uint64_t n, uint64_t start_bit, uint32_t lead, uint8_t* d_out,
                       uint64_t out_cap, uint64_t* d_index) {
    return pack_impl(c, d_in, n, start_bit, lead, d_out, out_cap, d_index, nullptr);
}

extern "C" int hz_pack_ranges(hz_ctx* c, const uint8_t* d_in, uint64_t n, uint64_t start_bit, uint32_t lead,
                              uint8_t* d_out, uint64_t out_cap, uint64_t* d_index, void* d_ranges) {
    if (c) c->last_pack_ranges = 0;
    if (range_geom(n / 2).bytes && (!d_ranges || (((uintptr_t)d_ranges) & 15))) return HZ_EINVAL;
    return pack_impl(c, d_in, n, start_bit, lead, d_out, out_cap, d_index, range_geom(n / 2).bytes ? d_ranges : nullptr);
}

extern "C" int hz_last_pack_ranges(hz_ctx* c) { return c ? c->last_pack_ranges : 0; }

extern "C" int hz_decode(hz_ctx* c, const uint8_t* d_payload, uint64_t payload_bytes, uint64_t nsym,
                         const uint64_t* d_index, uint8_t* d_out) {
    if (!c) return HZ_EINVAL;
    if (nsym == 0) return HZ_OK;
    if (!d_payload || !d_index || !d_out || (((uintptr_t)d_out) & 15)) return HZ_EINVAL;
    if (c->t.dec_mode < 0) return HZ_EINVAL;
    HZ_TRY(hipSetDevice(c->device));
    HZ_TRY(stage_event(c, HZ_STAGE_DECODE, 0));
    HZ_TRY(launch_decode(c->t, d_payload, payload_bytes, nsym, reinterpret_cast<const unsigned long long*>(d_index),
                         d_out, c->d_err, c->ncu, c->stream));
    HZ_TRY(stage_event(c, HZ_STAGE_DECODE, 1));
    c->ev_used[HZ_STAGE_DECODE] = true;
    return arm_err_check(c);
}

extern "C" int hz_index_build(hz_ctx* c, const uint8_t* d_payload, uint64_t payload_bytes, uint64_t start_bit,
                              uint64_t nsym, uint64_t* d_index) {
    if (!c) return HZ_EINVAL;
    if (nsym == 0) return HZ_OK;
    if (!d_payload || !d_index) return HZ_EINVAL;
    if (c->t.dec_mode < 0) return HZ_EINVAL;
    HZ_TRY(hipSetDevice(c->device));
    // nsym codewords end within nsym * max_len bits: the rest of a longer buffer is never walked
    const uint64_t reach = (start_bit + nsym * (uint64_t)std::max(c->t.dec_max_len, 1) + 7) / 8 + 8;
    if (nsym <= (UINT64_MAX - start_bit) / 64 && payload_bytes > reach) payload_bytes = reach;
    int rc = ensure_scratch(c, index_scratch_words(payload_bytes, start_bit));
    if (rc) return rc;
    if ((rc = staging_flush(c, c->stage_walk))) return rc;  // the walk tables
    HZ_TRY(stage_event(c, HZ_STAGE_INDEX, 0));
    HZ_TRY(launch_index_build(c->t, d_payload, payload_bytes, start_bit, nsym,
                              reinterpret_cast<unsigned long long*>(d_index), c->d_desc, c->d_err, c->h_err + 2,
                              c->ncu, c->stream));
    HZ_TRY(stage_event(c, HZ_STAGE_INDEX, 1));
    c->ev_used[HZ_STAGE_INDEX] = true;
    return arm_err_check(c);
}

extern "C" int hz_decode_indexless(hz_ctx* c, const uint8_t* d_payload, uint64_t payload_bytes, uint64_t start_bit,
                                   uint64_t nsym, uint8_t* d_out, uint64_t* d_end_bit) {
    if (!c) return HZ_EINVAL;
    if (nsym == 0) return HZ_OK;
    if (!d_payload || !d_out || (((uintptr_t)d_out) & 15)) return HZ_EINVAL;
    if (c->t.dec_mode < 0) return HZ_EINVAL;
    HZ_TRY(hipSetDevice(c->device));
    // nsym codewords end within nsym * max_len bits: the rest of a longer buffer is never walked
    const uint64_t reach = (start_bit + nsym * (uint64_t)std::max(c->t.dec_max_len, 1) + 7) / 8 + 8;
    if (nsym <= (UINT64_MAX - start_bit) / 64 && payload_bytes > reach) payload_bytes = reach;
    if (c->t.dec_mode == DEC_FIXED16) {
        // every code 16 bits: symbol i at start_bit + 16 i, so no index and no walk (stream-ordered)
        const uint64_t endb = nsym <= (UINT64_MAX - start_bit) / 16 ? start_bit + 16 * nsym : ~0ull;
        const bool fits = endb <= payload_bytes * 8;  // else: the end bit past the payload, nothing decoded
        HZ_TRY(stage_event(c, HZ_STAGE_EXTRACT, 0));
        if (d_end_bit) {
            const uint64_t eb = fits ? endb : ~0ull;
            HZ_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_end_bit), (int)(uint32_t)eb, 1, c->stream));
            HZ_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(reinterpret_cast<uint32_t*>(d_end_bit) + 1),
                                     (int)(uint32_t)(eb >> 32), 1, c->stream));
        }
        if (fits)
            HZ_TRY(launch_decode(c->t, d_payload, payload_bytes, nsym, nullptr, d_out, c->d_err, c->ncu, c->stream,
                                 start_bit));
        HZ_TRY(stage_event(c, HZ_STAGE_EXTRACT, 1));
        c->ev_used[HZ_STAGE_EXTRACT] = true;
        return arm_err_check(c);
    }
    if (!seg_decode_supported(c->t)) return HZ_EINVAL;  // (every codebook but FIXED16 has chain tables)
    {
        const int rf = staging_flush(c, c->stage_walk);  // the chain tables
        if (rf) return rf;
    }
    if (payload_bytes < 16) {  // too short for the walk: one thread, serially (stream-ordered too)
        HZ_TRY(stage_event(c, HZ_STAGE_EXTRACT, 0));
        HZ_TRY(chain_decode_tiny(c->t, d_payload, payload_bytes, start_bit, nsym, d_out,
                                 reinterpret_cast<unsigned long long*>(d_end_bit), c->d_err, c->stream));
        HZ_TRY(stage_event(c, HZ_STAGE_EXTRACT, 1));
        c->ev_used[HZ_STAGE_EXTRACT] = true;
        return arm_err_check(c);
    }
    // stream-ordered from here: walk, fix-ups, scans, block decode, tails (no host synchronisation
    // unless the context's scratch has to grow)
    const uint64_t pbits = payload_bytes * 8 > start_bit ? payload_bytes * 8 - start_bit : 0;
    int rc = ensure_scratch(c, chain_scratch_words(0, pbits, nsym, c->t, c->ncu));
    if (rc) return rc;
    HZ_TRY(stage_event(c, HZ_STAGE_EXTRACT, 0));
    HZ_TRY(chain_scan(c->chain, c->t, d_payload, payload_bytes, 0, start_bit, nsym, 0, pbits, ~0ull, c->d_desc,
                      c->d_err, c->ncu, c->stream));
    HZ_TRY(chain_decode(c->chain, c->t, nsym, d_out, reinterpret_cast<unsigned long long*>(d_end_bit), c->ncu,
                        c->stream));
    chain_invalidate(c->chain);  // not a part: hz_indexless_refix / _decode may not continue it
    HZ_TRY(stage_event(c, HZ_STAGE_EXTRACT, 1));
    c->ev_used[HZ_STAGE_EXTRACT] = true;
    return arm_err_check(c);
}

// ---- one stream over several devices: the index-less decode in parts -----------------
static int part_summary(hz_ctx* c, uint64_t* d_summary) {
    if (!d_summary) return HZ_OK;
    if (!chain_info(c->chain)) return HZ_EINVAL;
    HZ_TRY(chain_summary(c->chain, reinterpret_cast<unsigned long long*>(d_summary), c->stream));
    return HZ_OK;
}

// FIXED16 parts: codeword i starts at start + 16 i, so a part's entry, exit and count are arithmetic.
static int fixed_part_summary(hz_ctx* c, uint64_t* d_summary) {
    if (!d_summary) return HZ_OK;
    HZ_TRY(put3(reinterpret_cast<unsigned long long*>(d_summary), (c->fx.xit - c->fx.entry) / 16, c->fx.xit,
                c->fx.entry, c->stream));
    return HZ_OK;
}

extern "C" int hz_indexless_scan(hz_ctx* c, const uint8_t* d_payload, uint64_t payload_bytes, uint64_t payload_bit_base,
                                 uint64_t start_bit, uint64_t nsym, uint64_t part_begin, uint64_t part_end,
                                 uint64_t entry_bit, uint64_t* d_summary) {
    if (!c || !d_payload || part_end <= part_begin || payload_bytes < 16) return HZ_EINVAL;
    if (c->t.dec_mode < 0) return HZ_EINVAL;
    if (start_bit > UINT64_MAX - part_end || payload_bytes > (UINT64_MAX - payload_bit_base) / 8) return HZ_EINVAL;
    // the view must hold the part, and the lead-in before it (the stream's bits from its start, when the
    // part begins less than HZ_INDEXLESS_LEAD_BITS into it)
    const uint64_t lead = part_begin < HZ_INDEXLESS_LEAD_BITS ? part_begin : HZ_INDEXLESS_LEAD_BITS;
    if (start_bit + part_begin - lead < payload_bit_base) return HZ_EINVAL;
    if (start_bit + part_end > payload_bit_base + payload_bytes * 8) return HZ_EINVAL;
    HZ_TRY(hipSetDevice(c->device));
    chain_invalidate(c->chain);
    c->fx.on = false;
    if (c->t.dec_mode == DEC_FIXED16) {
        c->fx.payload = d_payload;
        c->fx.bytes = payload_bytes;
        c->fx.base = payload_bit_base;
        c->fx.start = start_bit;
        c->fx.entry = entry_bit != UINT64_MAX ? entry_bit : start_bit + 16 * ((part_begin + 15) / 16);
        c->fx.xit = start_bit + 16 * ((part_end + 15) / 16);
        if (c->fx.entry < start_bit || (c->fx.entry - start_bit) % 16 || c->fx.entry > c->fx.xit) return HZ_EINVAL;
        c->fx.on = true;
        return fixed_part_summary(c, d_summary);
    }
    if (!seg_decode_supported(c->t)) return HZ_EINVAL;
    // record capacity from the stream's own bits per codeword when the caller knows its symbols
    const uint64_t pbits = payload_bit_base + payload_bytes * 8 > start_bit ? payload_bit_base + payload_bytes * 8 - start_bit : 0;
    const uint64_t hint = nsym ? std::max<uint64_t>(1, (uint64_t)((double)nsym * (double)(part_end - part_begin) /
                                                                  (double)std::max<uint64_t>(pbits, 1))) : 0;
    int rc = ensure_scratch(c, chain_scratch_words(part_begin, part_end, hint, c->t, c->ncu));
    if (rc) return rc;
    if ((rc = staging_flush(c, c->stage_walk))) return rc;  // the chain tables
    HZ_TRY(chain_scan(c->chain, c->t, d_payload, payload_bytes, payload_bit_base, start_bit, hint, part_begin, part_end,
                      entry_bit, c->d_desc, c->d_err, c->ncu, c->stream));
    if ((rc = part_summary(c, d_summary))) return rc;
    return arm_err_check(c);
}

extern "C" int hz_indexless_refix(hz_ctx* c, uint64_t entry_bit, uint64_t* d_summary) {
    if (c && c->fx.on) {
        if (entry_bit < c->fx.start || (entry_bit - c->fx.start) % 16 || entry_bit > c->fx.xit) return HZ_EINVAL;
        HZ_TRY(hipSetDevice(c->device));
        c->fx.entry = entry_bit;
        return fixed_part_summary(c, d_summary);
    }
    if (!c || !chain_info(c->chain)) return HZ_EINVAL;
    HZ_TRY(hipSetDevice(c->device));
    HZ_TRY(chain_refix(c->chain, c->t, entry_bit, c->ncu, c->stream));
    int rc = part_summary(c, d_summary);
    if (rc) return rc;
    return arm_err_check(c);
}

extern "C" int hz_indexless_decode(hz_ctx* c, uint64_t nsym, uint8_t* d_out, uint64_t* d_end_bit) {
    if (c && c->fx.on) {
        if (nsym && (!d_out || (((uintptr_t)d_out) & 15))) return HZ_EINVAL;
        HZ_TRY(hipSetDevice(c->device));
        const uint64_t count = (c->fx.xit - c->fx.entry) / 16;
        const uint64_t take = nsym < count ? nsym : count;
        if (take)
            HZ_TRY(launch_decode(c->t, c->fx.payload, c->fx.bytes, take, nullptr, d_out, c->d_err, c->ncu, c->stream,
                                 c->fx.entry - c->fx.base));
        if (d_end_bit) {
            const uint64_t eb = nsym && nsym <= count ? c->fx.entry + 16 * nsym : UINT64_MAX;
            HZ_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_end_bit), (int)(uint32_t)eb, 1, c->stream));
            HZ_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(reinterpret_cast<uint32_t*>(d_end_bit) + 1),
                                     (int)(uint32_t)(eb >> 32), 1, c->stream));
        }
        return arm_err_check(c);
    }
    if (!c || !chain_info(c->chain)) return HZ_EINVAL;
    if (nsym && (!d_out || (((uintptr_t)d_out) & 15))) return HZ_EINVAL;
    HZ_TRY(hipSetDevice(c->device));
    HZ_TRY(chain_decode(c->chain, c->t, nsym, d_out, reinterpret_cast<unsigned long long*>(d_end_bit), c->ncu,
                        c->stream));
    return arm_err_check(c);
}

// Zipf thresholds: thr[r-1] = floor(2^64 * sum_{j<=r} j^-alpha / H); thr[255] = max.
static void zipf_thresholds(double alpha, unsigned long long* thr) {
    double H = 0.0;
    for (int r = 1; r <= 256; ++r) H += pow((double)r, -alpha);
    double cum = 0.0;
    for (int r = 1; r <= 256; ++r) {
        cum += pow((double)r, -alpha);
        const double x = cum / H;
        thr[r - 1] = (r == 256 || x >= 1.0) ? ~0ull : (unsigned long long)ldexp(x, 64);
    }
}

extern "C" int hz_generate(hz_ctx* c, uint8_t* d_out, uint64_t n, uint64_t offset, int kind, double alpha,
                           uint64_t seed) {
    if (!c || (n && !d_out) || kind < 0 || kind > 1) return HZ_EINVAL;
    HZ_TRY(hipSetDevice(c->device));
    if (!c->d_thr) HZ_TRY(hipMalloc(&c->d_thr, 256 * sizeof(unsigned long long)));
    if (kind == 1 && c->thr_alpha != alpha) {
        static unsigned long long thr[256];
        zipf_thresholds(alpha, thr);
        HZ_TRY(hipMemcpy(c->d_thr, thr, sizeof(thr), hipMemcpyHostToDevice));
        c->thr_alpha = alpha;
    }
    HZ_TRY(launch_generate(d_out, n, offset, kind, seed, c->d_thr, c->stream));
    return HZ_OK;
}

// ---------------------------------------------------------------------------
// Whole-buffer flows (device work inside) used by the CLI and tests.
// ---------------------------------------------------------------------------
namespace {

constexpr uint64_t kArchiveChunk = 256ull << 20;  // archive: 256 MiB per streamed chunk (~1.2 GB pinned)
constexpr uint64_t kExtractWindow = 256ull << 20; // extract: 256 MiB payload windows (16 GiB: 1.9 s vs 2.6 s at 512 MiB, 3.2 s at 128)

std::mutex g_mu;
hz_ctx* g_ctx = nullptr;

int default_ctx(hz_ctx** out) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_ctx) {
        int rc = hz_ctx_create(0, nullptr, &g_ctx);
        if (rc) return rc;
    }
    *out = g_ctx;
    return HZ_OK;
}

struct DevBuf {
    void* p = nullptr;
    ~DevBuf() { if (p) (void)hipFree(p); }
    int alloc(size_t n) { return hipMalloc(&p, n ? n : 16) == hipSuccess ? HZ_OK : HZ_ENOMEM; }
};

struct EncodePlan {
    std::unique_ptr<hz_codebook> cb{new hz_codebook()};
    std::vector<uint64_t> hist = std::vector<uint64_t>(HZ_NSYM);
    uint64_t header_bits = 0, payload_bits = 0;
};

// Histogram on the device, codebook on the host.
int plan_encode(hz_ctx* c, const uint8_t* d_in, uint64_t n, EncodePlan& p) {
    DevBuf dh;
    int rc = dh.alloc(HZ_NSYM * 8);
    if (rc) return rc;
    if ((rc = hz_hist16(c, d_in, n, (uint64_t*)dh.p, 0))) return rc;
    HZ_TRY(hipMemcpyAsync(p.hist.data(), dh.p, HZ_NSYM * 8, hipMemcpyDeviceToHost, c->stream));
    if ((rc = hz_ctx_sync(c))) return rc;
    if ((rc = hz_codebook_build(p.hist.data(), p.cb.get()))) return rc;
    hz_header_bits(p.cb.get(), n, &p.header_bits);
    hz_payload_bits(p.cb.get(), p.hist.data(), &p.payload_bits);
    return HZ_OK;
}

// Encode a host buffer into a complete .compressed image.
int encode_image(const uint8_t* in, uint64_t n, std::vector<uint8_t>& out, uint32_t* nsym_out) {
    hz_ctx* c;
    int rc = default_ctx(&c);
    if (rc) return rc;
    HZ_TRY(hipSetDevice(c->device));
    DevBuf din;
    if ((rc = din.alloc(n))) return rc;
    if (n) HZ_TRY(hipMemcpyAsync(din.p, in, n, hipMemcpyHostToDevice, c->stream));
    EncodePlan p;
    if ((rc = plan_encode(c, (const uint8_t*)din.p, n, p))) return rc;
    if (nsym_out) *nsym_out = p.cb->nsym;
    const uint64_t hbytes_full = p.header_bits / 8;
    const uint64_t total_bits = p.header_bits + p.payload_bits;
    const uint64_t file_bytes = (total_bits + 7) / 8;
    out.assign(file_bytes + 8, 0);
    uint64_t hb;
    uint32_t pend_bits;
    uint8_t pend;
    rc = hz_header_write(p.cb.get(), n, n & 1 ? in[n - 1] : 0, out.data(), out.size(), &hb, &pend_bits, &pend);
    if (rc) return rc;
    if (hb != hbytes_full) return HZ_EINVAL;
    const uint64_t nsym = n / 2;
    if (nsym > 0) {
        if ((rc = hz_codebook_upload(c, p.cb.get()))) return rc;
        const uint64_t start_bit = pend_bits;
        const uint64_t pay_bytes = file_bytes - hbytes_full;
        const uint64_t words = (start_bit + p.payload_bits + 31) / 32;
        DevBuf dout;
        if ((rc = dout.alloc(words * 4))) return rc;
        if ((rc = hz_pack(c, (const uint8_t*)din.p, n, start_bit, (uint32_t)(pend >> (8 - pend_bits)) * (pend_bits ? 1 : 0),
                          (uint8_t*)dout.p, words * 4, nullptr)))
            return rc;
        HZ_TRY(hipMemcpyAsync(out.data() + hbytes_full, dout.p, pay_bytes, hipMemcpyDeviceToHost, c->stream));
        if ((rc = hz_ctx_sync(c))) return rc;
    } else if (pend_bits) {
        out[hbytes_full] = pend;  // unreachable (header is byte aligned without symbols) but kept exact
    }
    out.resize(file_bytes);
    return HZ_OK;
}

// Decode a complete .compressed image.
int decode_image(const uint8_t* f, uint64_t len, std::vector<uint8_t>& out) {
    std::unique_ptr<hz_codebook> cb(new hz_codebook());
    hz_header_info info;
    int rc = hz_header_parse(f, len, cb.get(), &info);
    if (rc) return rc;
    const uint64_t nsym = info.n / 2;
    const uint64_t pay = len - info.payload_byte;
    // every codeword is >= min_len bits: a header claiming more symbols than the
    // payload can hold is malformed (checked before anything is allocated)
    const uint64_t pay_bits = pay * 8 > info.payload_bit ? pay * 8 - info.payload_bit : 0;
    if (nsym > 0 && nsym > pay_bits / std::max<uint32_t>(cb->min_len, 1)) return HZ_EFORMAT;
    try {
        out.assign(2 * nsym + (info.is_odd ? 1 : 0), 0);
    } catch (const std::bad_alloc&) {
        return HZ_ENOMEM;
    }
    if (nsym > 0) {
        hz_ctx* c;
        if ((rc = default_ctx(&c))) return rc;
        HZ_TRY(hipSetDevice(c->device));
        if ((rc = hz_codebook_upload(c, cb.get()))) return rc;
        DevBuf dpay, didx, dout;
        if ((rc = dpay.alloc(pay + 16))) return rc;
        HZ_TRY(hipMemsetAsync(dpay.p, 0, pay + 16, c->stream));
        HZ_TRY(hipMemcpyAsync(dpay.p, f + info.payload_byte, pay, hipMemcpyHostToDevice, c->stream));
        if ((rc = didx.alloc(16))) return rc;
        if ((rc = dout.alloc(2 * nsym + 16))) return rc;
        // index-less decode (no block index); a payload with fewer than nsym codewords (truncated
        // or corrupt file) ends past the payload: rejected
        if ((rc = hz_decode_indexless(c, (const uint8_t*)dpay.p, pay, info.payload_bit, nsym, (uint8_t*)dout.p,
                                      (uint64_t*)didx.p)))
            return rc;
        uint64_t end_bit = 0;
        HZ_TRY(hipMemcpyAsync(&end_bit, didx.p, 8, hipMemcpyDeviceToHost, c->stream));
        if ((rc = hz_ctx_sync(c))) return rc;
        if (end_bit > pay * 8) return HZ_EFORMAT;
        HZ_TRY(hipMemcpyAsync(out.data(), dout.p, 2 * nsym, hipMemcpyDeviceToHost, c->stream));
        if ((rc = hz_ctx_sync(c))) return rc;
    }
    if (info.is_odd) out[2 * nsym] = (uint8_t)info.last_byte;
    return HZ_OK;
}

bool file_exists(const char* name) {
    struct stat st;
    return stat(name, &st) == 0;
}

// Decompressor.cu:185-219: "DECOMPRESSED_FILE", else "DECOMPRESSED_FILE(k)", k = 1..9.
std::string output_name() {
    std::string base = "DECOMPRESSED_FILE";
    if (!file_exists(base.c_str())) return base;
    std::string name;
    for (int k = 1; k < 10; ++k) {
        name = base + "(" + std::to_string(k) + ")";
        if (!file_exists(name.c_str())) break;
    }
    return name;
}

}  // namespace

// ---- streaming archive: bounded host and device memory ----
// Pass 1 reads the file in chunks and accumulates the histogram on the device;
// pass 2 packs chunk by chunk at the running bit offset. Each chunk's last,
// partial word is carried into the next chunk as its `lead` bits, so the file
// is byte-identical to the whole-buffer encoder's. Double-buffered pinned and
// device buffers keep the host's fread of chunk k + 1 and fwrite of chunk
// k - 1 beside the device's upload and pack of chunk k, and the copy-out of
// chunk k runs on a second stream beside the upload and pack of chunk k + 1.
namespace {

struct PinnedBuf {
    uint8_t* p = nullptr;
    ~PinnedBuf() { if (p) (void)hipHostFree(p); }
    int alloc(size_t n) { return hipHostMalloc(&p, n ? n : 16, hipHostMallocDefault) == hipSuccess ? HZ_OK : HZ_ENOMEM; }
};

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); }

thread_local hz_stream_timing g_timing;  // the calling thread's last streamed call

// Device busy time per stage: an event pair around each copy or kernel
// launch (events are never shared between spans), folded into its stage once
// the end event has completed.
class Spans {
  public:
    ~Spans() {
        for (auto& s : open_) {
            (void)hipEventDestroy(s.a);
            (void)hipEventDestroy(s.b);
        }
        for (auto e : free_) (void)hipEventDestroy(e);
    }
    hipEvent_t mark(hipStream_t st) {
        hipEvent_t e = nullptr;
        if (!free_.empty()) {
            e = free_.back();
            free_.pop_back();
        } else if (hipEventCreate(&e) != hipSuccess) {
            return nullptr;
        }
        if (hipEventRecord(e, st) != hipSuccess) {
            free_.push_back(e);
            return nullptr;
        }
        return e;
    }
    void add(hipEvent_t a, hipEvent_t b, double* acc) {
        if (a && b) open_.push_back({a, b, acc});
        else {
            if (a) free_.push_back(a);
            if (b) free_.push_back(b);
        }
    }
    void fold() {
        for (size_t i = 0; i < open_.size();) {
            if (hipEventQuery(open_[i].b) != hipSuccess) { ++i; continue; }
            float ms = 0;
            if (hipEventElapsedTime(&ms, open_[i].a, open_[i].b) == hipSuccess) *open_[i].acc += ms;
            free_.push_back(open_[i].a);
            free_.push_back(open_[i].b);
            open_[i] = open_.back();
            open_.pop_back();
        }
    }
  private:
    struct Span { hipEvent_t a, b; double* acc; };
    std::vector<Span> open_;
    std::vector<hipEvent_t> free_;
};

// Reads of 16 MiB and more go through 8 threads' positional reads (from the
// stream's logical position, which is then moved past them): a single fread
// copies out of the page cache at ~15 GB/s on the MI355X host.
int read_exact(FILE* fp, uint8_t* p, uint64_t n) {
    if (n == 0) return HZ_OK;
    const auto t0 = Clock::now();
    bool ok;
    if (n < (16u << 20)) {
        ok = fread(p, 1, n, fp) == n;
    } else {
        const off_t pos = ftello(fp);
        const int fd = fileno(fp);
        constexpr uint64_t kReaders = 8;
        const uint64_t piece = ((n + kReaders - 1) / kReaders + 4095) & ~(uint64_t)4095;
        std::atomic<bool> bad{pos < 0};
        std::vector<std::thread> th;
        // joins every started reader on every exit, a failed thread spawn (std::system_error,
        // turned into an HZ_ status by guarded()) included
        struct Joiner {
            std::vector<std::thread>& v;
            ~Joiner() { for (auto& t : v) if (t.joinable()) t.join(); }
        } joiner{th};
        for (uint64_t a = 0; a < n && !bad; a += piece) {
            const uint64_t len = std::min(piece, n - a);
            th.emplace_back([&bad, fd, p, a, len, pos] {
                uint64_t done = 0;
                while (done < len) {
                    const ssize_t r = ::pread(fd, p + a + done, len - done, (off_t)(pos + a + done));
                    if (r <= 0) { bad = true; return; }
                    done += (uint64_t)r;
                }
            });
        }
        for (auto& t : th) t.join();
        th.clear();
        ok = !bad && fseeko(fp, pos + (off_t)n, SEEK_SET) == 0;
    }
    g_timing.fread_ms += ms_since(t0);
    g_timing.bytes_in += ok ? n : 0;
    return ok ? HZ_OK : HZ_EIO;
}

// Output file written by background positional writes, so a chunk's write
// overlaps the next chunk's device work. The file's final size is reserved
// first (posix_fallocate): into page cache, 8 threads then write ~12 GB/s on
// the MI355X host, against ~5 GB/s for one or 8 threads into a file that grows
// (block allocation under the inode lock), 6.8 GB/s with O_DIRECT and 1.7 GB/s
// copying into a shared mmap (tools/debug/write_bw.py, 8 GiB). start() hands a
// buffer to kWriters threads (one slice each) and returns; wait() joins them.
// One write is in flight at a time, so the caller double-buffers.
class FileWriter {
  public:
    ~FileWriter() {
        (void)wait();
        if (fd_ >= 0) ::close(fd_);
    }
    int open(const char* path) {
        fd_ = ::open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
        return fd_ >= 0 ? HZ_OK : HZ_EIO;
    }
    // Reserve the file's final size (best effort: a file system without
    // fallocate only loses the speed-up).
    void reserve(uint64_t size) {
        if (fd_ >= 0 && size > 0) reserved_ = ::posix_fallocate(fd_, 0, (off_t)size) == 0;
    }
    void start(const uint8_t* p, uint64_t n, uint64_t off) {
        if (n == 0) return;
        t0_ = Clock::now();
        end_ = std::max(end_, off + n);
        const uint64_t nt = n < (8u << 20) ? 1 : kWriters;
        const uint64_t piece = ((n + nt - 1) / nt + 4095) & ~(uint64_t)4095;
        for (uint64_t a = 0; a < n; a += piece) {
            const uint64_t len = std::min(piece, n - a);
            th_.emplace_back([this, p, a, len, off] {
                uint64_t done = 0;
                while (done < len) {
                    const ssize_t w = ::pwrite(fd_, p + a + done, len - done, (off_t)(off + a + done));
                    if (w <= 0) { err_ = true; return; }
                    done += (uint64_t)w;
                }
            });
        }
        g_timing.bytes_out += n;
    }
    int wait() {
        if (th_.empty()) return err_ ? HZ_EIO : HZ_OK;
        for (auto& t : th_) t.join();
        th_.clear();
        g_timing.fwrite_ms += ms_since(t0_);
        return err_ ? HZ_EIO : HZ_OK;
    }
    int write_now(const uint8_t* p, uint64_t n, uint64_t off) {
        int rc = wait();
        if (rc) return rc;
        start(p, n, off);
        return wait();
    }
    int close() {
        int rc = wait();
        // the file ends at its last written byte, whatever reserve() allocated
        if (fd_ >= 0 && reserved_ && ::ftruncate(fd_, (off_t)end_) != 0) rc = HZ_EIO;
        if (fd_ >= 0 && ::close(fd_) != 0) rc = HZ_EIO;
        fd_ = -1;
        return rc;
    }
  private:
    static constexpr uint64_t kWriters = 8;
    int fd_ = -1;
    bool reserved_ = false;
    uint64_t end_ = 0;
    std::vector<std::thread> th_;
    std::atomic<bool> err_{false};
    Clock::time_point t0_;
};

// Declared after the host buffers a FileWriter reads: an early return waits
// for the writes in flight before those buffers are freed.
struct WriterDrain {
    FileWriter& w;
    ~WriterDrain() { (void)w.wait(); }
};

struct StreamGuard {
    hipStream_t s = nullptr;
    ~StreamGuard() {
        if (s) {
            (void)hipStreamSynchronize(s);  // no copy may outlive the buffers it targets
            (void)hipStreamDestroy(s);
        }
    }
};

// Declared after a function's pinned and device buffers, so it runs before
// they are freed: an early return (I/O error) waits for the copies in flight.
struct DrainGuard {
    hipStream_t s;
    explicit DrainGuard(hipStream_t st) : s(st) {}
    ~DrainGuard() { (void)hipStreamSynchronize(s); }
};

struct EventPair {
    hipEvent_t e[2] = {nullptr, nullptr};
    ~EventPair() {
        for (auto x : e)
            if (x) (void)hipEventDestroy(x);
    }
    int create(bool timing = false) {
        for (auto& x : e)
            if (hipEventCreateWithFlags(&x, timing ? hipEventDefault : hipEventDisableTiming) != hipSuccess) return HZ_EHIP;
        return HZ_OK;
    }
};

}  // namespace

extern "C" int hz_stream_last_timing(hz_stream_timing* t) {
    if (!t) return HZ_EINVAL;
    *t = g_timing;
    return HZ_OK;
}

// resident: keep the input on the device after pass 1 when the file fits
// (hz_archive_file; Compressor.cu:324-367 reads the file once into pinned
// memory), so pass 2 packs it in one launch without reading the file again.
static int hz_archive_stream_impl(const char* in_path, const char* out_path, uint64_t chunk_bytes, int verbose,
                                  bool resident) {
    if (!in_path || !out_path || chunk_bytes < 64) return HZ_EINVAL;
    chunk_bytes &= ~(uint64_t)15;  // even (whole symbols) and 16-byte aligned device reads
    struct stat st;
    if (stat(in_path, &st) != 0) return HZ_ENOENT;
    const uint64_t n = (uint64_t)st.st_size;
    hz_ctx* c;
    const auto tc = Clock::now();
    int rc = default_ctx(&c);
    g_timing.alloc_ms += ms_since(tc);
    if (rc) return rc;
    HZ_TRY(hipSetDevice(c->device));
    Spans spans;
    const uint64_t chunk = std::min<uint64_t>(chunk_bytes, std::max<uint64_t>(n, 16));
    PinnedBuf hin[2];
    DevBuf din[2], dhist, dall;
    const auto ta = Clock::now();
    if (resident && n > chunk) {
        // the whole input plus a payload of the same size must fit in free device memory
        size_t fr = 0, tot = 0;
        resident = hipMemGetInfo(&fr, &tot) == hipSuccess && 2 * n + (1ull << 30) <= fr && dall.alloc(n + 16) == HZ_OK;
    } else {
        resident = false;
    }
    for (int i = 0; i < 2; ++i) {
        if ((rc = hin[i].alloc(chunk))) return rc;
        if (!resident && (rc = din[i].alloc(chunk + 16))) return rc;
    }
    if ((rc = dhist.alloc(HZ_NSYM * 8))) return rc;
    g_timing.alloc_ms += ms_since(ta);
    DrainGuard drain_in(c->stream);
    uint8_t last_byte = 0;
    FILE* fp = fopen(in_path, "rb");
    if (!fp) return HZ_EIO;
    std::unique_ptr<FILE, int (*)(FILE*)> fin(fp, fclose);
    // ---- pass 1: histogram (resident: the chunks stay in dall)
    const auto t_hist = Clock::now();  // "Histograming took" (Compressor.cu:395-399): read + upload + histogram
    HZ_TRY(hipMemsetAsync(dhist.p, 0, HZ_NSYM * 8, c->stream));
    EventPair done;
    if ((rc = done.create())) return rc;
    for (uint64_t off = 0, k = 0; off < n; off += chunk, ++k) {
        const uint64_t len = std::min(chunk, n - off);
        const int b = (int)(k & 1);
        if (k >= 2) HZ_TRY(hipEventSynchronize(done.e[b]));  // buffer b's previous chunk is consumed
        spans.fold();
        if ((rc = read_exact(fp, hin[b].p, len))) return rc;
        if (off + len == n && (n & 1)) last_byte = hin[b].p[len - 1];
        uint8_t* dst = resident ? (uint8_t*)dall.p + off : (uint8_t*)din[b].p;
        hipEvent_t t0 = spans.mark(c->stream);
        HZ_TRY(hipMemcpyAsync(dst, hin[b].p, len, hipMemcpyHostToDevice, c->stream));
        spans.add(t0, spans.mark(c->stream), &g_timing.h2d_ms);
        hipEvent_t t1 = spans.mark(c->stream);
        if ((rc = hz_hist16(c, dst, len, (uint64_t*)dhist.p, 1))) return rc;
        spans.add(t1, spans.mark(c->stream), &g_timing.kernel_ms);
        HZ_TRY(hipEventRecord(done.e[b], c->stream));
    }
    // the codebook is built on the device from the device histogram (k_cb_*, 0.26 ms for
    // U = 65 536 against 0.43 ms on the host plus the histogram's D2H; profiles/r03_codebook_*);
    // HZ_HOST_CODEBOOK=1 builds it on the host instead. Both are bit-exact with GenerateCL.
    static const bool host_cb = [] { const char* v = getenv("HZ_HOST_CODEBOOK"); return v && v[0] == '1'; }();
    // and so is the header (k_hw_*, 0.014 ms against 0.25 ms on the host)
    std::vector<uint64_t> hist(HZ_NSYM);
    std::unique_ptr<hz_codebook> cb(new hz_codebook());
    constexpr uint64_t kHeadCap = 16 + 65536ull * 11;  // the longest header
    std::vector<uint8_t> head;
    uint64_t dinfo_h[4] = {0, 0, 0, 0};
    DevBuf dcb, dhead, dinfo;
    EventPair cbt;  // "construction time" (gpuHuffmanConstruction.h:776-782): the device codebook
    if ((rc = cbt.create(true))) return rc;
    if (!host_cb) {
        if ((rc = dcb.alloc(sizeof(hz_codebook))) || (rc = dhead.alloc(kHeadCap)) || (rc = dinfo.alloc(4 * 8))) return rc;
        head.resize(kHeadCap);
        hipEvent_t t0 = spans.mark(c->stream);
        HZ_TRY(hipEventRecord(cbt.e[0], c->stream));
        if ((rc = hz_codebook_build_device(c, (const uint64_t*)dhist.p, (hz_codebook*)dcb.p))) return rc;
        HZ_TRY(hipEventRecord(cbt.e[1], c->stream));
        if ((rc = hz_header_write_device(c, (const hz_codebook*)dcb.p, n, last_byte, (uint8_t*)dhead.p, kHeadCap,
                                         (uint64_t*)dinfo.p)))
            return rc;
        spans.add(t0, spans.mark(c->stream), &g_timing.kernel_ms);
    }
    {
        hipEvent_t t0 = spans.mark(c->stream);
        HZ_TRY(hipMemcpyAsync(hist.data(), dhist.p, HZ_NSYM * 8, hipMemcpyDeviceToHost, c->stream));
        if (!host_cb) {
            HZ_TRY(hipMemcpyAsync(cb.get(), dcb.p, sizeof(hz_codebook), hipMemcpyDeviceToHost, c->stream));
            HZ_TRY(hipMemcpyAsync(dinfo_h, dinfo.p, sizeof(dinfo_h), hipMemcpyDeviceToHost, c->stream));
            HZ_TRY(hipMemcpyAsync(head.data(), dhead.p, kHeadCap, hipMemcpyDeviceToHost, c->stream));
        }
        spans.add(t0, spans.mark(c->stream), &g_timing.d2h_ms);
    }
    if ((rc = hz_ctx_sync(c))) return rc;
    const double hist_ms = ms_since(t_hist);
    const auto th = Clock::now();
    if (host_cb && (rc = hz_codebook_build(hist.data(), cb.get()))) return rc;
    float cb_ms = 0.0f;
    if (host_cb) cb_ms = (float)ms_since(th);
    else HZ_TRY(hipEventElapsedTime(&cb_ms, cbt.e[0], cbt.e[1]));
    uint64_t hbits = 0, pbits = 0;
    hz_header_bits(cb.get(), n, &hbits);
    hz_payload_bits(cb.get(), hist.data(), &pbits);
    if (verbose) {  // the reference's stdout lines, its stage timers included
        std::cout << "The size of the sum of ORIGINAL files is: " << n << " bytes" << std::endl;
        std::cout << "Unique symbols count: " << cb->nsym << std::endl;
        std::cout << "Histograming took " << hist_ms << " ms" << std::endl;
        printf("construction time: %.3f ms, symbols/s: %.3f\n", cb_ms,
               cb_ms > 0 ? (float)cb->nsym / (cb_ms * 1e-3f) : 0.0f);
        fflush(stdout);
    }
    const auto t_enc = Clock::now();  // "Encoding took" (Compressor.cu:588-593): header, pack, payload out
    // ---- header
    uint64_t hb;
    uint32_t pend_bits;
    uint8_t pend;
    if (host_cb) {
        head.resize(hbits / 8 + 8);
        if ((rc = hz_header_write(cb.get(), n, last_byte, head.data(), head.size(), &hb, &pend_bits, &pend))) return rc;
    } else {
        hb = dinfo_h[0];
        pend_bits = (uint32_t)dinfo_h[1];
        pend = (uint8_t)dinfo_h[2];
        if (dinfo_h[3] != hbits) return HZ_EFORMAT;  // the device writer disagrees with the header length
    }
    g_timing.host_ms += ms_since(th);
    FileWriter fout;
    if ((rc = fout.open(out_path))) return rc;
    fout.reserve(hb + (pend_bits + pbits + 7) / 8);
    if ((rc = fout.write_now(head.data(), hb, 0))) return rc;
    uint64_t written = hb;
    const uint64_t nsym_total = n / 2;
    const uint64_t body = 2 * nsym_total;  // the odd last byte travels in the header
    uint32_t lead = pend_bits ? (uint32_t)(pend >> (8 - pend_bits)) : 0u;
    DevBuf dpay;
    if (resident && nsym_total) {
        const uint64_t pay_bytes = (pend_bits + pbits + 7) / 8;
        const uint64_t cap = ((pend_bits + pbits + 31) / 32 + 1) * 4;
        const auto tb = Clock::now();
        resident = dpay.alloc(cap) == HZ_OK;
        g_timing.alloc_ms += ms_since(tb);
        if (resident) {
            // ---- pass 2, resident: one pack launch over the whole input, then the payload
            // leaves in chunks (copy-out double-buffered against the parallel file writes)
            const auto tu = Clock::now();
            if ((rc = hz_codebook_upload_encode(c, cb.get()))) return rc;
            g_timing.host_ms += ms_since(tu);
            hipEvent_t t1 = spans.mark(c->stream);
            if ((rc = hz_pack(c, (const uint8_t*)dall.p, body, pend_bits, lead, (uint8_t*)dpay.p, cap, nullptr)))
                return rc;
            spans.add(t1, spans.mark(c->stream), &g_timing.kernel_ms);
            for (uint64_t off = 0, k = 0; off < pay_bytes; off += chunk, ++k) {
                const int b = (int)(k & 1);
                const uint64_t len = std::min(chunk, pay_bytes - off);
                hipEvent_t t2 = spans.mark(c->stream);
                HZ_TRY(hipMemcpyAsync(hin[b].p, (const uint8_t*)dpay.p + off, len, hipMemcpyDeviceToHost, c->stream));
                spans.add(t2, spans.mark(c->stream), &g_timing.d2h_ms);
                HZ_TRY(hipEventRecord(done.e[b], c->stream));
                HZ_TRY(hipEventSynchronize(done.e[b]));
                if ((rc = hz_ctx_sync(c))) return rc;
                spans.fold();
                if ((rc = fout.wait())) return rc;  // the write of chunk k - 1 (buffer 1 - b)
                fout.start(hin[b].p, len, written);
                written += len;
            }
        } else {  // no room for the payload beside the input: stream pass 2 from the file
            (void)hipFree(dall.p);
            dall.p = nullptr;
        }
    }
    if (nsym_total == 0) {
        if (pend_bits && (rc = fout.write_now(&pend, 1, written))) return rc;
        written += pend_bits ? 1 : 0;
    } else if (!resident) {
        // ---- pass 2: pack chunk by chunk at the running bit offset
        const auto tu = Clock::now();
        if ((rc = hz_codebook_upload_encode(c, cb.get()))) return rc;
        g_timing.host_ms += ms_since(tu);
        const uint64_t csym = chunk / 2;
        const uint64_t out_cap = ((32 + csym * (uint64_t)cb->max_len + 31) / 32 + 1) * 4;
        DevBuf dout[2], didx;
        PinnedBuf hout[2];
        const auto tb = Clock::now();
        for (int i = 0; i < 2; ++i) {
            if (!din[i].p && (rc = din[i].alloc(chunk + 16))) return rc;
            if ((rc = dout[i].alloc(out_cap))) return rc;
            if ((rc = hout[i].alloc(out_cap))) return rc;
        }
        if ((rc = didx.alloc(hz_index_bytes(csym)))) return rc;
        g_timing.alloc_ms += ms_since(tb);
        WriterDrain wdrain{fout};
        DrainGuard drain_out(c->stream);
        StreamGuard cs;  // copy-out stream
        HZ_TRY(hipStreamCreateWithFlags(&cs.s, hipStreamNonBlocking));
        EventPair packed, copied;
        if ((rc = packed.create()) || (rc = copied.create())) return rc;
        if (fseek(fp, 0, SEEK_SET) != 0) return HZ_EIO;
        uint32_t sbit = pend_bits;                       // bit of the chunk's first code in its first word
        if ((rc = read_exact(fp, hin[0].p, std::min(chunk, body)))) return rc;
        int wbuf = -1;          // chunk waiting for its write: buffer, bytes
        uint64_t wbytes = 0;
        for (uint64_t off = 0, k = 0; off < body; off += chunk, ++k) {
            const int b = (int)(k & 1);
            const uint64_t len = std::min(chunk, body - off);
            hipEvent_t t0 = spans.mark(c->stream);
            HZ_TRY(hipMemcpyAsync(din[b].p, hin[b].p, len, hipMemcpyHostToDevice, c->stream));
            spans.add(t0, spans.mark(c->stream), &g_timing.h2d_ms);
            if (k >= 2) HZ_TRY(hipStreamWaitEvent(c->stream, copied.e[b], 0));  // dout[b] copied out
            hipEvent_t t1 = spans.mark(c->stream);
            if ((rc = hz_pack(c, (const uint8_t*)din[b].p, len, sbit, lead, (uint8_t*)dout[b].p, out_cap,
                              (uint64_t*)didx.p)))
                return rc;
            spans.add(t1, spans.mark(c->stream), &g_timing.kernel_ms);
            HZ_TRY(hipEventRecord(packed.e[b], c->stream));
            const uint64_t nb = (len / 2 + 2047) / 2048;
            uint64_t end_bit = 0;
            HZ_TRY(hipMemcpyAsync(&end_bit, (const uint64_t*)didx.p + nb, 8, hipMemcpyDeviceToHost, c->stream));
            // host work beside the upload and pack: the previous chunk's write, the next chunk's fread
            if (wbuf >= 0) {
                HZ_TRY(hipEventSynchronize(copied.e[wbuf]));
                if ((rc = fout.wait())) return rc;  // hout[b] (two chunks back) is free again after this
                fout.start(hout[wbuf].p, wbytes, written);
                written += wbytes;
                wbuf = -1;
            }
            const uint64_t next = off + len;
            if (next < body && (rc = read_exact(fp, hin[1 - b].p, std::min(chunk, body - next)))) return rc;
            if ((rc = hz_ctx_sync(c))) return rc;
            spans.fold();
            const bool last = next >= body;
            const uint64_t bytes = last ? (end_bit + 7) / 8 : end_bit / 32 * 4;  // complete words until the end
            sbit = (uint32_t)(end_bit % 32);
            lead = 0;
            if (sbit && !last) {  // the partial word, carried into the next chunk as its lead bits
                uint32_t w = 0;
                HZ_TRY(hipMemcpyAsync(&w, (const uint8_t*)dout[b].p + bytes, 4, hipMemcpyDeviceToHost, c->stream));
                if ((rc = hz_ctx_sync(c))) return rc;
                lead = __builtin_bswap32(w) >> (32 - sbit);
            }
            if ((rc = fout.wait())) return rc;  // hout[b] may still be leaving from two chunks back
            HZ_TRY(hipStreamWaitEvent(cs.s, packed.e[b], 0));
            hipEvent_t t2 = spans.mark(cs.s);
            if (bytes) HZ_TRY(hipMemcpyAsync(hout[b].p, dout[b].p, bytes, hipMemcpyDeviceToHost, cs.s));
            spans.add(t2, spans.mark(cs.s), &g_timing.d2h_ms);
            HZ_TRY(hipEventRecord(copied.e[b], cs.s));
            wbuf = b;
            wbytes = bytes;
        }
        if (wbuf >= 0) {
            HZ_TRY(hipEventSynchronize(copied.e[wbuf]));
            if ((rc = fout.wait())) return rc;
            fout.start(hout[wbuf].p, wbytes, written);
            written += wbytes;
        }
        if ((rc = fout.wait())) return rc;
        HZ_TRY(hipStreamSynchronize(cs.s));
    }
    if ((rc = fout.close())) return rc;
    spans.fold();
    if (written != (hbits + pbits + 7) / 8) return HZ_EFORMAT;
    if (verbose) {
        std::cout << "Encoding took " << ms_since(t_enc) << " ms" << std::endl;
        std::cout << "The size of the COMPRESSED file is: " << written << " bytes" << std::endl;
        const float ratio = 100.0f * (float)written / (float)(n ? n : 1);
        std::cout << "Compressed file's size is [" << ratio << "%] of the original files." << std::endl;
        if (written > n) std::cout << "\nWARNING: The compressed file's size is larger than the sum of the originals.\n\n";
        std::cout << std::endl << "Created compressed file: " << out_path << std::endl;
        std::cout << "Compression is complete" << std::endl;
    }
    return HZ_OK;
}

extern "C" int hz_archive_stream(const char* in_path, const char* out_path, uint64_t chunk_bytes, int verbose) {
    g_timing = hz_stream_timing();
    const auto t0 = Clock::now();
    const int rc = guarded([&] { return hz_archive_stream_impl(in_path, out_path, chunk_bytes, verbose, false); });
    g_timing.total_ms = ms_since(t0);
    return rc;
}

// hz_archive_file's archive: the input stays on the device between the passes when it fits.
static int archive_resident(const char* in_path, const char* out_path, uint64_t chunk_bytes, int verbose) {
    g_timing = hz_stream_timing();
    const auto t0 = Clock::now();
    const int rc = guarded([&] { return hz_archive_stream_impl(in_path, out_path, chunk_bytes, verbose, true); });
    g_timing.total_ms = ms_since(t0);
    return rc;
}

// The header of a file to extract: parsed on the device (k_hdr_*, 0.05 ms for
// U = 65 536 against 0.25+ ms on the host; profiles/r03_codebook_*), the codebook
// and the info copied back for the host-built decode tables. HZ_HOST_HEADER=1
// parses on the host. Both follow Decompressor.cu:65-103 and reject the same files.
static int parse_header_for_extract(const std::vector<uint8_t>& head, hz_codebook* cb, hz_header_info* info) {
    static const bool host_hdr = [] { const char* v = getenv("HZ_HOST_HEADER"); return v && v[0] == '1'; }();
    const auto th = Clock::now();
    int rc;
    if (host_hdr || head.size() < 12) {  // a header-only file: no device work at all
        rc = hz_header_parse(head.data(), head.size(), cb, info);
        g_timing.host_ms += ms_since(th);
        return rc;
    }
    hz_ctx* c;
    if ((rc = default_ctx(&c))) return rc;
    HZ_TRY(hipSetDevice(c->device));
    DevBuf dhead, dcb, dinfo;
    if ((rc = dhead.alloc(head.size())) || (rc = dcb.alloc(sizeof(hz_codebook))) || (rc = dinfo.alloc(6 * 8))) return rc;
    g_timing.alloc_ms += ms_since(th);  // context and buffers: allocation, as on the host path
    const auto tp = Clock::now();
    uint64_t hi[6];
    HZ_TRY(hipMemcpyAsync(dhead.p, head.data(), head.size(), hipMemcpyHostToDevice, c->stream));
    if ((rc = hz_header_parse_device(c, (const uint8_t*)dhead.p, head.size(), (hz_codebook*)dcb.p, (uint64_t*)dinfo.p)))
        return rc;
    HZ_TRY(hipMemcpyAsync(cb, dcb.p, sizeof(hz_codebook), hipMemcpyDeviceToHost, c->stream));
    HZ_TRY(hipMemcpyAsync(hi, dinfo.p, sizeof(hi), hipMemcpyDeviceToHost, c->stream));
    if ((rc = hz_ctx_sync(c))) return rc;  // HZ_EFORMAT for a malformed header
    info->n = hi[0];
    info->payload_byte = hi[1];
    info->payload_bit = (uint32_t)hi[2];
    info->is_odd = (uint32_t)hi[3];
    info->last_byte = (uint32_t)hi[4];
    info->nsym = (uint32_t)hi[5];
    g_timing.host_ms += ms_since(tp);
    return HZ_OK;
}

// Streaming extract: the payload passes through a device window of chunk_bytes.
// Each round decodes as many symbols as the window surely holds (the file's
// mean code length with a margin; a round whose codes overrun the window is
// redone at the max_len bound), and moves the unconsumed tail of the window to
// the front of the other buffer before refilling it. The host's fread of the
// next window overlaps the decode, and its fwrite of a round's output overlaps
// the next round's upload and index-less decode (hz_decode_indexless).
static int hz_extract_stream_impl(const char* in_path, const char* out_path, uint64_t chunk_bytes, int verbose) {
    if (!in_path || !out_path || chunk_bytes < 4096) return HZ_EINVAL;
    chunk_bytes &= ~(uint64_t)15;
    struct stat st;
    if (stat(in_path, &st) != 0) return HZ_ENOENT;
    const uint64_t fsize = (uint64_t)st.st_size;
    FILE* fp = fopen(in_path, "rb");
    if (!fp) return HZ_EIO;
    std::unique_ptr<FILE, int (*)(FILE*)> fin(fp, fclose);
    // the header is at most 12 + 65536 * (3 + 8) bytes
    std::vector<uint8_t> head(std::min<uint64_t>(fsize, 1u << 20));
    int rc = read_exact(fp, head.data(), head.size());
    if (rc) return rc;
    std::unique_ptr<hz_codebook> cb(new hz_codebook());
    hz_header_info info;
    if ((rc = parse_header_for_extract(head, cb.get(), &info))) return rc;
    FileWriter fout;
    if ((rc = fout.open(out_path))) return rc;
    {
        // Reserve no more than the payload can decode to: a header whose N overstates it (corrupt or
        // crafted) must not allocate disk before the decode rejects it. nsym codewords need at least
        // nsym * min_len payload bits.
        const uint64_t pay_bits = fsize > info.payload_byte ? (fsize - info.payload_byte) * 8 - info.payload_bit : 0;
        const uint64_t min_len = std::max<uint32_t>(cb->min_len, 1);
        const uint64_t most = 2 * (pay_bits / min_len) + (info.is_odd ? 1 : 0);
        fout.reserve(std::min<uint64_t>(info.n, most));
    }
    uint64_t out_off = 0;
    const uint64_t nsym = info.n / 2;
    if (nsym > 0) {
        hz_ctx* c;
        const auto tc = Clock::now();
        rc = default_ctx(&c);
        g_timing.alloc_ms += ms_since(tc);
        if (rc) return rc;
        HZ_TRY(hipSetDevice(c->device));
        Spans spans;
        const auto tu = Clock::now();
        if ((rc = hz_codebook_upload_decode(c, cb.get()))) return rc;
        g_timing.host_ms += ms_since(tu);
        const uint64_t W = chunk_bytes;               // window bytes
        const uint64_t pay_total = fsize > info.payload_byte ? fsize - info.payload_byte : 0;
        const uint64_t max_len = std::max<uint32_t>(cb->max_len, 1);
        // mean bits per symbol of this file, 3% margin (a mispredicted round is redone exactly)
        const double mean = pay_total ? ((double)pay_total * 8 - info.payload_bit) / (double)nsym : (double)max_len;
        const uint64_t sym_cap = std::max<uint64_t>(W / 2, kBlockSyms);  // output per round <= W bytes
        DevBuf dwin[2], didx, dout;
        PinnedBuf hin, hout[2];  // hout: a round's output leaves (parallel writes) beside the next round
        int ob = 0;
        const auto ta = Clock::now();
        for (int i = 0; i < 2; ++i)
            if ((rc = dwin[i].alloc(W + 16))) return rc;
        if ((rc = didx.alloc(16))) return rc;  // the round's end bit
        if ((rc = dout.alloc(2 * sym_cap + 16))) return rc;
        if ((rc = hin.alloc(W))) return rc;
        for (int i = 0; i < 2; ++i)
            if ((rc = hout[i].alloc(2 * sym_cap))) return rc;
        WriterDrain wdrain{fout};
        g_timing.alloc_ms += ms_since(ta);
        DrainGuard drain(c->stream);
        if (fseek(fp, (long)info.payload_byte, SEEK_SET) != 0) return HZ_EIO;
        uint64_t file_left = pay_total, have = 0, done = 0;
        uint64_t bit = info.payload_bit;
        int cur = 0;
        // symbols this round decodes from the window: what it surely holds
        auto round_syms = [&]() {
            const uint64_t left = nsym - done, avail = have * 8 - bit;
            if (file_left == 0) return std::min(left, sym_cap);
            uint64_t k = (uint64_t)((double)avail / (mean * 1.03));
            k = std::min(std::min(left, sym_cap), k);
            // whole blocks when the window holds at least one; a smaller window keeps k
            if (k < left && k >= (uint64_t)kBlockSyms) k = k / kBlockSyms * kBlockSyms;
            return std::max<uint64_t>(k, 1);
        };
        uint64_t end_bit = 0;
        // a round: the window's first kk codewords decoded index-less into dout, and their end bit
        auto launch_index = [&](uint64_t kk) -> int {
            hipEvent_t t0 = spans.mark(c->stream);
            int r2 = hz_decode_indexless(c, (const uint8_t*)dwin[cur].p, have, bit, kk, (uint8_t*)dout.p,
                                         (uint64_t*)didx.p);
            if (r2) return r2;
            spans.add(t0, spans.mark(c->stream), &g_timing.kernel_ms);
            HZ_TRY(hipMemcpyAsync(&end_bit, didx.p, 8, hipMemcpyDeviceToHost, c->stream));
            return HZ_OK;
        };
        // first fill
        uint64_t r = std::min(W, file_left);
        if ((rc = read_exact(fp, hin.p, r))) return rc;
        HZ_TRY(hipMemsetAsync(dwin[cur].p, 0, W + 16, c->stream));
        {
            hipEvent_t t0 = spans.mark(c->stream);
            HZ_TRY(hipMemcpyAsync(dwin[cur].p, hin.p, r, hipMemcpyHostToDevice, c->stream));
            spans.add(t0, spans.mark(c->stream), &g_timing.h2d_ms);
        }
        have = r;
        file_left -= r;
        uint64_t k = round_syms();
        if ((rc = launch_index(k))) return rc;
        while (done < nsym) {
            if ((rc = hz_ctx_sync(c))) return rc;
            if (end_bit > have * 8 && file_left > 0) {  // the round's codes overran the window: redo at the bound
                k = std::max<uint64_t>((have * 8 - bit) / max_len, 1);
                if ((rc = launch_index(k)) || (rc = hz_ctx_sync(c))) return rc;
            }
            if (end_bit > have * 8) return HZ_EFORMAT;    // truncated file
            hipEvent_t t1 = spans.mark(c->stream);
            HZ_TRY(hipMemcpyAsync(hout[ob].p, dout.p, 2 * k, hipMemcpyDeviceToHost, c->stream));
            spans.add(t1, spans.mark(c->stream), &g_timing.d2h_ms);
            // move the unconsumed tail to the other window and read the refill behind the decode
            const uint64_t used = end_bit / 8, tail = have - used;
            const int nxt = cur ^ 1;
            const bool more = done + k < nsym;
            r = 0;
            if (more) {
                if (tail) HZ_TRY(hipMemcpyAsync(dwin[nxt].p, (const uint8_t*)dwin[cur].p + used, tail,
                                                hipMemcpyDeviceToDevice, c->stream));
                r = std::min(W - tail, file_left);
                if ((rc = read_exact(fp, hin.p, r))) return rc;
            }
            if ((rc = hz_ctx_sync(c))) return rc;    // decode, output copy and tail move done
            spans.fold();
            const uint64_t kdone = k;
            if (more) {  // next window and its index build, beside this round's fwrite
                if (r < W - tail) HZ_TRY(hipMemsetAsync((uint8_t*)dwin[nxt].p + tail + r, 0, W + 16 - tail - r, c->stream));
                if (r) {
                    hipEvent_t t2 = spans.mark(c->stream);
                    HZ_TRY(hipMemcpyAsync((uint8_t*)dwin[nxt].p + tail, hin.p, r, hipMemcpyHostToDevice, c->stream));
                    spans.add(t2, spans.mark(c->stream), &g_timing.h2d_ms);
                }
                have = tail + r;
                file_left -= r;
                bit = end_bit % 8;
                cur = nxt;
                done += kdone;
                k = round_syms();
                if ((rc = launch_index(k))) return rc;
            } else {
                done += kdone;
            }
            if ((rc = fout.wait())) return rc;  // the previous round's write: hout[ob ^ 1] free for the next
            fout.start(hout[ob].p, 2 * kdone, out_off);
            out_off += 2 * kdone;
            ob ^= 1;
        }
        if ((rc = fout.wait())) return rc;
        spans.fold();
    }
    if (info.is_odd) {
        const uint8_t b = (uint8_t)info.last_byte;
        if ((rc = fout.write_now(&b, 1, out_off))) return rc;
    }
    if ((rc = fout.close())) return rc;
    if (verbose) std::cout << "Decompression is complete" << std::endl;
    return HZ_OK;
}

extern "C" int hz_extract_stream(const char* in_path, const char* out_path, uint64_t chunk_bytes, int verbose) {
    g_timing = hz_stream_timing();
    const auto t0 = Clock::now();
    const int rc = guarded([&] { return hz_extract_stream_impl(in_path, out_path, chunk_bytes, verbose); });
    g_timing.total_ms = ms_since(t0);
    return rc;
}

static int hz_encode_host_impl(const uint8_t* in, uint64_t n, uint8_t* out, uint64_t cap, uint64_t* out_len) {
    if ((!in && n) || !out_len) return HZ_EINVAL;
    std::vector<uint8_t> img;
    int rc = encode_image(in, n, img, nullptr);
    if (rc) return rc;
    *out_len = img.size();
    if (!out || cap < img.size()) return HZ_ECAP;
    memcpy(out, img.data(), img.size());
    return HZ_OK;
}

extern "C" int hz_encode_host(const uint8_t* in, uint64_t n, uint8_t* out, uint64_t cap, uint64_t* out_len) {
    return guarded([&] { return hz_encode_host_impl(in, n, out, cap, out_len); });
}

static int hz_encoded_size_impl(const uint8_t* in, uint64_t n, uint64_t* out_len) {
    if ((!in && n) || !out_len) return HZ_EINVAL;
    hz_ctx* c;
    int rc = default_ctx(&c);
    if (rc) return rc;
    HZ_TRY(hipSetDevice(c->device));
    DevBuf din;
    if ((rc = din.alloc(n))) return rc;
    if (n) HZ_TRY(hipMemcpyAsync(din.p, in, n, hipMemcpyHostToDevice, c->stream));
    EncodePlan p;
    if ((rc = plan_encode(c, (const uint8_t*)din.p, n, p))) return rc;
    *out_len = (p.header_bits + p.payload_bits + 7) / 8;
    return HZ_OK;
}

extern "C" int hz_encoded_size(const uint8_t* in, uint64_t n, uint64_t* out_len) {
    return guarded([&] { return hz_encoded_size_impl(in, n, out_len); });
}

static int hz_decode_host_impl(const uint8_t* file, uint64_t len, uint8_t* out, uint64_t cap, uint64_t* out_n) {
    if (!file || !out_n) return HZ_EINVAL;
    std::vector<uint8_t> dec;
    int rc = decode_image(file, len, dec);
    if (rc) return rc;
    *out_n = dec.size();
    if (cap < dec.size() || (!out && dec.size())) return HZ_ECAP;
    if (dec.size()) memcpy(out, dec.data(), dec.size());
    return HZ_OK;
}

extern "C" int hz_decode_host(const uint8_t* file, uint64_t len, uint8_t* out, uint64_t cap, uint64_t* out_n) {
    return guarded([&] { return hz_decode_host_impl(file, len, out, cap, out_n); });
}

// Compressor.cu:315-632, stdout lines kept (:335-336,385,612-631).
extern "C" int hz_archive_file(const char* path, int verbose) {
    if (!path) return HZ_EINVAL;
    struct stat st;
    if (stat(path, &st) != 0) {
        if (verbose) std::cout << path << " file does not exist" << std::endl << "Process has been terminated" << std::endl;
        return HZ_ENOENT;
    }
    const std::string outname = std::string(path) + ".compressed";
    // HZ_ARCHIVE_CHUNK: chunk bytes of the file reads and payload writes (tests use small ones)
    const char* ce = getenv("HZ_ARCHIVE_CHUNK");
    const uint64_t chunk = ce && strtoull(ce, nullptr, 10) >= 64 ? strtoull(ce, nullptr, 10) : kArchiveChunk;
    const int rc = archive_resident(path, outname.c_str(), chunk, verbose);
    if (rc) {
        remove(outname.c_str());  // never leave a truncated archive behind
        if (verbose) std::cerr << "archive: " << hz_strerror(rc) << std::endl;
    }
    return rc;
}

// Decompressor.cu:47-114.
extern "C" int hz_extract_file(const char* path, char* out_name, size_t out_name_cap, int verbose) {
    if (!path) return HZ_EINVAL;
    struct stat st;
    if (stat(path, &st) != 0) {
        if (verbose) std::cout << path << " does not exist" << std::endl;
        return HZ_ENOENT;
    }
    std::string name = output_name();
    // HZ_EXTRACT_WINDOW: payload window bytes (>= 4096)
    const char* we = getenv("HZ_EXTRACT_WINDOW");
    const uint64_t window = we && strtoull(we, nullptr, 10) >= 4096 ? strtoull(we, nullptr, 10) : kExtractWindow;
    int rc = hz_extract_stream(path, name.c_str(), window, 0);
    if (rc) {
        remove(name.c_str());
        if (verbose) std::cerr << "extract: " << hz_strerror(rc) << std::endl;
        return rc;
    }
    if (out_name && out_name_cap) {
        strncpy(out_name, name.c_str(), out_name_cap - 1);
        out_name[out_name_cap - 1] = 0;
    }
    if (verbose) std::cout << "Decompression is complete" << std::endl;
    return HZ_OK;
}
