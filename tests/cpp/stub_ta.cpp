// tests/cpp/stub_ta.cpp -- a CPU stand-in for the part of the C ABI
// (include/team_align_c.h) that the drop-in team::Align shim calls, backed by
// the oracle (oracle/align_oracle.c).  Only for the ThreadSanitizer run of
// the shim (tests/test_host_sanitizers.py): the shim's per-thread contexts
// and buffers are exercised from many threads without a GPU.  Never part of
// the product (which has no CPU path).
#include <atomic>
#include <cstring>
#include <thread>
#include <string>

#include "team_align_c.h"

extern "C" int oracle_align(const char* q, unsigned n, const char* t, unsigned m, int type, int match, int mismatch,
                            int gap, int want_cigar, int* score_out, unsigned* target_begin_out, char* cigar_out,
                            size_t cigar_cap, size_t* cigar_len);

struct ta_context {
    std::string last_error;
    int device = 0;
};

extern "C" {

const char* ta_status_string(int status) {
    switch (status) {
        case TA_OK: return "ok";
        case TA_ERR_BAD_TYPE: return "Unknown AlignmentType provided.";
        case TA_ERR_CIGAR: return "Unknown error in determining cigar string.";
        default: return "error";
    }
}

const char* ta_last_error(const ta_context* ctx) { return ctx ? ctx->last_error.c_str() : ""; }

int ta_context_create(int device, ta_context** out) {
    *out = new ta_context();
    (*out)->device = device;
    return TA_OK;
}

void ta_context_destroy(ta_context* ctx) { delete ctx; }

// the thread's "current device" (stub_set_current_device) and the device of
// the last call served for this thread (stub_last_device): the device-choice
// test of tests/cpp/shim_caller.cpp ("devices")
thread_local int t_stub_current = 0, t_stub_last = -1;
void stub_set_current_device(int d) { t_stub_current = d; }
int stub_last_device() { return t_stub_last; }
int ta_current_device(void) { return t_stub_current; }
int ta_device_count(void) { return 4; }

// The single-pair server: the oracle again, for pairs of even query length
// (the others take the shim's batch path, so both run under TSan).
struct ta_server {
    int type = 0, device = 0;
    std::atomic<int> active{0}, paused{0};  // the pause protocol of ta_server.cpp
};

int ta_server_create(int device, int type, uint32_t slots, ta_server** out) {
    (void)slots;
    *out = new ta_server();
    (*out)->type = type;
    (*out)->device = device;
    return TA_OK;
}

void ta_server_destroy(ta_server* s) { delete s; }

int ta_server_fits(const ta_server* s, uint32_t n, uint32_t m, int match, int mismatch, int gap) {
    (void)s, (void)m, (void)match, (void)mismatch, (void)gap;
    return n % 2 == 0;
}

int ta_server_running(const ta_server* s) { return s != nullptr; }

int ta_server_pause(ta_server* s) {
    s->paused.fetch_add(1);
    while (s->active.load() != 0) std::this_thread::yield();
    return TA_OK;
}

int ta_server_resume(ta_server* s) {
    s->paused.fetch_sub(1);
    return TA_OK;
}

int ta_server_align(ta_server* s, const char* q, uint32_t n, const char* t, uint32_t m, int match, int mismatch,
                    int gap, int want_cigar, int32_t* score, uint32_t* target_begin, char* cigar, uint64_t cigar_cap,
                    uint32_t* cigar_len) {
    s->active.fetch_add(1);
    if (s->paused.load() > 0) {
        s->active.fetch_sub(1);
        return TA_ERR_UNSERVED;
    }
    struct Leave {
        std::atomic<int>& a;
        ~Leave() { a.fetch_sub(1); }
    } leave{s->active};
    t_stub_last = s->device;
    int sc = 0;
    unsigned b = 0;
    size_t cl = 0;
    const int r = oracle_align(q, n, t, m, s->type, match, mismatch, gap, want_cigar, &sc, &b,
                               want_cigar ? cigar : nullptr, want_cigar ? cigar_cap : 0, &cl);
    if (r) return r;
    *score = sc;
    *target_begin = b;
    if (want_cigar) *cigar_len = (uint32_t)cl;
    return TA_OK;
}

uint64_t ta_cigar_slot_bytes(uint32_t n, uint32_t m) { return 2ull * ((uint64_t)n + m) + 2; }

int ta_align_batch(ta_context* ctx, uint32_t n_pairs, const char* qb, const uint64_t* qoff, const uint32_t* qlen,
                   const char* tb, const uint64_t* toff, const uint32_t* tlen, int type, int match, int mismatch,
                   int gap, int want_cigar, int32_t* score, uint32_t* target_begin, char* arena, uint64_t arena_bytes,
                   uint64_t* cigar_off, uint32_t* cigar_len) {
    uint64_t at = 0;
    t_stub_last = ctx->device;  // (the leader's thread: the device-choice test runs one thread)
    for (uint32_t p = 0; p < n_pairs; ++p) {
        int s = 0;
        unsigned b = 0;
        size_t cl = 0;
        const int r = oracle_align(qb + qoff[p], qlen[p], tb + toff[p], tlen[p], type, match, mismatch, gap,
                                   want_cigar, &s, &b, want_cigar ? arena + at : nullptr,
                                   want_cigar ? arena_bytes - at : 0, &cl);
        if (r) {
            ctx->last_error = ta_status_string(r);
            return r;
        }
        if (score) score[p] = s;
        if (target_begin) target_begin[p] = b;
        if (want_cigar) {
            cigar_off[p] = at;
            cigar_len[p] = (uint32_t)cl;
            at += cl;
        }
    }
    return TA_OK;
}

int ta_align_batch_flags(ta_context* ctx, uint32_t n_pairs, const char* qb, const uint64_t* qoff,
                         const uint32_t* qlen, const char* tb, const uint64_t* toff, const uint32_t* tlen, int type,
                         int match, int mismatch, int gap, int want_cigar, int32_t* score, uint32_t* target_begin,
                         char* arena, uint64_t arena_bytes, uint64_t* cigar_off, uint32_t* cigar_len, uint32_t) {
    return ta_align_batch(ctx, n_pairs, qb, qoff, qlen, tb, toff, tlen, type, match, mismatch, gap, want_cigar, score,
                          target_begin, arena, arena_bytes, cigar_off, cigar_len);
}

}  // extern "C"
