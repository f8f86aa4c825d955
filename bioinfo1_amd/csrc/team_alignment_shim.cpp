// bioinfo1_amd/csrc/team_alignment_shim.cpp -- the drop-in team::Align.
//
// Exports the reference's C++ entry point with the identical signature and
// mangled name (include/team_alignment.hpp; reference
// team_alignment.hpp:14-23 / team_alignment.cpp:49-56) so team_mapper.cpp's
// four call sites (team_mapper.cpp:666, 674, 755, 763) link unchanged.  The
// calls are forwarded as batches to the extern "C" ABI, which runs the HIP
// kernels; there is no CPU fallback.  Error behaviour mirrors the reference:
// std::invalid_argument with the same two messages; a missing or failing GPU
// raises std::runtime_error (the mapper's catch (std::exception&) at
// team_mapper.cpp:680-683 handles both).
//
// Concurrent calls are combined: the mapper calls Align once per read from
// OpenMP threads (team_mapper.cpp:596), and one pair cannot fill a GPU.  A
// call queues its pair; if no batch is running, the caller becomes the
// leader: it takes the queued pairs, aligns them as one batch (one upload,
// the kernels, one download) and wakes their callers; otherwise it waits for
// a leader to take its pair.  A lone caller runs its own one-pair
// batch at once (no added wait), and under load a batch holds every pair
// that arrived while the previous one ran.
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/team_align_c.h"
#include "../../include/team_alignment.hpp"

namespace {

// One context (device stream + grow-only device and pinned staging buffers)
// per leader thread; after the first calls a batch allocates nothing: one
// pinned upload, the kernels, one download, one synchronisation
// (ta_host_batch.h).  The host staging vectors are grow-only too.
struct ThreadCtx {
    ta_context* ctx = nullptr;
    std::vector<char> qbytes, tbytes, arena;
    std::vector<uint64_t> qoff, toff, coff;
    std::vector<uint32_t> qlen, tlen, tb, clen;
    std::vector<int32_t> score;
    ~ThreadCtx() { ta_context_destroy(ctx); }
};

thread_local ThreadCtx tc;

ta_context* thread_context() {
    if (!tc.ctx) {
        int r = ta_context_create(0, &tc.ctx);
        if (r != TA_OK) throw std::runtime_error("team::Align: no usable gfx950 GPU (" + std::string(ta_status_string(r)) + ")");
    }
    return tc.ctx;
}

struct Request {
    const char* q;
    uint32_t ql;
    const char* t;
    uint32_t tl;
    int type, match, mismatch, gap;
    std::string* cigar;
    int32_t score = 0;
    uint32_t target_begin = 0;
    int status = TA_OK;
    std::string error;
    bool filled = false;  // results (or the batch's error) recorded
    bool taken = false;   // in a running batch
    bool done = false;
};

// One batch at a time.  A new leader first waits (at most kGather) until as
// many pairs are queued as its predecessor's batch held: the callers that
// batch just released are on their way back with their next pairs, and taking
// the queue at once would alternate one-pair and (T - 1)-pair batches.  A lone
// caller (last batch: one pair) never waits.
constexpr auto kGather = std::chrono::microseconds(50);

std::mutex g_mu;
std::condition_variable g_cv;      // batch done / leader free
std::condition_variable g_arrive;  // a pair was queued
std::vector<Request*> g_queue;
bool g_leading = false;
size_t g_last_batch = 1;

bool same_batch(const Request* a, const Request* b) {
    return a->type == b->type && a->match == b->match && a->mismatch == b->mismatch && a->gap == b->gap &&
           (a->cigar != nullptr) == (b->cigar != nullptr);
}

// Align reqs[0..n) (same type, scores and CIGAR request) as one batch.
void run_batch(Request* const* reqs, size_t n) {
    ThreadCtx& c = tc;
    c.qoff.resize(n), c.toff.resize(n), c.qlen.resize(n), c.tlen.resize(n);
    c.score.resize(n), c.tb.resize(n), c.coff.resize(n), c.clen.resize(n);
    uint64_t qn = 0, tn = 0, slots = 0;
    for (size_t k = 0; k < n; ++k) {
        c.qoff[k] = qn, c.toff[k] = tn;
        c.qlen[k] = reqs[k]->ql, c.tlen[k] = reqs[k]->tl;
        qn += reqs[k]->ql, tn += reqs[k]->tl;
        slots += ta_cigar_slot_bytes(reqs[k]->ql, reqs[k]->tl);
    }
    if (c.qbytes.size() < qn) c.qbytes.resize(qn);
    if (c.tbytes.size() < tn) c.tbytes.resize(tn);
    for (size_t k = 0; k < n; ++k) {
        if (reqs[k]->ql) std::memcpy(c.qbytes.data() + c.qoff[k], reqs[k]->q, reqs[k]->ql);
        if (reqs[k]->tl) std::memcpy(c.tbytes.data() + c.toff[k], reqs[k]->t, reqs[k]->tl);
    }
    const bool want = reqs[0]->cigar != nullptr;
    if (want && c.arena.size() < slots) c.arena.resize(slots);
    int r = TA_OK;
    std::string err;
    try {
        ta_context* ctx = thread_context();
        // (the default plan also for small batches: packed couples and the lane
        // walk beat one int32 wave per pair with its walk inside the fill from 2
        // pairs up, 200x200: 8 pairs 221 vs 267 us, scripts/exp/batch_latency.py)
        r = ta_align_batch(ctx, (uint32_t)n, c.qbytes.data(), c.qoff.data(), c.qlen.data(), c.tbytes.data(),
                           c.toff.data(), c.tlen.data(), reqs[0]->type, reqs[0]->match, reqs[0]->mismatch,
                           reqs[0]->gap, want, c.score.data(), c.tb.data(), c.arena.data(), c.arena.size(),
                           c.coff.data(), c.clen.data());
        if (r != TA_OK) err = ta_last_error(ctx);
    } catch (const std::exception& e) {
        r = TA_ERR_DEVICE;
        err = e.what();
    }
    for (size_t k = 0; k < n; ++k) {
        Request* q = reqs[k];
        q->status = r;
        if (r != TA_OK) {
            q->error = err;
        } else {
            q->score = c.score[k];
            q->target_begin = c.tb[k];
            if (want) q->cigar->assign(c.arena.data() + c.coff[k], c.clen[k]);  // assigned, not appended (:160)
        }
        q->filled = true;
    }
}

// The leader's work: the taken requests grouped by scoring (in arrival order).
void run_taken(std::vector<Request*>& taken) {
    std::vector<Request*> group;
    std::vector<bool> used(taken.size(), false);
    for (size_t i = 0; i < taken.size(); ++i) {
        if (used[i]) continue;
        group.clear();
        for (size_t j = i; j < taken.size(); ++j)
            if (!used[j] && same_batch(taken[i], taken[j])) {
                used[j] = true;
                group.push_back(taken[j]);
            }
        run_batch(group.data(), group.size());
    }
}

}  // namespace

namespace team {

int Align(const char* query, unsigned int query_len, const char* target, unsigned int target_len,
          AlignmentType type, int match, int mismatch, int gap, std::string* cigar, unsigned int* target_begin) {
    const int t = static_cast<int>(type);
    if (t != TA_GLOBAL && t != TA_LOCAL && t != TA_SEMI_GLOBAL)
        throw std::invalid_argument("Unknown AlignmentType provided.");  // team_alignment.cpp:73
    Request req{query, query_len, target, target_len, t, match, mismatch, gap, cigar};
    {
        std::unique_lock<std::mutex> lk(g_mu);
        g_queue.push_back(&req);
        g_arrive.notify_one();
        while (!req.done) {
            if (req.taken || g_leading) {
                g_cv.wait(lk);
                continue;
            }
            g_leading = true;
            // (system_clock: pthread_cond_timedwait, which TSan models; the steady
            // clock's pthread_cond_clockwait is not intercepted by GCC 11's TSan)
            g_arrive.wait_until(lk, std::chrono::system_clock::now() + kGather,
                                [] { return g_queue.size() >= g_last_batch; });
            std::vector<Request*> taken;
            taken.swap(g_queue);
            for (Request* q : taken) q->taken = true;
            g_last_batch = taken.size();
            lk.unlock();
            try {
                run_taken(taken);  // errors of the batch are recorded per request
            } catch (...) {        // (a host allocation failure): never leave the queue leaderless
                for (Request* q : taken)
                    if (!q->filled) q->status = TA_ERR_DEVICE, q->error = "host allocation failed";
            }
            lk.lock();
            for (Request* q : taken) q->done = true;
            g_leading = false;
            g_cv.notify_all();
        }
    }
    if (req.status == TA_ERR_BAD_TYPE || req.status == TA_ERR_CIGAR)
        throw std::invalid_argument(ta_status_string(req.status));
    if (req.status != TA_OK)
        throw std::runtime_error(std::string("team::Align: ") + ta_status_string(req.status) + ": " + req.error);
    if (target_begin) *target_begin = req.target_begin;
    return req.score;
}

}  // namespace team
