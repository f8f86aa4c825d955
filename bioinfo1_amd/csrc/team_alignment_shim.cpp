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
// team_mapper.cpp:680-683 handles both).  The GPU a call runs on:
// ta_set_default_device, else TEAM_ALIGN_DEVICE, else the calling thread's
// current HIP device.
//
// A pair that fits (n <= 4096, m <= 16384) goes to a resident single-pair
// server (ta_server.cpp): no launch and no copy per call.  Others, or every
// call with TEAM_ALIGN_SERVER=0, take the batch path:
// concurrent calls are combined: the mapper calls Align once per read from
// OpenMP threads (team_mapper.cpp:596), and one pair cannot fill a GPU.  A
// call queues its pair; if no batch is running, the caller becomes the
// leader: it takes the queued pairs, aligns them as one batch (one upload,
// the kernels, one download) and wakes their callers; otherwise it waits for
// a leader to take its pair.  A lone caller runs its own one-pair
// batch at once (no added wait), and under load a batch holds every pair
// that arrived while the previous one ran.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
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
    std::map<int, ta_context*> ctx;  // per device
    std::vector<char> qbytes, tbytes, arena;
    std::vector<uint64_t> qoff, toff, coff;
    std::vector<uint32_t> qlen, tlen, tb, clen;
    std::vector<int32_t> score;
    ~ThreadCtx() {
        for (auto& kv : ctx) ta_context_destroy(kv.second);
    }
};

thread_local ThreadCtx tc;

ta_context* thread_context(int device) {
    ta_context*& c = tc.ctx[device];
    if (!c) {
        int r = ta_context_create(device, &c);
        if (r != TA_OK) {
            c = nullptr;
            throw std::runtime_error("team::Align: no usable gfx950 GPU " + std::to_string(device) + " (" +
                                     std::string(ta_status_string(r)) + ")");
        }
    }
    return c;
}

// The device a call runs on: ta_set_default_device's choice, else the
// TEAM_ALIGN_DEVICE environment variable (read once), else the calling
// thread's current HIP device (hipSetDevice) as of the thread's first call --
// so a multi-GPU process whose threads each select their GPU gets its calls
// there.
std::atomic<int> g_default_device{-1};

int env_device() {
    static const int d = [] {
        const char* e = std::getenv("TEAM_ALIGN_DEVICE");
        return (e && *e) ? std::atoi(e) : -1;
    }();
    return d;
}

// This thread's device: set by ta_set_thread_device, else its current HIP
// device read at its first call (or first call after ta_set_thread_device(-1)):
// hipGetDevice costs ~6 µs per call on this runtime, a third of a small pair's
// whole call.  -1: not read yet.
thread_local int t_dev = -1;
thread_local bool t_dev_pinned = false;  // set by ta_set_thread_device (outranks the process-wide choices)

int call_device() {
    if (t_dev_pinned) return t_dev;
    int d = g_default_device.load(std::memory_order_relaxed);
    if (d >= 0) return d;
    if ((d = env_device()) >= 0) return d;
    if (t_dev < 0) t_dev = ta_current_device();
    return t_dev;
}

struct Request {
    const char* q;
    uint32_t ql;
    const char* t;
    uint32_t tl;
    int type, match, mismatch, gap;
    std::string* cigar;
    int device = 0;
    int32_t score = 0;
    uint32_t target_begin = 0;
    int status = TA_OK;
    std::string error;
    bool filled = false;  // results (or the batch's error) recorded
    bool taken = false;   // in a running batch
    bool done = false;
};

// ---- the low-latency path: one process-wide single-pair server per (device,
// type), created on first use (TEAM_ALIGN_SERVER=0 turns it off: every call
// then goes through the combined batches below).
constexpr uint32_t kServerSlots = 32;

bool server_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("TEAM_ALIGN_SERVER");
        return !(e && std::strcmp(e, "0") == 0);
    }();
    return on;
}

std::mutex g_srv_mu;
std::map<std::pair<int, int>, ta_server*> g_servers;  // nullptr: creation failed, do not retry

ta_server* server_for(int device, int type) {
    std::lock_guard<std::mutex> g(g_srv_mu);
    auto it = g_servers.find({device, type});
    if (it != g_servers.end()) return it->second;
    ta_server* s = nullptr;
    if (ta_server_create(device, type, kServerSlots, &s) != TA_OK) s = nullptr;
    g_servers[{device, type}] = s;
    return s;
}

// A batch's streams may share a hardware queue with a server's persistent
// kernel (GPU_MAX_HW_QUEUES: 4 per process), and a kernel queued behind it
// would wait until the server stops.  A batch therefore pauses the device's
// servers around its launches (calls meanwhile take the batch path; the
// server restarts with the next call after the batch).
struct ServersPaused {
    std::vector<ta_server*> s;
    explicit ServersPaused(int device) {
        {
            std::lock_guard<std::mutex> g(g_srv_mu);
            for (auto& kv : g_servers)
                if (kv.first.first == device && kv.second) s.push_back(kv.second);
        }
        for (ta_server* x : s) (void)ta_server_pause(x);
    }
    ~ServersPaused() {
        for (ta_server* x : s) (void)ta_server_resume(x);
    }
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
           (a->cigar != nullptr) == (b->cigar != nullptr) && a->device == b->device;
}

// Align reqs[0..n) (same type, scores, CIGAR request and device) as one batch.
// A failed batch of several pairs is rerun pair by pair: one caller's pair
// (a huge pair the device cannot hold) must not fail the callers it was
// combined with -- the reference's calls are independent.
void run_batch(Request* const* reqs, size_t n);

void run_batch_once(Request* const* reqs, size_t n, int& status) {
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
        ta_context* ctx = thread_context(reqs[0]->device);
        const ServersPaused paused(reqs[0]->device);
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
    status = r;
    if (r != TA_OK && n > 1) return;  // run_batch reruns the pairs one by one
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

void run_batch(Request* const* reqs, size_t n) {
    int r = TA_OK;
    run_batch_once(reqs, n, r);
    if (r != TA_OK && n > 1)
        for (size_t k = 0; k < n; ++k) run_batch_once(reqs + k, 1, r);
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
    const int device = call_device();
    // A large pair (>= 256k cells, no other call on the server) finishes sooner
    // as a one-pair batch (the packed kernel, both halves computing it) than on
    // one int32 wave, and so does a single caller's pair from ~45k cells
    // (~212 x 212) up: 224 x 224 178 vs 200 us, 256 x 256 196 vs 226
    // (profiles/bench/r06u_server_vs_batch.txt).  Concurrent calls of that size
    // are better off on the server (16 threads of 256 x 256: 70k vs 52k calls/s),
    // and a batch pauses the server: "single caller" means no call has had
    // company in the last 100 ms, not just none at this instant (which sent a
    // share of 8 threads' calls to the batch path, 256 x 256 35k -> 16k calls/s).
    static std::atomic<int> in_server{0}, in_align{0};
    static std::atomic<int64_t> last_company{INT64_MIN / 2};
    struct Active {
        std::atomic<int>& c;
        int k;
        explicit Active(std::atomic<int>& x) : c(x), k(x.fetch_add(1) + 1) {}
        ~Active() { c.fetch_sub(1); }
    } active(in_align);
    const uint64_t cells = (uint64_t)query_len * target_len;
    const bool mid = cells >= 45000 && cells < (1u << 18);
    bool single = false;
    if (mid || active.k > 1) {  // (a lone small call reads no clock)
        const int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                                std::chrono::steady_clock::now().time_since_epoch()).count();
        // (refreshed every 10 ms at most: concurrent callers do not bounce the line per call)
        if ((active.k > 1 || in_align.load() > 1) && now - last_company.load(std::memory_order_relaxed) > 10000000)
            last_company.store(now);
        single = mid && now - last_company.load() > 100000000;
    }
    const bool lone_large = (cells >= (1u << 18) && in_server.load() == 0) || single;
    if (server_enabled() && !lone_large) {
        ta_server* srv = server_for(device, t);
        if (srv && ta_server_fits(srv, query_len, target_len, match, mismatch, gap)) {
            struct Count {
                std::atomic<int>& c;
                explicit Count(std::atomic<int>& x) : c(x) { c.fetch_add(1); }
                ~Count() { c.fetch_sub(1); }
            } count(in_server);
            thread_local std::vector<char> cbuf;
            const uint64_t cap = ta_cigar_slot_bytes(query_len, target_len);
            if (cigar && cbuf.size() < cap) cbuf.resize(cap);
            int32_t sc = 0;
            uint32_t tb = 0, cl = 0;
            const int r = ta_server_align(srv, query, query_len, target, target_len, match, mismatch, gap,
                                          cigar != nullptr, &sc, &tb, cigar ? cbuf.data() : nullptr, cap, &cl);
            if (r == TA_OK) {
                if (cigar) cigar->assign(cbuf.data(), cl);  // assigned, not appended (:160)
                if (target_begin) *target_begin = tb;
                return sc;
            }
            if (r != TA_ERR_UNSERVED)
                throw std::runtime_error(std::string("team::Align: ") + ta_status_string(r));
        }
    }
    Request req{query, query_len, target, target_len, t, match, mismatch, gap, cigar, device};
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

extern "C" int ta_set_default_device(int device) {
    if (device >= ta_device_count()) return TA_ERR_ARG;
    g_default_device.store(device < 0 ? -1 : device, std::memory_order_relaxed);
    return TA_OK;
}

extern "C" int ta_set_thread_device(int device) {
    if (device >= ta_device_count()) return TA_ERR_ARG;
    t_dev = device < 0 ? -1 : device;  // -1: re-read the current HIP device at the next call
    t_dev_pinned = device >= 0;
    return TA_OK;
}
