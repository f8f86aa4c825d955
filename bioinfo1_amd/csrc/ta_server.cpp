// bioinfo1_amd/csrc/ta_server.cpp -- the low-latency single-pair path behind
// team::Align (include/team_align_c.h ta_server_*).
//
// The reference's Align is a synchronous per-call function
// (team_alignment.cpp:49-56) that team_mapper.cpp calls once per read
// (:666-678, :755-767).  Through the batch ABI one tiny call costs a pinned
// upload, two kernel launches, a download and a stream synchronisation
// (~37 us).  A server instead keeps a persistent kernel resident (serve_kernel,
// ta_kernels.hip): one wave per slot polls its slot in fine-grained pinned
// host memory.  A call claims a free slot, writes its pair into it and bumps
// the slot's sequence number; the slot's wave copies the bytes to HBM, runs
// the int32 fill with the walk fused into it (one wave, the pair's passes in
// turn), writes score, target_begin and CIGAR back into the slot and
// publishes `done`.  No launch, no copy, no stream operation per call.
//
// Lifetime: the kernel is launched by the first call and stopped (stop flag,
// then the end event) after kIdleStop without calls; a keeper thread bumps a
// heartbeat every millisecond while it runs, and every wave exits by itself
// when the heartbeat stops for kHeartbeatTimeout (the process died or hung),
// so the grid always drains.  A call whose kernel ended under it (it stalled
// past the timeout) sees the end event complete, restarts the kernel and is
// served: a restarted wave resumes from its slot's last `done`.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/team_align_c.h"
#include "ta_internal.h"
#include "ta_planner.h"

namespace {

using Clock = std::chrono::steady_clock;
constexpr auto kIdleStop = std::chrono::milliseconds(200);  // no calls this long: the kernel stops
constexpr uint64_t kHeartbeatTimeout = 200000000ull;         // 2 s of the 100 MHz wall clock
constexpr uint32_t kMaxSlots = 64;

inline uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}

// Restores the calling thread's HIP device on scope exit (the server's
// launches run on its own device without moving the caller's).
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceScope() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

}  // namespace

struct ta_server {
    int device = 0, type = 0;
    uint32_t slots = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev_end = nullptr;  // completes when every wave of the running kernel has exited
    char* host = nullptr;         // slots (fine-grained pinned)
    ta::ServeCtl* ctl = nullptr;  // fine-grained pinned
    void* dev = nullptr;          // per-slot HBM scratch
    ta::ServeArgs args{};
    std::mutex mu;                // running / start / stop
    bool running = false;
    std::atomic<uint32_t> active{0};
    std::atomic<int> paused{0};   // > 0: calls are turned away (ta_server_pause)
    std::atomic<uint64_t> last_call{0};
    std::unique_ptr<std::atomic<uint32_t>[]> busy;
    std::thread keeper;
    bool quit = false;
    std::condition_variable cv;
    std::string last_error;

    ta::ServeHdr* hdr(uint32_t s) { return reinterpret_cast<ta::ServeHdr*>(host + (uint64_t)s * ta::kSrvStride); }

    int start_locked() {
        DeviceScope ds(device);
        __atomic_store_n(&ctl->stop, 0u, __ATOMIC_RELEASE);
        if (ta::launch_serve(type, args, slots, stream) != hipSuccess) return TA_ERR_DEVICE;
        if (hipEventRecord(ev_end, stream) != hipSuccess) return TA_ERR_DEVICE;
        running = true;
        return TA_OK;
    }

    void stop_locked() {
        if (!running) return;
        __atomic_store_n(&ctl->stop, 1u, __ATOMIC_RELEASE);
        (void)hipEventSynchronize(ev_end);  // every wave sees the flag within one poll
        running = false;
    }

    // true when the kernel ended although the host did not stop it
    bool ended() { return hipEventQuery(ev_end) == hipSuccess; }

    void keep() {
        std::unique_lock<std::mutex> lk(mu);
        while (!quit) {
            cv.wait_for(lk, std::chrono::milliseconds(1));
            if (quit) break;
            if (!running) continue;
            if (active.load() == 0 && now_ns() - last_call.load() > (uint64_t)std::chrono::nanoseconds(kIdleStop).count()) {
                stop_locked();
            } else {
                __atomic_fetch_add(&ctl->heartbeat, 1u, __ATOMIC_RELEASE);
            }
        }
    }
};

namespace {

std::mutex g_servers_mu;
std::vector<ta_server*> g_servers;
bool g_atexit = false;

void stop_all_servers() {
    std::lock_guard<std::mutex> g(g_servers_mu);
    for (ta_server* s : g_servers) {
        {
            std::lock_guard<std::mutex> lk(s->mu);
            s->quit = true;
            s->stop_locked();
        }
        s->cv.notify_all();
        if (s->keeper.joinable()) s->keeper.join();
    }
}

bool fits(const ta_server* s, uint32_t n, uint32_t m, int match, int mismatch, int gap) {
    if (n > ta::kSrvQMax || m > ta::kSrvTMax) return false;
    if (s->type == TA_LOCAL) {  // the scaled local kernel (ta_planner.cpp "wide")
        const uint64_t mag = std::max<uint64_t>({1ull, (uint64_t)std::llabs(match), (uint64_t)std::llabs(mismatch),
                                                 (uint64_t)std::llabs(gap)});
        if (((uint64_t)n + m) * mag >= (1ull << 25)) return false;
    }
    return true;
}

}  // namespace

extern "C" {

int ta_server_create(int device, int type, uint32_t slots, ta_server** out) {
    if (!out) return TA_ERR_ARG;
    *out = nullptr;
    if (type != TA_GLOBAL && type != TA_LOCAL && type != TA_SEMI_GLOBAL) return TA_ERR_BAD_TYPE;
    if (slots == 0 || slots > kMaxSlots) return TA_ERR_ARG;
    DeviceScope ds(device);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return TA_ERR_DEVICE;
    auto* s = new ta_server();
    s->device = device;
    s->type = type;
    s->slots = slots;
    s->busy.reset(new std::atomic<uint32_t>[slots]);
    for (uint32_t k = 0; k < slots; ++k) s->busy[k] = 0;
    auto fail = [&](const char* what) {
        ta_server_destroy(s);
        (void)what;
        return TA_ERR_DEVICE;
    };
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) return fail("stream");
    if (hipEventCreateWithFlags(&s->ev_end, hipEventDisableTiming) != hipSuccess) return fail("event");
    const unsigned pin = hipHostMallocCoherent | hipHostMallocMapped;
    if (hipHostMalloc(reinterpret_cast<void**>(&s->host), (size_t)slots * ta::kSrvStride, pin) != hipSuccess)
        return fail("slots");
    if (hipHostMalloc(reinterpret_cast<void**>(&s->ctl), sizeof(ta::ServeCtl), pin) != hipSuccess) return fail("ctl");
    std::memset(s->host, 0, (size_t)slots * ta::kSrvStride);
    std::memset(s->ctl, 0, sizeof(ta::ServeCtl));
    // per-slot HBM: sequence copies, codes, boundary rows, CIGAR slots, records
    const uint64_t ptr_dw = ta::ptr_dwords(ta::kSrvQMax, ta::kSrvTMax);
    const uint64_t bnd_w = ta::bnd_words(ta::kSrvQMax, ta::kSrvTMax);
    const uint64_t cslot = (ta::cigar_slot_bytes(ta::kSrvQMax, ta::kSrvTMax) + 255) & ~255ull;
    ta::BlockLayout L;
    const uint64_t o_q = L.add((uint64_t)slots * ta::kSrvQMax), o_t = L.add((uint64_t)slots * ta::kSrvTMax);
    const uint64_t o_p = L.add((uint64_t)slots * ptr_dw * 4), o_b = L.add((uint64_t)slots * bnd_w * 4);
    const uint64_t o_c = L.add((uint64_t)slots * cslot);
    const uint64_t o_off = L.add((uint64_t)slots * 8 * 6);   // qoff toff ptr_off bnd_off slot_off cigar_start
    const uint64_t o_u32 = L.add((uint64_t)slots * 4 * 8);   // qlen tlen score tb goal_i goal_j cigar_len (+1)
    if (hipMalloc(&s->dev, L.bytes) != hipSuccess) return fail("scratch");
    uint8_t* d = static_cast<uint8_t*>(s->dev);
    std::vector<uint64_t> off((size_t)slots * 6);
    for (uint32_t k = 0; k < slots; ++k) {
        off[0 * slots + k] = (uint64_t)k * ta::kSrvQMax;
        off[1 * slots + k] = (uint64_t)k * ta::kSrvTMax;
        off[2 * slots + k] = (uint64_t)k * ptr_dw;
        off[3 * slots + k] = (uint64_t)k * bnd_w;
        off[4 * slots + k] = (uint64_t)k * cslot;
        off[5 * slots + k] = 0;
    }
    if (hipMemcpy(d + o_off, off.data(), off.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(d + o_u32, 0, (size_t)slots * 4 * 8) != hipSuccess)
        return fail("init");
    uint64_t* offs = reinterpret_cast<uint64_t*>(d + o_off);
    uint32_t* u32 = reinterpret_cast<uint32_t*>(d + o_u32);
    ta::FillArgs& a = s->args.fa;
    a = ta::FillArgs{};
    a.qbytes = d + o_q;
    a.tbytes = d + o_t;
    a.qoff = offs;
    a.toff = offs + slots;
    a.ptr_off = offs + 2 * slots;
    a.bnd_off = offs + 3 * slots;
    a.slot_off = offs + 4 * slots;
    a.cigar_start = offs + 5 * slots;
    a.qlen = u32;
    a.tlen = u32 + slots;
    a.score = reinterpret_cast<int32_t*>(u32 + 2 * slots);
    a.target_begin = u32 + 3 * slots;
    a.goal_i = u32 + 4 * slots;
    a.goal_j = u32 + 5 * slots;
    a.cigar_len = u32 + 6 * slots;
    a.ptrs = reinterpret_cast<uint32_t*>(d + o_p);
    a.bnd = reinterpret_cast<int32_t*>(d + o_b);
    a.slots = reinterpret_cast<char*>(d + o_c);
    s->args.host = s->host;
    s->args.ctl = s->ctl;
    s->args.hb_timeout = kHeartbeatTimeout;
    s->keeper = std::thread([s] { s->keep(); });
    {
        std::lock_guard<std::mutex> g(g_servers_mu);
        g_servers.push_back(s);
        if (!g_atexit) {  // registered after the HIP runtime's own handlers: runs before them
            g_atexit = true;
            std::atexit(stop_all_servers);
        }
    }
    *out = s;
    return TA_OK;
}

void ta_server_destroy(ta_server* s) {
    if (!s) return;
    {
        std::lock_guard<std::mutex> g(g_servers_mu);
        for (auto it = g_servers.begin(); it != g_servers.end(); ++it)
            if (*it == s) {
                g_servers.erase(it);
                break;
            }
    }
    {
        std::lock_guard<std::mutex> lk(s->mu);
        s->quit = true;
        s->stop_locked();
    }
    s->cv.notify_all();
    if (s->keeper.joinable()) s->keeper.join();
    DeviceScope ds(s->device);
    if (s->dev) (void)hipFree(s->dev);
    if (s->host) (void)hipHostFree(s->host);
    if (s->ctl) (void)hipHostFree(s->ctl);
    if (s->ev_end) (void)hipEventDestroy(s->ev_end);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
}

int ta_server_fits(const ta_server* s, uint32_t n, uint32_t m, int match, int mismatch, int gap) {
    return s && fits(s, n, m, match, mismatch, gap) ? 1 : 0;
}

int ta_server_align(ta_server* s, const char* q, uint32_t n, const char* t, uint32_t m, int match, int mismatch,
                    int gap, int want_cigar, int32_t* score, uint32_t* target_begin, char* cigar, uint64_t cigar_cap,
                    uint32_t* cigar_len) {
    if (!s || (n && !q) || (m && !t) || (want_cigar && (!cigar || !cigar_len))) return TA_ERR_ARG;
    if (!fits(s, n, m, match, mismatch, gap)) return TA_ERR_UNSERVED;
    // a free slot (callers start at a per-thread hint: a thread keeps its slot)
    static thread_local uint32_t hint = 0;
    uint32_t k = UINT32_MAX;
    for (uint32_t i = 0; i < s->slots; ++i) {
        const uint32_t c = (hint + i) % s->slots;
        uint32_t z = 0;
        if (s->busy[c].load(std::memory_order_relaxed) == 0 && s->busy[c].compare_exchange_strong(z, 1u)) {
            k = c;
            break;
        }
    }
    if (k == UINT32_MAX) return TA_ERR_UNSERVED;  // more concurrent callers than slots: the batch path
    hint = k;
    s->active.fetch_add(1);
    if (s->paused.load() > 0) {  // (after counting itself: ta_server_pause waits for `active` to drain)
        s->active.fetch_sub(1);
        s->busy[k].store(0, std::memory_order_release);
        return TA_ERR_UNSERVED;
    }
    s->last_call.store(now_ns());
    {
        // (no hipEventQuery on this path: a HIP call per request costs microseconds;
        // a kernel that ended under a running server -- its heartbeat timed out --
        // is noticed by the wait below within 10 ms and restarted)
        std::lock_guard<std::mutex> lk(s->mu);
        if (!s->running) {
            if (int r = s->start_locked()) {
                s->active.fetch_sub(1);
                s->busy[k].store(0);
                return r;
            }
        }
    }
    ta::ServeHdr* h = s->hdr(k);
    char* slot = reinterpret_cast<char*>(h);
    h->n = n;
    h->m = m;
    h->match = match;
    h->mismatch = mismatch;
    h->gap = gap;
    h->want_cigar = want_cigar ? 1u : 0u;
    if (n) std::memcpy(slot + ta::kSrvQOff, q, n);
    if (m) std::memcpy(slot + ta::kSrvTOff, t, m);
    const uint32_t seq = h->seq + 1u;
    __atomic_store_n(&h->seq, seq, __ATOMIC_RELEASE);
    // wait for `done`: spin first (a small pair takes microseconds), then yield;
    // now and then check that the kernel still runs
    int rc = TA_OK;
    const uint64_t t0 = now_ns();
    uint64_t next_check = t0 + 10000000ull;
    for (uint64_t spins = 0; __atomic_load_n(&h->done, __ATOMIC_ACQUIRE) != seq; ++spins) {
        if (spins < 20000) {
            __builtin_ia32_pause();
            continue;
        }
        std::this_thread::yield();
        const uint64_t now = now_ns();
        if (now < next_check) continue;
        next_check = now + 10000000ull;
        std::lock_guard<std::mutex> lk(s->mu);
        if (s->ended()) {  // the kernel stopped under this call: start it again (the slot resumes from `done`)
            s->running = false;
            if ((rc = s->start_locked()) != TA_OK) break;
        }
    }
    if (rc == TA_OK) {
        rc = (int)h->status;
        if (rc == TA_OK) {
            if (score) *score = h->score;
            if (target_begin) *target_begin = h->target_begin;
            if (want_cigar) {
                if (h->cigar_len > cigar_cap) {
                    rc = TA_ERR_CAPACITY;
                } else {
                    std::memcpy(cigar, slot + ta::kSrvCOff, h->cigar_len);
                    *cigar_len = h->cigar_len;
                }
            }
        }
    }
    s->last_call.store(now_ns());
    s->active.fetch_sub(1);
    s->busy[k].store(0, std::memory_order_release);
    return rc;
}

int ta_server_last_times(const ta_server* s, uint32_t slot, double* us) {
    if (!s || !us || slot >= s->slots) return TA_ERR_ARG;
    const ta::ServeHdr* h = const_cast<ta_server*>(s)->hdr(slot);
    for (int k = 0; k < 4; ++k) us[k] = h->pad1[k] * 0.01;  // 100 MHz ticks
    return TA_OK;
}

int ta_server_pause(ta_server* s) {
    if (!s) return TA_ERR_ARG;
    s->paused.fetch_add(1);
    while (s->active.load() != 0) std::this_thread::yield();  // calls in flight finish (bounded by their pairs)
    std::lock_guard<std::mutex> lk(s->mu);
    s->stop_locked();
    return TA_OK;
}

int ta_server_resume(ta_server* s) {
    if (!s) return TA_ERR_ARG;
    s->paused.fetch_sub(1);
    return TA_OK;
}

int ta_server_running(const ta_server* s) {
    if (!s) return 0;
    std::lock_guard<std::mutex> lk(const_cast<ta_server*>(s)->mu);
    return s->running ? 1 : 0;
}

}  // extern "C"
