// bioinfo1_amd/csrc/ta_api.hip -- host side of the extern "C" ABI
// (include/team_align_c.h): contexts, device plans, chunk launches and the
// host-memory batch entry point.  The planning itself (which kernel each pair
// runs in, chunks, offsets) is ta_planner.cpp; the DP is in ta_kernels.hip,
// ta_dual.hip and ta_flex.hip.
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/team_align_c.h"
#include "ta_context.h"
#include "ta_host_batch.h"
#include "ta_internal.h"
#include "ta_planner.h"

using ta_host::fail;

struct ta_plan {
    ta_context* ctx = nullptr;
    ta::Plan h;               // host plan (ta_planner.h)
    void* own_block = nullptr;  // device arrays of a plan made by ta_plan_create (one allocation)
    // device arrays (inside own_block, or inside ctx->blk for host-memory batches)
    uint32_t *d_qlen = nullptr, *d_tlen = nullptr, *d_order = nullptr, *d_singles = nullptr, *d_duals = nullptr,
             *d_flexes = nullptr;
    uint64_t *d_ptr_off = nullptr, *d_bnd_off = nullptr, *d_slot_off = nullptr;
    uint32_t *d_goal_i = nullptr, *d_goal_j = nullptr;
    uint32_t* d_fb = nullptr;  // packed-fill hand-back: [n_dual_pairs] list, then one counter per chunk
    uint32_t *d_flex_task_off = nullptr, *d_tickets = nullptr, *d_err = nullptr, *d_flex_tasks = nullptr;
    void* d_pout = nullptr;  // PassOut[2] per flex task
    void* d_dpout = nullptr;  // PassOut[2] per (pass, dual couple) of one multi-pass chunk
    uint32_t* d_stask_off = nullptr;  // pipelined int32 fill: per single, its first task
    uint64_t* d_stasks = nullptr;     // ... its tasks in ticket order
    void* d_spout = nullptr;          // ... PassOut per task
    uint8_t* d_pflag = nullptr;       // blk plans: per pair, handed back by the dual fill (band walk skips it)
};

namespace {

bool valid_type(int t) { return t == TA_GLOBAL || t == TA_LOCAL || t == TA_SEMI_GLOBAL; }

// Offsets of a linear plan's arrays in its device block.  Everything before
// `upload_end` is copied from the host (the error word and ticket counters
// as zeros); goal cells, the hand-back list and the pass results are device-only.
struct PlanOffs {
    uint64_t qlen, tlen, order, singles, duals, flexes, task_off, tasks, stask_off, stasks, ptr_off, bnd_off, slot_off,
        err, tickets;
    uint64_t goal_i, goal_j, fb, pout, dpout, spout, pflag;
};

// PassOut[2] (24 bytes each) per (pass, couple) of the largest multi-pass dual chunk
uint64_t dual_pout_bytes(const ta::Plan& h) {
    uint64_t n = 0;
    for (const auto& ch : h.chunks)
        if (ch.dpasses > 1) n = std::max<uint64_t>(n, 2ull * ch.dcount * ch.dpasses);
    return n * 24ull;
}

template <class T>
uint64_t vbytes(const std::vector<T>& v) {
    return v.size() * sizeof(T);
}

PlanOffs layout_uploaded(const ta::Plan& h, ta::BlockLayout& L) {
    PlanOffs o{};
    o.qlen = L.add(vbytes(h.qlen));
    o.tlen = L.add(vbytes(h.tlen));
    o.order = L.add(vbytes(h.order));
    o.singles = L.add(vbytes(h.singles));
    o.duals = L.add(vbytes(h.duals));
    o.flexes = L.add(vbytes(h.flexes));
    o.task_off = L.add(vbytes(h.flex_task_off));
    o.tasks = L.add(vbytes(h.flex_tasks));
    o.stask_off = L.add(vbytes(h.single_task_off));
    o.stasks = L.add(vbytes(h.single_tasks));
    o.ptr_off = L.add(vbytes(h.ptr_off));
    o.bnd_off = L.add(vbytes(h.bnd_off));
    o.slot_off = L.add(vbytes(h.slot_off));
    o.err = L.add(4);
    o.tickets = L.add(12ull * h.chunks.size());  // per chunk: flex, then dual, then pipelined int32
    return o;
}

void layout_scratch(const ta::Plan& h, ta::BlockLayout& L, PlanOffs& o) {
    o.goal_i = L.add(4ull * h.n_pairs);
    o.goal_j = L.add(4ull * h.n_pairs);
    o.fb = L.add(4ull * (h.n_dual_pairs + h.chunks.size()));
    o.pout = L.add(h.flexes.empty() ? 0 : h.flex_task_off.back() * 48ull + 16);
    o.dpout = L.add(dual_pout_bytes(h));
    o.spout = L.add(h.single_tasks.size() * 24ull);
    o.pflag = L.add(h.blk ? h.n_pairs : 0);
}

void pack(const ta::Plan& h, const PlanOffs& o, uint8_t* base) {
    auto put = [&](uint64_t at, const auto& v) {
        if (!v.empty()) std::memcpy(base + at, v.data(), vbytes(v));
    };
    put(o.qlen, h.qlen);
    put(o.tlen, h.tlen);
    put(o.order, h.order);
    put(o.singles, h.singles);
    put(o.duals, h.duals);
    put(o.flexes, h.flexes);
    put(o.task_off, h.flex_task_off);
    put(o.tasks, h.flex_tasks);
    put(o.stask_off, h.single_task_off);
    put(o.stasks, h.single_tasks);
    put(o.ptr_off, h.ptr_off);
    put(o.bnd_off, h.bnd_off);
    put(o.slot_off, h.slot_off);
    std::memset(base + o.err, 0, 4);
    std::memset(base + o.tickets, 0, 12ull * h.chunks.size());
}

void bind(ta_plan* pl, uint8_t* d, const PlanOffs& o) {
    auto u32 = [&](uint64_t at) { return reinterpret_cast<uint32_t*>(d + at); };
    auto u64 = [&](uint64_t at) { return reinterpret_cast<uint64_t*>(d + at); };
    pl->d_qlen = u32(o.qlen);
    pl->d_tlen = u32(o.tlen);
    pl->d_order = u32(o.order);
    pl->d_singles = u32(o.singles);
    pl->d_duals = u32(o.duals);
    pl->d_flexes = u32(o.flexes);
    pl->d_flex_task_off = u32(o.task_off);
    pl->d_flex_tasks = u32(o.tasks);
    pl->d_ptr_off = u64(o.ptr_off);
    pl->d_bnd_off = u64(o.bnd_off);
    pl->d_slot_off = u64(o.slot_off);
    pl->d_err = u32(o.err);
    pl->d_tickets = u32(o.tickets);
    pl->d_goal_i = u32(o.goal_i);
    pl->d_goal_j = u32(o.goal_j);
    pl->d_fb = u32(o.fb);
    pl->d_pout = d + o.pout;
    pl->d_dpout = d + o.dpout;
    pl->d_stask_off = u32(o.stask_off);
    pl->d_stasks = u64(o.stasks);
    pl->d_spout = d + o.spout;
    pl->d_pflag = d + o.pflag;
}

int check_args(ta_context* ctx, uint32_t n_pairs, const uint32_t* qlen, const uint32_t* tlen, int type) {
    if (!ctx) return TA_ERR_ARG;
    if (n_pairs && (!qlen || !tlen)) return fail(ctx, TA_ERR_ARG, "null argument");
    if (!valid_type(type)) return fail(ctx, TA_ERR_BAD_TYPE, ta_status_string(TA_ERR_BAD_TYPE));
    return TA_OK;
}

// Launches of one chunk: the fill kernels (int32 singles, equal-shape dual
// couples, rebased flex couples, and the int32 fill of the couples the packed
// kernels hand back), then the traceback kernel.
int exec_chunk(ta_plan* pl, const ta_device_io* io, hipStream_t s, uint32_t c, bool fill, bool trace) {
    const ta::Plan& h = pl->h;
    const auto& ch = h.chunks[c];
    ta_context* ctx = pl->ctx;
    if (h.ws_ptr_dwords)
        if (int r = ta_host::grow(ctx, ctx->ws_ptrs, h.ws_ptr_dwords * 4ull)) return r;
    if (h.ws_bnd_words)
        if (int r = ta_host::grow(ctx, ctx->ws_bnd, h.ws_bnd_words * 4ull)) return r;
    if (h.walk_group == 64 && h.want_cigar)
        if (int r = ta_host::grow(ctx, ctx->ws_runs, 4 * (h.slots_bytes + 4))) return r;  // band_runs_off
    uint32_t* d_ptrs = static_cast<uint32_t*>(ctx->ws_ptrs.p);
    int32_t* d_bnd = static_cast<int32_t*>(ctx->ws_bnd.p);
    if (fill) {
        roctxRangePushA("ta fill");
        // The flexible fill's pass hand-off records live in this buffer and are
        // recognised by their tag alone, so whatever an earlier user of the
        // memory left there (traceback codes of a freed workspace, other
        // plans' records) must not survive: zero it (tag 0 is never valid)
        // before any kernel of this chunk is enqueued.
        if ((ch.fcount || ch.dpasses > 1 || ch.spasses > 1) && ch.bnd_words) TA_HIP(ctx, hipMemsetAsync(d_bnd, 0, ch.bnd_words * 4ull, s));
        ta::FillArgs a{};
        a.order = pl->d_order;
        a.begin = ch.begin;
        a.count = ch.count;
        a.qbytes = reinterpret_cast<const uint8_t*>(io->query_bytes);
        a.qoff = io->query_off;
        a.qlen = pl->d_qlen;
        a.tbytes = reinterpret_cast<const uint8_t*>(io->target_bytes);
        a.toff = io->target_off;
        a.tlen = pl->d_tlen;
        a.match = h.match;
        a.mismatch = h.mismatch;
        a.gap = h.gap;
        a.ptrs = d_ptrs;
        a.ptr_off = pl->d_ptr_off;
        a.bnd = d_bnd;
        a.bnd_off = pl->d_bnd_off;
        a.score = io->score;
        a.target_begin = io->target_begin;
        a.goal_i = pl->d_goal_i;
        a.goal_j = pl->d_goal_j;
        a.fused = h.fused ? 1 : 0;
        a.slots = io->cigar_slots;
        a.slot_off = pl->d_slot_off;
        a.cigar_start = io->cigar_start;
        a.cigar_len = io->cigar_len;
        a.blk = h.blk ? (h.ck ? 2u : 1u) : 0u;
        a.pflag = (h.blk && h.walk_group == 64) ? pl->d_pflag : nullptr;
        if (ch.scount) {  // launched first: it may run on the aux stream beside the packed fill
            ta::FillArgs a1 = a;
            a1.order = pl->d_singles;
            a1.begin = ch.sbegin;
            a1.count = ch.scount;
            if (ch.spasses > 1) {  // one wave per (pair, pass), tickets pass-major
                a1.task_off = pl->d_stask_off;
                a1.tasks64 = pl->d_stasks;
                a1.ticket = pl->d_tickets + 2 * h.chunks.size() + c;
                a1.n_tasks = h.single_task_off[ch.sbegin + ch.scount] - h.single_task_off[ch.sbegin];
                a1.err = pl->d_err;
                a1.pout = pl->d_spout;
                TA_HIP(ctx, hipMemsetAsync(a1.ticket, 0, 4, s));
            }
            if (ch.dcount || ch.fcount) {  // beside the packed fill: fork onto the aux stream, join below
                if (int r = ta_host::lazy_stream(ctx, ctx->aux)) return r;
                TA_HIP(ctx, hipEventRecord(ctx->ev_fork, s));
                TA_HIP(ctx, hipStreamWaitEvent(ctx->aux, ctx->ev_fork, 0));
                TA_HIP(ctx, ta::launch_fill(h.type, h.want_cigar, h.wide, a1, ctx->aux));
            } else {
                TA_HIP(ctx, ta::launch_fill(h.type, h.want_cigar, h.wide, a1, s));
            }
        }
        if (ch.dcount || ch.fcount) {
            uint32_t* fb_list = pl->d_fb + 2ull * ch.cbegin;
            uint32_t* fb_count = pl->d_fb + h.n_dual_pairs + c;
            TA_HIP(ctx, hipMemsetAsync(fb_count, 0, 4, s));
            if (ch.dcount) {
                ta::FillArgs d = a;
                d.order = pl->d_duals;
                d.begin = ch.dbegin;
                d.count = ch.dcount;
                d.fb_list = fb_list;
                d.fb_count = fb_count;
                if (ch.dpasses > 1) {  // one wave per (couple, pass), tickets pass-major
                    d.ticket = pl->d_tickets + h.chunks.size() + c;
                    d.n_tasks = ch.dcount * ch.dpasses;
                    d.epoch = ++ctx->epoch & 0x3FFFFFFu;
                    d.err = pl->d_err;
                    d.pout = pl->d_dpout;
                    d.end_aligned = h.end_aligned ? 1u : 0u;
                    TA_HIP(ctx, hipMemsetAsync(d.ticket, 0, 4, s));
                }
                if (ch.fcount) {  // beside the flexible fill: fork onto aux2 (after the counter reset), join below
                    if (int r = ta_host::lazy_stream(ctx, ctx->aux2)) return r;
                    TA_HIP(ctx, hipEventRecord(ctx->ev_fork, s));
                    TA_HIP(ctx, hipStreamWaitEvent(ctx->aux2, ctx->ev_fork, 0));
                    TA_HIP(ctx, ta::launch_dual(h.type, h.want_cigar, d, ctx->aux2));
                    TA_HIP(ctx, hipEventRecord(ctx->ev_join2, ctx->aux2));
                } else {
                    TA_HIP(ctx, ta::launch_dual(h.type, h.want_cigar, d, s));
                }
            }
            if (ch.fcount) {
                ta::FillArgs d = a;
                d.order = pl->d_flexes;
                d.begin = ch.fbegin;
                d.count = ch.fcount;
                d.fb_list = fb_list;
                d.fb_count = fb_count;
                d.task_off = pl->d_flex_task_off;
                d.tasks = pl->d_flex_tasks;
                d.ticket = pl->d_tickets + c;
                d.n_tasks = h.flex_task_off[ch.fbegin + ch.fcount] - h.flex_task_off[ch.fbegin];
                d.epoch = ++ctx->epoch & 0x3FFFFFFu;
                d.err = pl->d_err;
                d.pout = pl->d_pout;
                TA_HIP(ctx, hipMemsetAsync(d.ticket, 0, 4, s));
                TA_HIP(ctx, ta::launch_flex(h.type, h.want_cigar, d, s));
            }
            if (ch.dcount && ch.fcount) TA_HIP(ctx, hipStreamWaitEvent(s, ctx->ev_join2, 0));
            // couples the packed kernels handed back ('-' in a query): int32
            // fill, wave count read on the device (grid sized for all of them)
            ta::FillArgs f = a;
            f.order = fb_list;
            f.begin = 0;
            f.count = 2 * (ch.dcount + ch.fcount);
            f.count_dev = fb_count;
            TA_HIP(ctx, ta::launch_fill(h.type, h.want_cigar, h.wide, f, s));
        }
        if (ch.scount && (ch.dcount || ch.fcount)) {  // join the aux stream
            TA_HIP(ctx, hipEventRecord(ctx->ev_join, ctx->aux));
            TA_HIP(ctx, hipStreamWaitEvent(s, ctx->ev_join, 0));
        }
        roctxRangePop();
    }
    if (trace && h.want_cigar && !h.fused) {
        roctxRangePushA("ta traceback");
        ta::TraceArgs t{};
        t.order = pl->d_order;
        t.begin = ch.begin;
        t.count = ch.count;
        t.qlen = pl->d_qlen;
        t.tlen = pl->d_tlen;
        t.ptrs = d_ptrs;
        t.ptr_off = pl->d_ptr_off;
        t.goal_i = pl->d_goal_i;
        t.goal_j = pl->d_goal_j;
        t.slots = io->cigar_slots;
        t.slot_off = pl->d_slot_off;
        t.cigar_start = io->cigar_start;
        t.cigar_len = io->cigar_len;
        t.score = io->score;
        t.qbytes = reinterpret_cast<const uint8_t*>(io->query_bytes);
        t.qoff = io->query_off;
        t.tbytes = reinterpret_cast<const uint8_t*>(io->target_bytes);
        t.toff = io->target_off;
        t.match = h.match;
        t.mismatch = h.mismatch;
        t.gap = h.gap;
        t.blk = h.blk ? (h.ck ? 2u : 1u) : 0u;
        if (h.walk_group == 64) {
            // band walks (one lane per pair), then the pairs of the couples the dual
            // fill handed back ('-' bytes) in the one-pair walk: its list and count
            t.pflag = pl->d_pflag;
            t.runs = static_cast<uint32_t*>(ctx->ws_runs.p);
            t.err = pl->d_err;
            t.fb_order = pl->d_fb + 2ull * ch.cbegin;
            t.fb_count = pl->d_fb + h.n_dual_pairs + c;
            TA_HIP(ctx, ta::launch_traceback(h.type, t, s, 64));
        } else {
            TA_HIP(ctx, ta::launch_traceback(h.type, t, s, h.walk_group));
        }
        roctxRangePop();
    }
    return TA_OK;
}

int check_io(ta_plan* pl, const ta_device_io* io) {
    if (!pl || !io) return TA_ERR_ARG;
    if (pl->h.n_pairs && (!io->query_off || !io->target_off || !io->score || !io->target_begin))
        return fail(pl->ctx, TA_ERR_ARG, "null device pointer");
    if (pl->h.want_cigar && pl->h.n_pairs && (!io->cigar_slots || !io->cigar_start || !io->cigar_len))
        return fail(pl->ctx, TA_ERR_ARG, "null cigar device pointer");
    return TA_OK;
}

// chunk == UINT32_MAX: every chunk
int exec(ta_plan* pl, const ta_device_io* io, hipStream_t s, uint32_t chunk, bool fill, bool trace) {
    ta_context* ctx = pl->ctx;
    TA_HIP(ctx, hipSetDevice(ctx->device));
    if (int r = ta_host::stream_enter(ctx, s)) return r;
    const uint32_t c0 = chunk == UINT32_MAX ? 0 : chunk;
    const uint32_t c1 = chunk == UINT32_MAX ? (uint32_t)pl->h.chunks.size() : chunk + 1;
    for (uint32_t c = c0; c < c1; ++c)
        if (int r = exec_chunk(pl, io, s, c, fill, trace)) return r;
    return ta_host::stream_leave(ctx, s);
}

// The linear plan as the host-memory batch driver sees it (ta_host_batch.h).
const char* plan_err_message(uint32_t err) {
    if (err & ta::kErrWalkCap) return "traceback: a band walk reached its event cap with cost left; results of this plan are invalid";
    return "packed fill: a pass hand-off poll timed out; results of this plan are invalid";
}

struct LinearHostPlan final : ta_host::HostPlan {
    ta_plan* pl;
    PlanOffs o{};
    explicit LinearHostPlan(ta_plan* p) : pl(p) {}
    void layout(ta::BlockLayout& L) override { o = layout_uploaded(pl->h, L); }
    void pack(uint8_t* base) override { ::pack(pl->h, o, base); }
    void layout_device_only(ta::BlockLayout& L) override { layout_scratch(pl->h, L, o); }
    void bind(uint8_t* dev) override { ::bind(pl, dev, o); }
    int execute(const ta_device_io* io, hipStream_t s) override { return exec(pl, io, s, UINT32_MAX, true, true); }
    uint64_t slots_bytes() const override { return pl->h.slots_bytes; }
    uint64_t err_offset() const override {
        return pl->h.flexes.empty() && pl->h.duals.empty() && pl->h.single_tasks.empty() ? UINT64_MAX : o.err;
    }
    const char* err_message(uint32_t err) const override { return plan_err_message(err); }
};

}  // namespace

extern "C" {

const char* ta_status_string(int status) {
    switch (status) {
        case TA_OK: return "ok";
        case TA_ERR_BAD_TYPE: return "Unknown AlignmentType provided.";
        case TA_ERR_CIGAR: return "Unknown error in determining cigar string.";
        case TA_ERR_ARG: return "invalid argument";
        case TA_ERR_DEVICE: return "device error";
        case TA_ERR_CAPACITY: return "cigar arena too small";
        case TA_ERR_RANGE: return "affine scoring out of range";
        case TA_ERR_UNSERVED: return "pair outside the single-pair server's limits";
        default: return "unknown status";
    }
}

const char* ta_last_error(const ta_context* ctx) { return ctx ? ctx->last_error.c_str() : ""; }

uint64_t ta_cigar_slot_bytes(uint32_t n, uint32_t m) { return ta::cigar_slot_bytes(n, m); }

int ta_context_create(int device, ta_context** out) {
    if (!out) return TA_ERR_ARG;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= device || device < 0) return TA_ERR_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return TA_ERR_DEVICE;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return TA_ERR_DEVICE;  // kernels are gfx950-only
    auto* c = new ta_context();
    c->device = device;
    c->cu_count = (uint32_t)std::max(1, prop.multiProcessorCount);
    // (streams: created on first use, ta_host::lazy_stream)
    if (hipSetDevice(device) != hipSuccess || hipEventCreateWithFlags(&c->ev_join2, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_last, hipEventDisableTiming) != hipSuccess) {
        ta_context_destroy(c);
        return TA_ERR_DEVICE;
    }
    *out = c;
    return TA_OK;
}

void ta_context_release(ta_context* ctx) {
    if (!ctx) return;
    std::lock_guard<std::mutex> lock(ctx->mu);
    (void)hipSetDevice(ctx->device);
    if (ctx->used) (void)hipEventSynchronize(ctx->ev_last);
    for (auto* b : {&ctx->blk, &ctx->out, &ctx->dst, &ctx->ws_ptrs, &ctx->ws_bnd, &ctx->ws_runs}) ta_host::release(*b, false);
    for (auto* b : {&ctx->pin_in, &ctx->pin_out}) ta_host::release(*b, true);
}

int ta_current_device(void) {
    int d = 0;
    return hipGetDevice(&d) == hipSuccess ? d : 0;
}

int ta_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

uint64_t ta_context_held_bytes(const ta_context* ctx) {
    if (!ctx) return 0;
    uint64_t n = 0;
    // only what a plan's code workspace can reuse: the code and pass-boundary
    // buffers (staging and output buffers are not handed to a plan's chunks, and
    // the band walk's event words, ws_runs, are needed beside the codes)
    for (const auto* b : {&ctx->ws_ptrs, &ctx->ws_bnd}) n += b->cap;
    return n;
}

void ta_context_destroy(ta_context* ctx) {
    if (!ctx) return;
    ta_context_release(ctx);
    for (hipStream_t s : {ctx->stream, ctx->aux, ctx->aux2})
        if (s) (void)hipStreamDestroy(s);
    for (hipEvent_t e : {ctx->ev_fork, ctx->ev_join, ctx->ev_join2, ctx->ev_last})
        if (e) (void)hipEventDestroy(e);
    delete ctx;
}

void ta_plan_destroy(ta_plan* pl) {
    if (!pl) return;
    if (pl->own_block) {
        (void)hipSetDevice(pl->ctx->device);
        (void)hipFree(pl->own_block);
    }
    delete pl;
}

int ta_plan_create(ta_context* ctx, uint32_t n_pairs, const uint32_t* qlen, const uint32_t* tlen, int type,
                   int match, int mismatch, int gap, int want_cigar, uint64_t budget, uint32_t flags, ta_plan** out) {
    if (!out) return TA_ERR_ARG;
    *out = nullptr;
    if (int r = check_args(ctx, n_pairs, qlen, tlen, type)) return r;
    TA_HIP(ctx, hipSetDevice(ctx->device));
    auto* pl = new ta_plan();
    pl->ctx = ctx;
    ta::build_plan(pl->h, n_pairs, qlen, tlen, type, match, mismatch, gap, want_cigar != 0,
                   budget ? budget : ta_host::default_budget(ctx), flags, 4 * ctx->cu_count);
    // all per-pair arrays in one device allocation, uploaded in one copy
    ta::BlockLayout L;
    PlanOffs o = layout_uploaded(pl->h, L);
    const uint64_t upload = L.bytes;
    layout_scratch(pl->h, L, o);
    std::vector<uint8_t> host(upload);
    pack(pl->h, o, host.data());
    hipError_t e = hipMalloc(&pl->own_block, std::max<uint64_t>(L.bytes, 256));
    if (e == hipSuccess) e = hipMemcpy(pl->own_block, host.data(), upload, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        ta_plan_destroy(pl);
        return fail(ctx, TA_ERR_DEVICE, std::string("ta_plan_create: ") + hipGetErrorString(e));
    }
    bind(pl, static_cast<uint8_t*>(pl->own_block), o);
    *out = pl;
    return TA_OK;
}

uint64_t ta_plan_cigar_slots_bytes(const ta_plan* pl) { return pl ? pl->h.slots_bytes : 0; }
uint64_t ta_plan_workspace_bytes(const ta_plan* pl) {
    if (!pl) return 0;
    const ta::Plan& h = pl->h;
    // codes / checkpoints, pass-boundary rows, and the walks' event words (exec_chunk ws_runs)
    const uint64_t runs = (h.walk_group == 64 && h.want_cigar) ? 4 * (h.slots_bytes + 4) : 0;
    return (h.ws_ptr_dwords + h.ws_bnd_words) * 4ull + runs;
}
uint32_t ta_plan_chunks(const ta_plan* pl) { return pl ? (uint32_t)pl->h.chunks.size() : 0; }
uint32_t ta_plan_dual_pairs(const ta_plan* pl) { return pl ? pl->h.n_dual_pairs : 0; }
uint32_t ta_plan_flex_pairs(const ta_plan* pl) { return pl ? (uint32_t)pl->h.flexes.size() : 0; }
int ta_plan_fused(const ta_plan* pl) { return pl && pl->h.fused ? 1 : 0; }

int ta_plan_walk(const ta_plan* pl) {
    if (!pl) return -1;
    return pl->h.walk_group | (pl->h.blk ? 0x100 : 0) | (pl->h.ck ? 0x200 : 0);
}

int ta_plan_pair_chunks(const ta_plan* pl, uint32_t* chunk_of_pair) {
    if (!pl || !chunk_of_pair) return TA_ERR_ARG;
    for (uint32_t c = 0; c < (uint32_t)pl->h.chunks.size(); ++c) {
        const auto& ch = pl->h.chunks[c];
        for (uint32_t k = ch.begin; k < ch.begin + ch.count; ++k) chunk_of_pair[pl->h.order[k]] = c;
    }
    return TA_OK;
}

int ta_plan_execute(ta_plan* pl, const ta_device_io* io, void* stream) {
    if (int r = check_io(pl, io)) return r;
    std::lock_guard<std::mutex> lock(pl->ctx->mu);
    return exec(pl, io, (hipStream_t)stream, UINT32_MAX, true, true);
}

int ta_plan_execute_fill(ta_plan* pl, const ta_device_io* io, void* stream, uint32_t chunk) {
    if (int r = check_io(pl, io)) return r;
    if (chunk >= pl->h.chunks.size()) return pl->h.n_pairs ? TA_ERR_ARG : TA_OK;
    std::lock_guard<std::mutex> lock(pl->ctx->mu);
    return exec(pl, io, (hipStream_t)stream, chunk, true, false);
}

int ta_plan_execute_traceback(ta_plan* pl, const ta_device_io* io, void* stream, uint32_t chunk) {
    if (int r = check_io(pl, io)) return r;
    if (chunk >= pl->h.chunks.size()) return pl->h.n_pairs ? TA_ERR_ARG : TA_OK;
    std::lock_guard<std::mutex> lock(pl->ctx->mu);
    return exec(pl, io, (hipStream_t)stream, chunk, false, true);
}

int ta_plan_check(ta_plan* pl) {
    if (!pl) return TA_ERR_ARG;
    if (pl->h.flexes.empty() && pl->h.duals.empty() && pl->h.single_tasks.empty()) return TA_OK;
    uint32_t err = 0;
    TA_HIP(pl->ctx, hipSetDevice(pl->ctx->device));
    TA_HIP(pl->ctx, hipMemcpy(&err, pl->d_err, 4, hipMemcpyDeviceToHost));
    if (!err) return TA_OK;
    TA_HIP(pl->ctx, hipMemset(pl->d_err, 0, 4));
    return fail(pl->ctx, TA_ERR_DEVICE, plan_err_message(err));
}

int ta_compact_cigars(ta_context* ctx, uint32_t n_pairs, const char* cigar_slots, const uint64_t* cigar_start,
                      const uint32_t* cigar_len, const uint64_t* dst_off, char* dst, void* stream) {
    if (!ctx) return TA_ERR_ARG;
    if (!n_pairs) return TA_OK;
    if (!cigar_slots || !cigar_start || !cigar_len || !dst_off || !dst) return fail(ctx, TA_ERR_ARG, "null device pointer");
    TA_HIP(ctx, hipSetDevice(ctx->device));
    ta::CompactArgs ca{n_pairs, cigar_slots, cigar_start, cigar_len, dst_off, dst};
    TA_HIP(ctx, ta::launch_compact(ca, (hipStream_t)stream));
    return TA_OK;
}

int ta_align_batch(ta_context* ctx, uint32_t n_pairs, const char* qb, const uint64_t* qoff, const uint32_t* qlen,
                   const char* tbytes, const uint64_t* toff, const uint32_t* tlen, int type, int match,
                   int mismatch, int gap, int want_cigar, int32_t* score, uint32_t* target_begin, char* arena,
                   uint64_t arena_bytes, uint64_t* cigar_off, uint32_t* cigar_len) {
    return ta_align_batch_flags(ctx, n_pairs, qb, qoff, qlen, tbytes, toff, tlen, type, match, mismatch, gap,
                                want_cigar, score, target_begin, arena, arena_bytes, cigar_off, cigar_len, 0);
}

int ta_align_batch_flags(ta_context* ctx, uint32_t n_pairs, const char* qb, const uint64_t* qoff,
                         const uint32_t* qlen, const char* tbytes, const uint64_t* toff, const uint32_t* tlen,
                         int type, int match, int mismatch, int gap, int want_cigar, int32_t* score,
                         uint32_t* target_begin, char* arena, uint64_t arena_bytes, uint64_t* cigar_off,
                         uint32_t* cigar_len, uint32_t flags) {
    uint64_t qend = 0, tend = 0;
    if (int r = ta_host::check_host_batch(ctx, type, n_pairs, qb, qoff, qlen, tbytes, toff, tlen, want_cigar, arena,
                                          cigar_off, cigar_len, &qend, &tend))
        return r;
    if (n_pairs == 0) return TA_OK;
    std::lock_guard<std::mutex> lock(ctx->mu);
    TA_HIP(ctx, hipSetDevice(ctx->device));
    ta_plan pl;
    pl.ctx = ctx;
    ta::build_plan(pl.h, n_pairs, qlen, tlen, type, match, mismatch, gap, want_cigar != 0,
                   ta_host::batch_budget(ctx, n_pairs, qlen, tlen, want_cigar, 4), flags, 4 * ctx->cu_count);
    LinearHostPlan hp(&pl);
    return ta_host::host_batch(ctx, hp, n_pairs, qb, qoff, qlen, tbytes, toff, tlen, qend, tend, want_cigar, score,
                               target_begin, arena, arena_bytes, cigar_off, cigar_len);
}

}  // extern "C"
