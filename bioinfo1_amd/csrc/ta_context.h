// bioinfo1_amd/csrc/ta_context.h -- the opaque ta_context of
// include/team_align_c.h and the host helpers shared by the drivers of the
// linear-gap plans (ta_api.hip) and the affine-gap extension (ta_affine.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <string>

#include "../../include/team_align_c.h"

struct ta_context {
    int device = 0;
    hipStream_t stream = nullptr;  // host-memory batches (ta_align_batch*)
    // a chunk's int32 fill (single pairs) runs on aux beside its packed fill,
    // the equal-shape dual fill on aux2 beside the flexible one; the caller's
    // stream waits for them (fork / join events)
    hipStream_t aux = nullptr, aux2 = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_join2 = nullptr;
    // Executions share the context's workspace: an execution on another
    // stream than the previous one first waits for this event, recorded at
    // the end of the previous execution (plans of one context on
    // several torch streams).
    hipStream_t last_stream = nullptr;
    hipEvent_t ev_last = nullptr;
    bool used = false;
    std::string last_error;
    std::mutex mu;  // one execution at a time per context
    struct Buf {
        void* p = nullptr;
        size_t cap = 0;
    };
    // Grow-only device buffers of the host-memory batches: `blk` holds the
    // plan arrays and the inputs (uploaded in one copy) and the plan's device
    // scratch; `out` the outputs (score, target_begin, cigar_len,
    // cigar_start, CIGAR slots); `dst` the compacted CIGARs.
    Buf blk, out, dst;
    // Grow-only pinned host staging of the host-memory batches (hipHostMalloc).
    Buf pin_in, pin_out;
    // Traceback-code and pass-boundary workspace, shared by every plan of this
    // context and grown at execute time (a plan's chunks are sized by its budget).
    Buf ws_ptrs, ws_bnd;
    // Band walks (ta_walk_band.h): the run words of every pair before they are
    // formatted into its CIGAR slot (2 x the plan's slot bytes).
    Buf ws_runs;
    uint32_t cu_count = 256;
    uint32_t epoch = 0;  // flexible-fill launches so far (tags of their pass hand-off records)
};

namespace ta_host {

inline int fail(ta_context* ctx, int code, const std::string& msg) {
    if (ctx) ctx->last_error = msg;
    return code;
}

// A context's own streams are created on first use: each HIP stream takes one
// of the process's few hardware queues (GPU_MAX_HW_QUEUES, 4 by default), and
// streams beyond that share queues, where a copy queued behind another
// stream's kernel waits for it.  A caller that drives plans on its own
// streams (config 2: the whole batch in one dual fill) then creates none.
inline int lazy_stream(ta_context* ctx, hipStream_t& s) {
    if (s) return TA_OK;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        s = nullptr;
        return fail(ctx, TA_ERR_DEVICE, "hipStreamCreateWithFlags failed");
    }
    return TA_OK;
}

#define TA_HIP(ctx, expr)                                                                                    \
    do {                                                                                                     \
        hipError_t e_ = (expr);                                                                              \
        if (e_ != hipSuccess)                                                                                \
            return ta_host::fail((ctx), TA_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// Grow-only device buffer (contents are not kept).
inline int grow(ta_context* ctx, ta_context::Buf& b, size_t bytes) {
    if (bytes <= b.cap) return TA_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    // small buffers get headroom (fewer regrowths); workspaces exactly what was asked
    const size_t want = std::max<size_t>(bytes < (64u << 20) ? bytes + bytes / 8 : bytes, 4096);
    TA_HIP(ctx, hipMalloc(&b.p, want));
    b.cap = want;
    return TA_OK;
}

// Grow-only pinned host buffer (contents are not kept).
inline int grow_pinned(ta_context* ctx, ta_context::Buf& b, size_t bytes) {
    if (bytes <= b.cap) return TA_OK;
    if (b.p) (void)hipHostFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    const size_t want = std::max<size_t>(bytes < (64u << 20) ? bytes + bytes / 8 : bytes, 1 << 16);
    TA_HIP(ctx, hipHostMalloc(&b.p, want, hipHostMallocDefault));
    b.cap = want;
    return TA_OK;
}

inline void release(ta_context::Buf& b, bool pinned) {
    if (b.p) (void)(pinned ? hipHostFree(b.p) : hipFree(b.p));
    b.p = nullptr;
    b.cap = 0;
}

// Start of an execution on stream s: wait for the context's previous
// execution when it ran on another stream (shared workspace).
inline int stream_enter(ta_context* ctx, hipStream_t s) {
    if (ctx->used && s != ctx->last_stream) TA_HIP(ctx, hipStreamWaitEvent(s, ctx->ev_last, 0));
    return TA_OK;
}

inline int stream_leave(ta_context* ctx, hipStream_t s) {
    TA_HIP(ctx, hipEventRecord(ctx->ev_last, s));
    ctx->last_stream = s;
    ctx->used = true;
    return TA_OK;
}

// Workspace budget (bytes of traceback codes per chunk) when the caller
// passes 0: half of what is free on the device (counting the context's
// cached workspace), at most 64 GiB -- a chunk of 64 GiB of 2-bit codes is
// 256 G cells, thousands of waves even for 20 kb reads; callers that want
// the whole HBM (bench.py's config 3 / 5 runs) pass their own budget.
inline uint64_t default_budget(const ta_context* ctx) {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return 16ull << 30;
    const uint64_t avail = (uint64_t)free_b + ctx->ws_ptrs.cap + ctx->ws_bnd.cap;
    return std::max<uint64_t>(std::min<uint64_t>(avail / 2, 64ull << 30), 1ull << 30);
}

}  // namespace ta_host
