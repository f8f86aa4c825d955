// bioinfo1_amd/csrc/ta_context.h -- the opaque ta_context of
// include/team_align_c.h, shared by the host drivers of the linear-gap plans
// (ta_api.hip) and the affine-gap extension (ta_affine.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>
#include <string>
#include <vector>

struct ta_context {
    int device = 0;
    hipStream_t stream = nullptr;
    // a second stream on which a chunk's int32 fill (single pairs) runs beside
    // its packed two-pair fill; the caller's stream waits for it (fork / join)
    hipStream_t aux = nullptr, aux2 = nullptr;  // aux2: the equal-shape dual fill beside the flexible one
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_join2 = nullptr;
    // staged plans: tracebacks on their own stream, one event per stage
    hipStream_t tbs = nullptr;
    hipEvent_t ev_tb_done = nullptr;
    std::vector<hipEvent_t> ev_stage;
    std::string last_error;
    std::mutex mu;  // one batch at a time per context
    // grow-only device staging for ta_align_batch
    struct Buf {
        void* p = nullptr;
        size_t cap = 0;
    };
    Buf qbytes, tbytes, qoff, toff, score, tb, slots, cstart, clen, dst_off, dst;
    // Traceback-code and pass-boundary workspace, shared by every plan of this
    // context and grown at execute time (a plan's chunks are sized by its
    // budget): plans of one context must not execute concurrently.
    Buf ws_ptrs, ws_bnd;
    // Second traceback-code buffer for ta_plan_execute_batches: batch k+1's
    // fill writes one while batch k's traceback reads the other.
    Buf ws_ptrs2;
    hipEvent_t ev_fill = nullptr, ev_slot[2] = {nullptr, nullptr};
    uint32_t cu_count = 256;
    uint32_t epoch = 0;  // flexible-fill launches so far (tags of their pass hand-off records)
};
