// bioinfo1_amd/csrc/ta_host_batch.h -- the host-memory batch driver shared by
// ta_align_batch (linear gap) and ta_align_batch_affine: host arrays in, host
// arrays out, no device allocation or free per call once the context's
// grow-only buffers are large enough.
//
// Per call: the plan's per-pair arrays, the offsets and (up to 4 MB) the
// sequences are packed into pinned staging and go to the device in ONE copy
// (larger sequences follow in their own copies, from wherever the caller
// keeps them); the kernels run on the context's stream; the outputs come back
// in one copy when the CIGAR slots are small (the CIGARs are then packed on
// the host), else the records first and the CIGARs compacted on the device.
// team::Align's one-pair calls thus cost one H2D copy, the fill kernel (which
// walks its own pair), one D2H copy and one stream synchronisation.
#pragma once

#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstring>
#include <string>

#include "ta_context.h"
#include "ta_internal.h"
#include "ta_planner.h"

namespace ta_host {

// A plan as the batch driver needs it.
struct HostPlan {
    virtual ~HostPlan() = default;
    virtual void layout(ta::BlockLayout& L) = 0;              // arrays copied from the host
    virtual void pack(uint8_t* base) = 0;                     // write them at their offsets
    virtual void layout_device_only(ta::BlockLayout& L) = 0;  // device scratch of the plan
    virtual void bind(uint8_t* dev) = 0;                      // point the plan at the device block
    virtual int execute(const ta_device_io* io, hipStream_t s) = 0;
    virtual uint64_t slots_bytes() const = 0;
    virtual uint64_t err_offset() const = 0;  // offset of the kernels' error word in the block, or UINT64_MAX
    virtual const char* err_message(uint32_t err) const = 0;  // the error word's meaning
};

constexpr uint64_t kPackSeqLimit = 4ull << 20;  // sequences up to this travel inside the pinned block
constexpr uint64_t kSmallSlots = 4ull << 20;    // CIGAR slots up to this come back whole (no compaction)

// Code-workspace budget of a host batch: everything in one chunk when the
// codes take at most 1 GiB (no device query per call), else the default.
inline uint64_t batch_budget(const ta_context* ctx, uint32_t n_pairs, const uint32_t* qlen, const uint32_t* tlen,
                             int want_cigar, uint64_t bytes_per_entry) {
    if (!want_cigar) return 1ull << 30;
    const uint64_t need = ta::host_batch_code_bytes(n_pairs, qlen, tlen, bytes_per_entry);
    return need <= (1ull << 30) ? std::max<uint64_t>(need, 1) : default_budget(ctx);
}

// Argument checks shared by the two host-memory batch entries; sets the input extents.
inline int check_host_batch(ta_context* ctx, int type, uint32_t n_pairs, const char* qb, const uint64_t* qoff,
                            const uint32_t* qlen, const char* tbytes, const uint64_t* toff, const uint32_t* tlen,
                            int want_cigar, char* arena, uint64_t* cigar_off, uint32_t* cigar_len, uint64_t* qend,
                            uint64_t* tend) {
    if (!ctx) return TA_ERR_ARG;
    if (type != TA_GLOBAL && type != TA_LOCAL && type != TA_SEMI_GLOBAL)
        return fail(ctx, TA_ERR_BAD_TYPE, ta_status_string(TA_ERR_BAD_TYPE));
    if (n_pairs == 0) return TA_OK;
    if (!qoff || !qlen || !toff || !tlen) return fail(ctx, TA_ERR_ARG, "null input array");
    if (want_cigar && (!arena || !cigar_off || !cigar_len)) return fail(ctx, TA_ERR_ARG, "null cigar output");
    *qend = *tend = 0;
    for (uint32_t p = 0; p < n_pairs; ++p) {
        *qend = std::max<uint64_t>(*qend, qoff[p] + qlen[p]);
        *tend = std::max<uint64_t>(*tend, toff[p] + tlen[p]);
    }
    if ((*qend && !qb) || (*tend && !tbytes)) return fail(ctx, TA_ERR_ARG, "null sequence bytes");
    return TA_OK;
}

// After the first enqueue an early return (a failed HIP call or plan execute)
// must not leave work in flight on the context's stream: the next call packs
// its inputs into the same pinned staging that an unfinished upload may still
// read.  The guard drains the stream and records the context's last event.
struct StreamGuard {
    ta_context* ctx;
    hipStream_t s;
    bool armed = true;
    ~StreamGuard() {
        if (!armed) return;
        (void)hipStreamSynchronize(s);
        if (hipEventRecord(ctx->ev_last, s) == hipSuccess) {
            ctx->last_stream = s;
            ctx->used = true;
        }
    }
};

// Called with ctx->mu held.
inline int host_batch(ta_context* ctx, HostPlan& hp, uint32_t n_pairs, const char* qb, const uint64_t* qoff,
                      const uint32_t* qlen, const char* tbytes, const uint64_t* toff, const uint32_t* tlen,
                      uint64_t qend, uint64_t tend, int want_cigar, int32_t* score, uint32_t* target_begin,
                      char* arena, uint64_t arena_bytes, uint64_t* cigar_off, uint32_t* cigar_len) {
    (void)qlen;
    (void)tlen;
    if (int r = lazy_stream(ctx, ctx->stream)) return r;
    hipStream_t s = ctx->stream;
    const uint64_t P = n_pairs;
    // ---- inputs: plan arrays + offsets (+ small sequences) in one pinned block
    ta::BlockLayout L;
    hp.layout(L);
    const uint64_t o_qoff = L.add(P * 8), o_toff = L.add(P * 8);
    const bool pack_seq = qend + tend <= kPackSeqLimit;
    const uint64_t o_qb = L.add(qend), o_tb = L.add(tend);
    const uint64_t upload = pack_seq ? L.bytes : o_qb;
    hp.layout_device_only(L);
    if (int r = grow(ctx, ctx->blk, L.bytes)) return r;
    if (int r = grow_pinned(ctx, ctx->pin_in, upload)) return r;
    uint8_t* hin = static_cast<uint8_t*>(ctx->pin_in.p);
    uint8_t* d = static_cast<uint8_t*>(ctx->blk.p);
    hp.pack(hin);
    std::memcpy(hin + o_qoff, qoff, P * 8);
    std::memcpy(hin + o_toff, toff, P * 8);
    if (pack_seq) {
        if (qend) std::memcpy(hin + o_qb, qb, qend);
        if (tend) std::memcpy(hin + o_tb, tbytes, tend);
    }
    if (int r = stream_enter(ctx, s)) return r;
    StreamGuard guard{ctx, s};
    roctxRangePushA("ta upload");
    TA_HIP(ctx, hipMemcpyAsync(d, hin, upload, hipMemcpyHostToDevice, s));
    if (!pack_seq) {  // pinned or pageable caller memory: HIP picks the path
        if (qend) TA_HIP(ctx, hipMemcpyAsync(d + o_qb, qb, qend, hipMemcpyHostToDevice, s));
        if (tend) TA_HIP(ctx, hipMemcpyAsync(d + o_tb, tbytes, tend, hipMemcpyHostToDevice, s));
    }
    roctxRangePop();
    hp.bind(d);
    // ---- outputs: records, then the CIGAR slots
    const uint64_t slots = want_cigar ? hp.slots_bytes() : 0;
    ta::BlockLayout O;
    const uint64_t o_sc = O.add(P * 4), o_tbg = O.add(P * 4), o_cl = O.add(P * 4), o_cs = O.add(P * 8);
    const uint64_t o_sl = O.add(slots);
    if (int r = grow(ctx, ctx->out, O.bytes)) return r;
    uint8_t* dout = static_cast<uint8_t*>(ctx->out.p);
    ta_device_io io{};
    io.query_bytes = reinterpret_cast<const char*>(d + o_qb);
    io.query_off = reinterpret_cast<const uint64_t*>(d + o_qoff);
    io.target_bytes = reinterpret_cast<const char*>(d + o_tb);
    io.target_off = reinterpret_cast<const uint64_t*>(d + o_toff);
    io.score = reinterpret_cast<int32_t*>(dout + o_sc);
    io.target_begin = reinterpret_cast<uint32_t*>(dout + o_tbg);
    io.cigar_len = reinterpret_cast<uint32_t*>(dout + o_cl);
    io.cigar_start = reinterpret_cast<uint64_t*>(dout + o_cs);
    io.cigar_slots = reinterpret_cast<char*>(dout + o_sl);
    if (int r = hp.execute(&io, s)) return r;
    const bool whole = !want_cigar || slots <= kSmallSlots;
    const uint64_t down = whole ? O.bytes : o_sl;
    const uint64_t err_off = hp.err_offset();
    if (int r = grow_pinned(ctx, ctx->pin_out, down + 256)) return r;
    uint8_t* hout = static_cast<uint8_t*>(ctx->pin_out.p);
    roctxRangePushA("ta download");
    TA_HIP(ctx, hipMemcpyAsync(hout, dout, down, hipMemcpyDeviceToHost, s));
    if (err_off != UINT64_MAX) TA_HIP(ctx, hipMemcpyAsync(hout + down, d + err_off, 4, hipMemcpyDeviceToHost, s));
    TA_HIP(ctx, hipStreamSynchronize(s));
    roctxRangePop();
    if (int r = stream_leave(ctx, s)) return r;
    guard.armed = false;  // drained and recorded (the compaction below synchronises itself)
    if (err_off != UINT64_MAX) {
        uint32_t err = 0;
        std::memcpy(&err, hout + down, 4);
        if (err) return fail(ctx, TA_ERR_DEVICE, hp.err_message(err));
    }
    if (want_cigar) {
        const uint32_t* cl = reinterpret_cast<const uint32_t*>(hout + o_cl);
        uint64_t total = 0;
        for (uint64_t p = 0; p < P; ++p) {
            cigar_off[p] = total;
            total += cl[p];
        }
        if (total > arena_bytes) return fail(ctx, TA_ERR_CAPACITY, "cigar arena too small");
        std::memcpy(cigar_len, cl, P * 4);
        if (whole) {
            const uint64_t* cs = reinterpret_cast<const uint64_t*>(hout + o_cs);
            for (uint64_t p = 0; p < P; ++p) std::memcpy(arena + cigar_off[p], hout + o_sl + cs[p], cl[p]);
        } else {
            // compaction on the device: offsets up through pinned staging (its upload is done)
            if (int r = grow_pinned(ctx, ctx->pin_in, P * 8)) return r;
            std::memcpy(ctx->pin_in.p, cigar_off, P * 8);
            if (int r = grow(ctx, ctx->dst, total + P * 8 + 256)) return r;
            uint8_t* dd = static_cast<uint8_t*>(ctx->dst.p);
            const uint64_t o_dst = (P * 8 + 255) & ~uint64_t(255);
            guard.armed = true;
            TA_HIP(ctx, hipMemcpyAsync(dd, ctx->pin_in.p, P * 8, hipMemcpyHostToDevice, s));
            ta::CompactArgs ca{n_pairs, io.cigar_slots, io.cigar_start, io.cigar_len,
                               reinterpret_cast<const uint64_t*>(dd), reinterpret_cast<char*>(dd + o_dst)};
            TA_HIP(ctx, ta::launch_compact(ca, s));
            TA_HIP(ctx, hipMemcpyAsync(arena, dd + o_dst, total, hipMemcpyDeviceToHost, s));
            TA_HIP(ctx, hipStreamSynchronize(s));
            guard.armed = false;
        }
    }
    if (score) std::memcpy(score, hout + o_sc, P * 4);
    if (target_begin) std::memcpy(target_begin, hout + o_tbg, P * 4);
    return TA_OK;
}

}  // namespace ta_host
