// bioinfo1_amd/csrc/ta_api.hip -- host side of the extern "C" ABI
// (include/team_align_c.h): contexts, batch plans, workspace layout, chunking
// and the host-memory batch entry point.  The DP itself is in ta_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/team_align_c.h"
#include "ta_context.h"
#include "ta_internal.h"

struct ta_plan {
    ta_context* ctx = nullptr;
    uint32_t n_pairs = 0;
    int type = 0, match = 0, mismatch = 0, gap = 0;
    bool want_cigar = false, wide = false;
    // Traceback inside the fill kernel (TA_FUSED_TRACEBACK=0 disables).  Only
    // for plans without dual couples: a dual wave would walk its two pairs one
    // after the other, all waves at once after the fill; the separate
    // traceback kernel walks every pair on its own wave (measured faster).
    bool fused = true;
    bool dual = true;   // packed two-pair int16 fill where it fits (TA_DUAL=0 disables)
    bool flex = true;   // ... also for couples of different shapes / long pairs (TA_FLEX=0 disables)
    bool staged = false;  // chunks use disjoint workspace: traceback k overlaps fill k+1
    std::vector<uint32_t> qlen, tlen, order, singles, duals, flexes;
    std::vector<uint32_t> flex_task_off;  // per flex couple: first task (one per query pass); + total
    // per chunk, the chunk's tasks in ticket order: pass-major (every couple's pass 0, then every
    // pass 1, ...), so a pass starts long after its predecessor instead of trailing it by a chunk
    std::vector<uint32_t> flex_tasks;
    std::vector<uint64_t> slot_off;
    struct Chunk {
        uint32_t begin, count;    // all pairs (traceback order)
        uint32_t sbegin, scount;  // int32 fill: pairs
        uint32_t dbegin, dcount;  // dual fill: pair couples
        uint32_t fbegin, fcount;  // flexible dual fill: pair couples
        uint32_t cbegin;          // couples (dual + flex) before this chunk: its slice of the fallback list
        uint64_t ptr_dwords, bnd_words;
    };
    uint32_t n_dual_pairs = 0;
    std::vector<Chunk> chunks;
    uint64_t slots_bytes = 0, ws_ptr_dwords = 0, ws_bnd_words = 0;
    // device
    uint32_t *d_qlen = nullptr, *d_tlen = nullptr, *d_order = nullptr, *d_singles = nullptr, *d_duals = nullptr,
             *d_flexes = nullptr;
    uint64_t *d_ptr_off = nullptr, *d_bnd_off = nullptr, *d_slot_off = nullptr;
    uint32_t *d_goal_i = nullptr, *d_goal_j = nullptr;
    uint32_t* d_fb = nullptr;  // dual fallback: [n_dual_pairs] list, then one counter per chunk
    uint32_t *d_flex_task_off = nullptr, *d_tickets = nullptr, *d_err = nullptr, *d_flex_tasks = nullptr;
    void* d_pout = nullptr;  // PassOut[2] per flex task
};

namespace {

int fail(ta_context* ctx, int code, const std::string& msg) {
    if (ctx) ctx->last_error = msg;
    return code;
}

#define TA_HIP(ctx, expr)                                                                            \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess)                                                                        \
            return fail((ctx), TA_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

bool valid_type(int t) { return t == TA_GLOBAL || t == TA_LOCAL || t == TA_SEMI_GLOBAL; }

// Workspace budget when the caller passes 0: TA_WORKSPACE_BYTES, else 85 % of
// what is free on the device (counting the context's cached workspace), so
// long-read batches run in as few chunks as HBM allows (fewer, fuller
// launches: one wave per pair needs thousands of pairs per chunk).
uint64_t default_budget(const ta_context* ctx) {
    if (const char* e = std::getenv("TA_WORKSPACE_BYTES")) return std::strtoull(e, nullptr, 10);
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return 48ull << 30;
    const uint64_t avail = (uint64_t)free_b + ctx->ws_ptrs.cap + ctx->ws_bnd.cap + ctx->ws_ptrs2.cap;
    return std::max<uint64_t>(avail / 100 * 85, 1ull << 30);
}

int grow(ta_context* ctx, ta_context::Buf& b, size_t bytes) {
    if (bytes <= b.cap) return TA_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    size_t want = std::max<size_t>(bytes, 4096);
    TA_HIP(ctx, hipMalloc(&b.p, want));
    b.cap = want;
    return TA_OK;
}

template <class T>
int upload(ta_context* ctx, T** dptr, const std::vector<T>& v) {
    if (v.empty()) return TA_OK;
    TA_HIP(ctx, hipMalloc(reinterpret_cast<void**>(dptr), v.size() * sizeof(T)));
    TA_HIP(ctx, hipMemcpy(*dptr, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return TA_OK;
}

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
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->aux2, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->tbs, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_tb_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_join2, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fill, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_slot[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_slot[1], hipEventDisableTiming) != hipSuccess) {
        delete c;
        return TA_ERR_DEVICE;
    }
    *out = c;
    return TA_OK;
}

void ta_context_destroy(ta_context* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    for (auto* b : {&ctx->qbytes, &ctx->tbytes, &ctx->qoff, &ctx->toff, &ctx->score, &ctx->tb, &ctx->slots,
                    &ctx->cstart, &ctx->clen, &ctx->dst_off, &ctx->dst, &ctx->ws_ptrs, &ctx->ws_bnd, &ctx->ws_ptrs2})
        if (b->p) (void)hipFree(b->p);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
    if (ctx->aux2) (void)hipStreamDestroy(ctx->aux2);
    if (ctx->tbs) (void)hipStreamDestroy(ctx->tbs);
    if (ctx->ev_tb_done) (void)hipEventDestroy(ctx->ev_tb_done);
    for (hipEvent_t e : ctx->ev_stage) (void)hipEventDestroy(e);
    if (ctx->ev_join2) (void)hipEventDestroy(ctx->ev_join2);
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
    for (hipEvent_t e : {ctx->ev_fill, ctx->ev_slot[0], ctx->ev_slot[1]})
        if (e) (void)hipEventDestroy(e);
    delete ctx;
}

void ta_plan_destroy(ta_plan* pl) {
    if (!pl) return;
    (void)hipSetDevice(pl->ctx->device);
    for (void* p : {(void*)pl->d_qlen, (void*)pl->d_tlen, (void*)pl->d_order, (void*)pl->d_singles, (void*)pl->d_duals, (void*)pl->d_flexes, (void*)pl->d_ptr_off,
                    (void*)pl->d_bnd_off, (void*)pl->d_slot_off, (void*)pl->d_goal_i, (void*)pl->d_goal_j,
                    (void*)pl->d_fb, (void*)pl->d_flex_task_off, (void*)pl->d_tickets, (void*)pl->d_err, pl->d_pout,
                    (void*)pl->d_flex_tasks})
        if (p) (void)hipFree(p);
    delete pl;
}

int ta_plan_create(ta_context* ctx, uint32_t n_pairs, const uint32_t* qlen, const uint32_t* tlen, int type,
                   int match, int mismatch, int gap, int want_cigar, uint64_t budget, ta_plan** out) {
    if (!ctx || !out || (n_pairs && (!qlen || !tlen))) return fail(ctx, TA_ERR_ARG, "null argument");
    *out = nullptr;
    if (!valid_type(type)) return fail(ctx, TA_ERR_BAD_TYPE, ta_status_string(TA_ERR_BAD_TYPE));
    TA_HIP(ctx, hipSetDevice(ctx->device));
    auto* pl = new ta_plan();
    pl->ctx = ctx;
    pl->n_pairs = n_pairs;
    pl->type = type;
    pl->match = match;
    pl->mismatch = mismatch;
    pl->gap = gap;
    pl->want_cigar = want_cigar != 0;
    if (const char* e = std::getenv("TA_FUSED_TRACEBACK")) pl->fused = std::atoi(e) != 0;
    pl->qlen.assign(qlen, qlen + n_pairs);
    pl->tlen.assign(tlen, tlen + n_pairs);
    // Local mode keeps V = 32*score + row tag in int32; take the unscaled
    // ("wide") kernel when any local value could reach 2^25 in magnitude.
    uint64_t maxlen = 0;
    for (uint32_t p = 0; p < n_pairs; ++p) maxlen = std::max<uint64_t>(maxlen, (uint64_t)qlen[p] + tlen[p]);
    const uint64_t mag = std::max<uint64_t>({1ull, (uint64_t)std::llabs(match), (uint64_t)std::llabs(mismatch),
                                             (uint64_t)std::llabs(gap)});
    pl->wide = (type == TA_LOCAL) && (maxlen * mag >= (1ull << 25));
    if (const char* e = std::getenv("TA_DUAL")) pl->dual = std::atoi(e) != 0;
    // Longest pairs first (fewer stragglers); equal shapes adjacent so they
    // can be coupled for the two-pair kernel.
    pl->order.resize(n_pairs);
    std::iota(pl->order.begin(), pl->order.end(), 0u);
    std::stable_sort(pl->order.begin(), pl->order.end(), [&](uint32_t a, uint32_t b) {
        const uint64_t ca = (uint64_t)pl->qlen[a] * pl->tlen[a], cb = (uint64_t)pl->qlen[b] * pl->tlen[b];
        if (ca != cb) return ca > cb;
        return pl->qlen[a] != pl->qlen[b] ? pl->qlen[a] > pl->qlen[b] : pl->tlen[a] > pl->tlen[b];
    });
    if (budget == 0) budget = default_budget(ctx);
    const uint64_t budget_dw = std::max<uint64_t>(budget / 4, 1);
    std::vector<uint64_t> ptr_off(n_pairs, 0), bnd_off(n_pairs, 0);
    pl->slot_off.assign(n_pairs, 0);
    uint64_t so = 0;
    for (uint32_t p = 0; p < n_pairs; ++p) {
        pl->slot_off[p] = so;
        so += ta::cigar_slot_bytes(pl->qlen[p], pl->tlen[p]);
    }
    pl->slots_bytes = so;
    if (const char* e = std::getenv("TA_FLEX")) pl->flex = std::atoi(e) != 0;
    // Work units: one pair (int32 fill), an equal-shape couple (dual fill) or
    // a couple of different shapes (flexible dual fill), then longest first.
    struct Unit {
        int kind;  // 0 single, 1 dual, 2 flex
        uint32_t a, b;
        uint64_t cost;  // cells one wave sweeps
    };
    std::vector<Unit> units;
    std::vector<uint32_t> rest;
    const bool flex_ok = pl->dual && pl->flex && ta::flex_fits(type, match, mismatch, gap);
    for (uint32_t k = 0; k < n_pairs;) {
        const uint32_t p = pl->order[k];
        const uint32_t n = pl->qlen[p], m = pl->tlen[p];
        // (equal shapes within int16 stay on the dual fill even when multi-pass: measured faster
        // than the pipelined flexible fill on config 5, 4,056 vs 3,765 GCUPS)
        const bool couple = pl->dual && k + 1 < n_pairs && pl->qlen[pl->order[k + 1]] == n &&
                            pl->tlen[pl->order[k + 1]] == m && ta::fits_int16(type, n, m, match, mismatch, gap);
        if (couple) {
            units.push_back({1, p, pl->order[k + 1], (uint64_t)n * m});
            k += 2;
        } else {
            rest.push_back(p);
            ++k;
        }
    }
    if (flex_ok) {
        // flexible couples: same pass count and n mod 16 (same rows in the last
        // lane), neighbours by (n, m), at most 25 % of the wave's cells wasted
        std::vector<uint32_t> cand;
        for (uint32_t p : rest) {
            if (pl->qlen[p] && pl->tlen[p]) cand.push_back(p);
            else units.push_back({0, p, p, (uint64_t)pl->qlen[p] * pl->tlen[p]});
        }
        auto key = [&](uint32_t p) { return ((uint64_t)ta::n_passes(pl->qlen[p]) << 4) | (pl->qlen[p] & 15u); };
        std::stable_sort(cand.begin(), cand.end(), [&](uint32_t a, uint32_t b) {
            if (key(a) != key(b)) return key(a) < key(b);
            if (pl->qlen[a] != pl->qlen[b]) return pl->qlen[a] > pl->qlen[b];
            return pl->tlen[a] > pl->tlen[b];
        });
        for (size_t i = 0; i < cand.size();) {
            const uint32_t A = cand[i];
            if (i + 1 < cand.size() && key(cand[i + 1]) == key(A) && ta::n_passes(pl->qlen[A]) < 64) {
                const uint32_t B = cand[i + 1];
                const uint64_t M = std::max(pl->tlen[A], pl->tlen[B]);
                const uint64_t wave = (uint64_t)pl->qlen[A] * M;
                const uint64_t useful = (uint64_t)pl->qlen[A] * pl->tlen[A] + (uint64_t)pl->qlen[B] * pl->tlen[B];
                if (4 * useful >= 3 * 2 * wave) {  // waste <= 25 %
                    units.push_back({2, A, B, wave});
                    i += 2;
                    continue;
                }
            }
            const uint32_t ps = ta::n_passes(pl->qlen[A]);
            units.push_back({ps >= 4 && ps < 64 ? 2 : 0, A, A, (uint64_t)pl->qlen[A] * pl->tlen[A]});
            ++i;
        }
    } else {
        for (uint32_t p : rest) units.push_back({0, p, p, (uint64_t)pl->qlen[p] * pl->tlen[p]});
    }
    std::stable_sort(units.begin(), units.end(), [](const Unit& x, const Unit& y) { return x.cost > y.cost; });
    pl->order.clear();
    // Staging: when the whole plan's codes fit the budget and the traceback runs
    // as its own kernel (packed couples), cut it into TA_STAGES chunks with
    // disjoint workspace, so stage k's traceback (SALU-bound) runs on a stream
    // of its own beside stage k+1's fill (VALU-bound).
    uint64_t total_pd = 0;
    bool any_couple = false;
    for (const Unit& u : units) {
        total_pd += !pl->want_cigar ? 0 : ta::ptr_dwords(pl->qlen[u.a], pl->tlen[u.a]) +
                                             (u.kind ? ta::ptr_dwords(pl->qlen[u.b], pl->tlen[u.b]) : 0);
        any_couple |= u.kind != 0;
    }
    uint32_t stages = 1;  // off by default: a quarter-size fill launch runs far below the full one (r01l: 2 stages 2,267 vs 2,812 GCUPS)
    if (const char* e = std::getenv("TA_STAGES")) stages = (uint32_t)std::max(1, std::atoi(e));
    pl->staged = pl->want_cigar && any_couple && total_pd <= budget_dw && stages > 1 && units.size() >= 8ull * stages;
    const size_t per_stage = pl->staged ? (units.size() + stages - 1) / stages : units.size();
    ta_plan::Chunk cur{};
    uint32_t couples_before = 0;
    uint64_t off_pd = 0, off_bw = 0;  // running offsets (reset per chunk unless staged)
    auto open_chunk = [&]() {
        cur = ta_plan::Chunk{(uint32_t)pl->order.size(), 0, (uint32_t)pl->singles.size(), 0,
                             (uint32_t)(pl->duals.size() / 2), 0, (uint32_t)(pl->flexes.size() / 2), 0,
                             couples_before, 0, 0};
        if (!pl->staged) off_pd = off_bw = 0;
    };
    open_chunk();
    for (size_t k = 0; k < units.size(); ++k) {
        const Unit& u = units[k];
        const uint32_t na = pl->qlen[u.a], ma = pl->tlen[u.a], nb = pl->qlen[u.b], mb = pl->tlen[u.b];
        const uint64_t pd = !pl->want_cigar ? 0 : ta::ptr_dwords(na, ma) + (u.kind && u.a != u.b ? ta::ptr_dwords(nb, mb) : 0);
        if (cur.count && (pl->staged ? k % per_stage == 0 : cur.ptr_dwords + pd > budget_dw)) {
            pl->chunks.push_back(cur);
            open_chunk();
        }
        const uint32_t q[2] = {u.a, u.b};
        const int halves = (u.kind && u.a != u.b) ? 2 : 1;
        for (int h = 0; h < halves; ++h) {
            const uint32_t x = q[h];
            ptr_off[x] = off_pd;
            bnd_off[x] = off_bw;
            const uint64_t xd = pl->want_cigar ? ta::ptr_dwords(pl->qlen[x], pl->tlen[x]) : 0;
            // flex: pair A holds both pairs' absolute int32 boundary rows, interleaved;
            // each pair keeps a region of its own for the int32 fallback ('-' in a query)
            uint64_t bw = ta::bnd_words(pl->qlen[x], pl->tlen[x]);
            if (u.kind == 2 && h == 0 && ta::n_passes(na) > 1)
                bw = std::max<uint64_t>(bw, 8ull * ((uint64_t)std::max(ma, mb) + 1));
            bw += bw & 1;  // keep every region 8-byte aligned (64-bit hand-off records)
            off_pd += xd;
            off_bw += bw;
            cur.ptr_dwords += xd;
            cur.bnd_words += bw;
            pl->order.push_back(x);
        }
        if (u.kind == 1) {
            pl->duals.push_back(u.a);
            pl->duals.push_back(u.b);
            ++cur.dcount;
        } else if (u.kind == 2) {
            pl->flexes.push_back(u.a);
            pl->flexes.push_back(u.b);
            ++cur.fcount;
        } else {
            pl->singles.push_back(u.a);
            ++cur.scount;
        }
        if (u.kind) {
            pl->n_dual_pairs += 2;
            ++couples_before;
        }
        cur.count += (u.kind && u.a != u.b) ? 2 : 1;
    }
    if (cur.count) pl->chunks.push_back(cur);
    if (pl->n_dual_pairs) pl->fused = false;
    pl->flex_task_off.assign(1, 0);
    for (size_t w = 0; w < pl->flexes.size() / 2; ++w)
        pl->flex_task_off.push_back(pl->flex_task_off.back() + ta::n_passes(pl->qlen[pl->flexes[2 * w]]));
    pl->flex_tasks.assign(pl->flex_task_off.back(), 0u);
    for (const auto& ch : pl->chunks) {
        uint32_t at = pl->flex_task_off[ch.fbegin], maxp = 0;
        for (uint32_t w = ch.fbegin; w < ch.fbegin + ch.fcount; ++w)
            maxp = std::max(maxp, pl->flex_task_off[w + 1] - pl->flex_task_off[w]);
        for (uint32_t ps = 0; ps < maxp; ++ps)
            for (uint32_t w = ch.fbegin; w < ch.fbegin + ch.fcount; ++w)
                if (pl->flex_task_off[w + 1] - pl->flex_task_off[w] > ps) pl->flex_tasks[at++] = w * 64u + ps;
    }
    if (pl->staged) {
        pl->ws_ptr_dwords = off_pd;
        pl->ws_bnd_words = off_bw;
    } else {
        for (auto& c : pl->chunks) {
            pl->ws_ptr_dwords = std::max(pl->ws_ptr_dwords, c.ptr_dwords);
            pl->ws_bnd_words = std::max(pl->ws_bnd_words, c.bnd_words);
        }
    }
    int rc = TA_OK;
    auto up = [&](int r) {
        if (r != TA_OK && rc == TA_OK) rc = r;
    };
    up(upload(ctx, &pl->d_qlen, pl->qlen));
    up(upload(ctx, &pl->d_tlen, pl->tlen));
    up(upload(ctx, &pl->d_order, pl->order));
    up(upload(ctx, &pl->d_singles, pl->singles));
    up(upload(ctx, &pl->d_duals, pl->duals));
    up(upload(ctx, &pl->d_flexes, pl->flexes));
    if (!pl->flexes.empty()) {
        up(upload(ctx, &pl->d_flex_task_off, pl->flex_task_off));
        up(upload(ctx, &pl->d_flex_tasks, pl->flex_tasks));
        up(upload(ctx, &pl->d_tickets, std::vector<uint32_t>(pl->chunks.size(), 0u)));
        up(upload(ctx, &pl->d_err, std::vector<uint32_t>(1, 0u)));
        if (rc == TA_OK && hipMalloc(&pl->d_pout, pl->flex_task_off.back() * 48ull + 16) != hipSuccess)
            rc = fail(ctx, TA_ERR_DEVICE, "hipMalloc flex pass results");
    }
    up(upload(ctx, &pl->d_ptr_off, ptr_off));
    up(upload(ctx, &pl->d_bnd_off, bnd_off));
    up(upload(ctx, &pl->d_slot_off, pl->slot_off));
    if (rc == TA_OK && n_pairs) {
        // two halves: ta_plan_execute_batches alternates them between batches
        if (hipMalloc(&pl->d_goal_i, 2 * n_pairs * 4ull) != hipSuccess ||
            hipMalloc(&pl->d_goal_j, 2 * n_pairs * 4ull) != hipSuccess)
            rc = fail(ctx, TA_ERR_DEVICE, "hipMalloc goal");
    }
    if (rc == TA_OK && pl->n_dual_pairs &&
        hipMalloc(&pl->d_fb, (pl->n_dual_pairs + pl->chunks.size()) * 4ull) != hipSuccess)
        rc = fail(ctx, TA_ERR_DEVICE, "hipMalloc dual fallback list");
    if (rc != TA_OK) {
        ta_plan_destroy(pl);
        return rc;
    }
    *out = pl;
    return TA_OK;
}

uint64_t ta_plan_cigar_slots_bytes(const ta_plan* pl) { return pl ? pl->slots_bytes : 0; }
uint64_t ta_plan_workspace_bytes(const ta_plan* pl) {
    return pl ? (pl->ws_ptr_dwords + pl->ws_bnd_words) * 4ull : 0;
}
uint32_t ta_plan_chunks(const ta_plan* pl) { return pl ? (uint32_t)pl->chunks.size() : 0; }
uint32_t ta_plan_dual_pairs(const ta_plan* pl) { return pl ? pl->n_dual_pairs : 0; }
uint32_t ta_plan_flex_pairs(const ta_plan* pl) { return pl ? (uint32_t)pl->flexes.size() : 0; }

// slot 1 = the second code buffer and goal half (ta_plan_execute_batches);
// tb_waves > 0 caps the traceback grid.
static int exec_chunk(ta_plan* pl, const ta_device_io* io, hipStream_t s, uint32_t c, bool fill, bool trace,
                      int slot = 0, uint32_t tb_waves = 0) {
    const auto& ch = pl->chunks[c];
    ta_context* ctx = pl->ctx;
    ta_context::Buf& ws = slot ? ctx->ws_ptrs2 : ctx->ws_ptrs;
    if (pl->ws_ptr_dwords)
        if (int r = grow(ctx, ws, pl->ws_ptr_dwords * 4ull)) return r;
    if (pl->ws_bnd_words)
        if (int r = grow(ctx, ctx->ws_bnd, pl->ws_bnd_words * 4ull)) return r;
    uint32_t* d_ptrs = static_cast<uint32_t*>(ws.p);
    uint32_t* goal_i = pl->d_goal_i + (slot ? pl->n_pairs : 0);
    uint32_t* goal_j = pl->d_goal_j + (slot ? pl->n_pairs : 0);
    int32_t* d_bnd = static_cast<int32_t*>(ctx->ws_bnd.p);
    if (fill) {
        // The flexible fill's pass hand-off records live in this buffer and are
        // recognised by their tag alone, so whatever an earlier user of the
        // memory left there (traceback codes of a freed workspace, other
        // plans' records) must not survive: zero it (tag 0 is never valid)
        // before any kernel of this chunk is enqueued.
        if (ch.fcount && pl->ws_bnd_words) TA_HIP(ctx, hipMemsetAsync(d_bnd, 0, pl->ws_bnd_words * 4ull, s));
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
        a.match = pl->match;
        a.mismatch = pl->mismatch;
        a.gap = pl->gap;
        a.ptrs = d_ptrs;
        a.ptr_off = pl->d_ptr_off;
        a.bnd = d_bnd;
        a.bnd_off = pl->d_bnd_off;
        a.score = io->score;
        a.target_begin = io->target_begin;
        a.goal_i = goal_i;
        a.goal_j = goal_j;
        a.fused = (pl->fused && pl->want_cigar) ? 1 : 0;
        a.slots = io->cigar_slots;
        a.slot_off = pl->d_slot_off;
        a.cigar_start = io->cigar_start;
        a.cigar_len = io->cigar_len;
        if (ch.scount) {  // launched first: it may run on the aux stream beside the packed fill
            ta::FillArgs a1 = a;
            a1.order = pl->d_singles;
            a1.begin = ch.sbegin;
            a1.count = ch.scount;
            if (ch.dcount || ch.fcount) {  // beside the packed fill: fork onto the aux stream, join below
                TA_HIP(ctx, hipEventRecord(ctx->ev_fork, s));
                TA_HIP(ctx, hipStreamWaitEvent(ctx->aux, ctx->ev_fork, 0));
                TA_HIP(ctx, ta::launch_fill(pl->type, pl->want_cigar, pl->wide, a1, ctx->aux));
            } else {
                TA_HIP(ctx, ta::launch_fill(pl->type, pl->want_cigar, pl->wide, a1, s));
            }
        }
        if (ch.dcount || ch.fcount) {
            uint32_t* fb_list = pl->d_fb + 2ull * ch.cbegin;
            uint32_t* fb_count = pl->d_fb + pl->n_dual_pairs + c;
            TA_HIP(pl->ctx, hipMemsetAsync(fb_count, 0, 4, s));
            if (ch.dcount) {
                ta::FillArgs d = a;
                d.order = pl->d_duals;
                d.begin = ch.dbegin;
                d.count = ch.dcount;
                d.fb_list = fb_list;
                d.fb_count = fb_count;
                if (ch.fcount) {  // beside the flexible fill: fork onto aux2 (after the counter reset), join below
                    TA_HIP(ctx, hipEventRecord(ctx->ev_fork, s));
                    TA_HIP(ctx, hipStreamWaitEvent(ctx->aux2, ctx->ev_fork, 0));
                    TA_HIP(ctx, ta::launch_dual(pl->type, pl->want_cigar, d, ctx->aux2));
                    TA_HIP(ctx, hipEventRecord(ctx->ev_join2, ctx->aux2));
                } else {
                    TA_HIP(ctx, ta::launch_dual(pl->type, pl->want_cigar, d, s));
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
                d.n_tasks = pl->flex_task_off[ch.fbegin + ch.fcount] - pl->flex_task_off[ch.fbegin];
                d.epoch = ++ctx->epoch & 0x3FFFFFFu;
                d.err = pl->d_err;
                d.pout = pl->d_pout;
                TA_HIP(ctx, hipMemsetAsync(d.ticket, 0, 4, s));
                TA_HIP(pl->ctx, ta::launch_flex(pl->type, pl->want_cigar, d, s));
            }
            if (ch.dcount && ch.fcount) TA_HIP(ctx, hipStreamWaitEvent(s, ctx->ev_join2, 0));
            // couples the packed kernels handed back ('-' in a query): int32
            // fill, wave count read on the device (grid sized for all of them)
            ta::FillArgs f = a;
            f.order = fb_list;
            f.begin = 0;
            f.count = 2 * (ch.dcount + ch.fcount);
            f.count_dev = fb_count;
            TA_HIP(pl->ctx, ta::launch_fill(pl->type, pl->want_cigar, pl->wide, f, s));
        }
        if (ch.scount && (ch.dcount || ch.fcount)) {  // join the aux stream
            TA_HIP(ctx, hipEventRecord(ctx->ev_join, ctx->aux));
            TA_HIP(ctx, hipStreamWaitEvent(s, ctx->ev_join, 0));
        }
    }
    if (trace && pl->want_cigar && !(fill && pl->fused)) {
        ta::TraceArgs t{};
        t.order = pl->d_order;
        t.begin = ch.begin;
        t.count = ch.count;
        t.qlen = pl->d_qlen;
        t.tlen = pl->d_tlen;
        t.ptrs = d_ptrs;
        t.ptr_off = pl->d_ptr_off;
        t.goal_i = goal_i;
        t.goal_j = goal_j;
        t.slots = io->cigar_slots;
        t.slot_off = pl->d_slot_off;
        t.cigar_start = io->cigar_start;
        t.cigar_len = io->cigar_len;
        t.score = io->score;
        t.qbytes = reinterpret_cast<const uint8_t*>(io->query_bytes);
        t.qoff = io->query_off;
        t.tbytes = reinterpret_cast<const uint8_t*>(io->target_bytes);
        t.toff = io->target_off;
        t.match = pl->match;
        t.mismatch = pl->mismatch;
        t.gap = pl->gap;
        TA_HIP(pl->ctx, ta::launch_traceback(pl->type, t, s, tb_waves));
    }
    return TA_OK;
}

static int check_io(ta_plan* pl, const ta_device_io* io) {
    if (!pl || !io) return TA_ERR_ARG;
    if (pl->n_pairs && (!io->query_off || !io->target_off || !io->score || !io->target_begin))
        return fail(pl->ctx, TA_ERR_ARG, "null device pointer");
    if (pl->want_cigar && pl->n_pairs && (!io->cigar_slots || !io->cigar_start || !io->cigar_len))
        return fail(pl->ctx, TA_ERR_ARG, "null cigar device pointer");
    return TA_OK;
}

int ta_plan_execute(ta_plan* pl, const ta_device_io* io, void* stream) {
    if (int r = check_io(pl, io)) return r;
    TA_HIP(pl->ctx, hipSetDevice(pl->ctx->device));
    hipStream_t s = (hipStream_t)stream;  // NULL = the HIP null stream
    ta_context* ctx = pl->ctx;
    if (!pl->staged) {
        for (uint32_t c = 0; c < pl->chunks.size(); ++c)
            if (int r = exec_chunk(pl, io, s, c, true, true)) return r;
        return TA_OK;
    }
    // fills back to back on the caller's stream; stage c's traceback on tbs once its fill is done
    while (ctx->ev_stage.size() < pl->chunks.size()) {
        hipEvent_t e = nullptr;
        TA_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->ev_stage.push_back(e);
    }
    TA_HIP(ctx, hipEventRecord(ctx->ev_fork, s));
    TA_HIP(ctx, hipStreamWaitEvent(ctx->tbs, ctx->ev_fork, 0));  // tracebacks after earlier work on s
    for (uint32_t c = 0; c < pl->chunks.size(); ++c) {
        if (int r = exec_chunk(pl, io, s, c, true, false)) return r;
        TA_HIP(ctx, hipEventRecord(ctx->ev_stage[c], s));
        TA_HIP(ctx, hipStreamWaitEvent(ctx->tbs, ctx->ev_stage[c], 0));
        if (int r = exec_chunk(pl, io, ctx->tbs, c, false, true)) return r;
    }
    TA_HIP(ctx, hipEventRecord(ctx->ev_tb_done, ctx->tbs));
    TA_HIP(ctx, hipStreamWaitEvent(s, ctx->ev_tb_done, 0));
    return TA_OK;
}

// Batches of one plan back to back with batch k's traceback (SALU-bound) on
// the context's traceback stream beside batch k+1's fill (VALU-bound) on the
// caller's stream.  Codes and goal cells alternate between two buffers; a fill
// waits only for the traceback that last read its buffer.  TA_TB_WAVES_PER_SIMD
// > 0 caps the traceback grid so it fits next to the fill's waves (dual fill:
// 5 waves x 88 VGPRs per SIMD, traceback 32 VGPRs); the last unit runs
// uncapped.  Default 0 (uncapped): on config 2 a capped traceback is
// latency-bound and starved of VALU issue by the fill, and ends after it
// (2 waves/SIMD: 3.88 ms per batch vs 3.44 unpipelined).
int ta_plan_execute_batches(ta_plan* pl, const ta_device_io* ios, uint32_t n_batches, void* stream) {
    if (!pl || (n_batches && !ios)) return TA_ERR_ARG;
    for (uint32_t b = 0; b < n_batches; ++b)
        if (int r = check_io(pl, ios + b)) return r;
    ta_context* ctx = pl->ctx;
    TA_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;  // NULL = the HIP null stream
    const uint32_t nc = (uint32_t)pl->chunks.size();
    const uint64_t units = (uint64_t)n_batches * nc;
    bool pipe = pl->want_cigar && !pl->fused && !pl->staged && units >= 2 && pl->ws_ptr_dwords;
    // both code buffers must fit; otherwise the batches run one after the other
    if (pipe && grow(ctx, ctx->ws_ptrs2, pl->ws_ptr_dwords * 4ull) != TA_OK) {
        pipe = false;
        (void)hipGetLastError();  // the failed allocation is not an error here
        ctx->last_error.clear();
    }
    if (!pipe) {
        for (uint32_t b = 0; b < n_batches; ++b)
            if (int r = ta_plan_execute(pl, ios + b, stream)) return r;
        return TA_OK;
    }
    uint32_t per_simd = 0;
    if (const char* e = std::getenv("TA_TB_WAVES_PER_SIMD")) per_simd = (uint32_t)std::max(0, std::atoi(e));
    const uint32_t cap = per_simd * 4u * ctx->cu_count;  // 0 = uncapped
    TA_HIP(ctx, hipEventRecord(ctx->ev_fork, s));
    TA_HIP(ctx, hipStreamWaitEvent(ctx->tbs, ctx->ev_fork, 0));  // tracebacks after earlier work on s
    for (uint64_t u = 0; u < units; ++u) {
        const int slot = (int)(u & 1);
        const uint32_t b = (uint32_t)(u / nc), c = (uint32_t)(u % nc);
        if (u >= 2) TA_HIP(ctx, hipStreamWaitEvent(s, ctx->ev_slot[slot], 0));  // unit u-2's traceback is done
        if (int r = exec_chunk(pl, ios + b, s, c, true, false, slot)) return r;
        TA_HIP(ctx, hipEventRecord(ctx->ev_fill, s));
        TA_HIP(ctx, hipStreamWaitEvent(ctx->tbs, ctx->ev_fill, 0));
        if (int r = exec_chunk(pl, ios + b, ctx->tbs, c, false, true, slot, u + 1 < units ? cap : 0)) return r;
        TA_HIP(ctx, hipEventRecord(ctx->ev_slot[slot], ctx->tbs));
    }
    TA_HIP(ctx, hipEventRecord(ctx->ev_tb_done, ctx->tbs));
    TA_HIP(ctx, hipStreamWaitEvent(s, ctx->ev_tb_done, 0));
    return TA_OK;
}

int ta_plan_check(ta_plan* pl) {
    if (!pl) return TA_ERR_ARG;
    if (!pl->d_err) return TA_OK;
    uint32_t err = 0;
    TA_HIP(pl->ctx, hipSetDevice(pl->ctx->device));
    TA_HIP(pl->ctx, hipMemcpy(&err, pl->d_err, 4, hipMemcpyDeviceToHost));
    if (!err) return TA_OK;
    TA_HIP(pl->ctx, hipMemset(pl->d_err, 0, 4));
    return fail(pl->ctx, TA_ERR_DEVICE, "flexible fill: a pass hand-off poll timed out; results of this plan are invalid");
}

int ta_plan_execute_fill(ta_plan* pl, const ta_device_io* io, void* stream, uint32_t chunk) {
    if (int r = check_io(pl, io)) return r;
    if (chunk >= pl->chunks.size()) return pl->n_pairs ? TA_ERR_ARG : TA_OK;
    hipStream_t s = (hipStream_t)stream;  // NULL = the HIP null stream
    return exec_chunk(pl, io, s, chunk, true, false);
}

int ta_plan_execute_traceback(ta_plan* pl, const ta_device_io* io, void* stream, uint32_t chunk) {
    if (int r = check_io(pl, io)) return r;
    if (chunk >= pl->chunks.size()) return pl->n_pairs ? TA_ERR_ARG : TA_OK;
    hipStream_t s = (hipStream_t)stream;  // NULL = the HIP null stream
    return exec_chunk(pl, io, s, chunk, false, true);
}

}  // extern "C"

namespace {

// The host-memory batch around a device plan (linear or affine): stage the
// inputs in the context's grow-only buffers, run `exec`, bring back scores,
// target_begins and the compacted CIGARs.  `slots_bytes` is the plan's CIGAR
// slot arena.  Called with ctx->mu held.
template <class Exec>
int host_batch(ta_context* ctx, uint32_t n_pairs, const char* qb, const uint64_t* qoff, const uint32_t* qlen,
               const char* tbytes, const uint64_t* toff, const uint32_t* tlen, uint64_t qend, uint64_t tend,
               int want_cigar, int32_t* score, uint32_t* target_begin, char* arena, uint64_t arena_bytes,
               uint64_t* cigar_off, uint32_t* cigar_len, uint64_t slots_bytes, Exec&& exec) {
    hipStream_t s = ctx->stream;
    int rc = TA_OK;
    auto chk = [&](int r) {
        if (r != TA_OK && rc == TA_OK) rc = r;
        return rc == TA_OK;
    };
    const size_t P = n_pairs;
    if (chk(grow(ctx, ctx->qbytes, qend)) && chk(grow(ctx, ctx->tbytes, tend)) &&
        chk(grow(ctx, ctx->qoff, P * 8)) && chk(grow(ctx, ctx->toff, P * 8)) && chk(grow(ctx, ctx->score, P * 4)) &&
        chk(grow(ctx, ctx->tb, P * 4)) &&
        (!want_cigar || (chk(grow(ctx, ctx->slots, slots_bytes)) && chk(grow(ctx, ctx->cstart, P * 8)) &&
                         chk(grow(ctx, ctx->clen, P * 4)) && chk(grow(ctx, ctx->dst_off, P * 8))))) {
        auto cp = [&](void* d, const void* h, size_t b) {
            if (!b || rc != TA_OK) return;
            hipError_t e = hipMemcpyAsync(d, h, b, hipMemcpyHostToDevice, s);
            if (e != hipSuccess) rc = fail(ctx, TA_ERR_DEVICE, hipGetErrorString(e));
        };
        cp(ctx->qbytes.p, qb, qend);
        cp(ctx->tbytes.p, tbytes, tend);
        cp(ctx->qoff.p, qoff, P * 8);
        cp(ctx->toff.p, toff, P * 8);
        ta_device_io io{};
        io.query_bytes = (const char*)ctx->qbytes.p;
        io.query_off = (const uint64_t*)ctx->qoff.p;
        io.target_bytes = (const char*)ctx->tbytes.p;
        io.target_off = (const uint64_t*)ctx->toff.p;
        io.score = (int32_t*)ctx->score.p;
        io.target_begin = (uint32_t*)ctx->tb.p;
        io.cigar_slots = (char*)ctx->slots.p;
        io.cigar_start = (uint64_t*)ctx->cstart.p;
        io.cigar_len = (uint32_t*)ctx->clen.p;
        if (rc == TA_OK) chk(exec(&io, s));
        std::vector<int32_t> sc(P);
        std::vector<uint32_t> tb(P);
        auto dn = [&](void* h, const void* d, size_t b) {
            if (!b || rc != TA_OK) return;
            hipError_t e = hipMemcpyAsync(h, d, b, hipMemcpyDeviceToHost, s);
            if (e != hipSuccess) rc = fail(ctx, TA_ERR_DEVICE, hipGetErrorString(e));
        };
        dn(sc.data(), io.score, P * 4);
        dn(tb.data(), io.target_begin, P * 4);
        if (want_cigar) dn(cigar_len, io.cigar_len, P * 4);
        if (rc == TA_OK) {
            hipError_t e = hipStreamSynchronize(s);
            if (e != hipSuccess) rc = fail(ctx, TA_ERR_DEVICE, hipGetErrorString(e));
        }
        if (rc == TA_OK && want_cigar) {
            uint64_t total = 0;
            for (size_t p = 0; p < P; ++p) {
                cigar_off[p] = total;
                total += cigar_len[p];
            }
            if (total > arena_bytes) {
                rc = fail(ctx, TA_ERR_CAPACITY, "cigar arena too small");
            } else if (chk(grow(ctx, ctx->dst, total))) {
                cp(ctx->dst_off.p, cigar_off, P * 8);
                ta::CompactArgs ca{};
                ca.n_pairs = n_pairs;
                ca.slots = io.cigar_slots;
                ca.cigar_start = io.cigar_start;
                ca.cigar_len = io.cigar_len;
                ca.dst_off = (const uint64_t*)ctx->dst_off.p;
                ca.dst = (char*)ctx->dst.p;
                if (rc == TA_OK) {
                    hipError_t e = ta::launch_compact(ca, s);
                    if (e != hipSuccess) rc = fail(ctx, TA_ERR_DEVICE, hipGetErrorString(e));
                }
                dn(arena, ctx->dst.p, total);
                if (rc == TA_OK) {
                    hipError_t e = hipStreamSynchronize(s);
                    if (e != hipSuccess) rc = fail(ctx, TA_ERR_DEVICE, hipGetErrorString(e));
                }
            }
        }
        if (rc == TA_OK) {
            if (score) std::memcpy(score, sc.data(), P * 4);
            if (target_begin) std::memcpy(target_begin, tb.data(), P * 4);
        }
    }
    return rc;
}

// Argument checks shared by the two host-memory batch entries; sets the input extents.
int check_host_batch(ta_context* ctx, int type, uint32_t n_pairs, const char* qb, const uint64_t* qoff,
                     const uint32_t* qlen, const char* tbytes, const uint64_t* toff, const uint32_t* tlen,
                     int want_cigar, char* arena, uint64_t* cigar_off, uint32_t* cigar_len, uint64_t* qend,
                     uint64_t* tend) {
    if (!ctx) return TA_ERR_ARG;
    if (!valid_type(type)) return fail(ctx, TA_ERR_BAD_TYPE, ta_status_string(TA_ERR_BAD_TYPE));
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

}  // namespace

extern "C" {

int ta_align_batch(ta_context* ctx, uint32_t n_pairs, const char* qb, const uint64_t* qoff, const uint32_t* qlen,
                   const char* tbytes, const uint64_t* toff, const uint32_t* tlen, int type, int match,
                   int mismatch, int gap, int want_cigar, int32_t* score, uint32_t* target_begin, char* arena,
                   uint64_t arena_bytes, uint64_t* cigar_off, uint32_t* cigar_len) {
    uint64_t qend = 0, tend = 0;
    if (int r = check_host_batch(ctx, type, n_pairs, qb, qoff, qlen, tbytes, toff, tlen, want_cigar, arena,
                                 cigar_off, cigar_len, &qend, &tend))
        return r;
    if (n_pairs == 0) return TA_OK;
    std::lock_guard<std::mutex> lock(ctx->mu);
    TA_HIP(ctx, hipSetDevice(ctx->device));
    ta_plan* pl = nullptr;
    if (int r = ta_plan_create(ctx, n_pairs, qlen, tlen, type, match, mismatch, gap, want_cigar, 0, &pl)) return r;
    const int rc = host_batch(ctx, n_pairs, qb, qoff, qlen, tbytes, toff, tlen, qend, tend, want_cigar, score,
                              target_begin, arena, arena_bytes, cigar_off, cigar_len, pl->slots_bytes,
                              [&](const ta_device_io* io, hipStream_t s) { return ta_plan_execute(pl, io, s); });
    const int rc2 = rc == TA_OK ? ta_plan_check(pl) : rc;  // host_batch synchronised the stream
    ta_plan_destroy(pl);
    return rc2;
}

int ta_align_batch_affine(ta_context* ctx, uint32_t n_pairs, const char* qb, const uint64_t* qoff,
                          const uint32_t* qlen, const char* tbytes, const uint64_t* toff, const uint32_t* tlen,
                          int type, int match, int mismatch, int gap_open, int gap_extend, int want_cigar,
                          int32_t* score, uint32_t* target_begin, char* arena, uint64_t arena_bytes,
                          uint64_t* cigar_off, uint32_t* cigar_len) {
    uint64_t qend = 0, tend = 0;
    if (int r = check_host_batch(ctx, type, n_pairs, qb, qoff, qlen, tbytes, toff, tlen, want_cigar, arena,
                                 cigar_off, cigar_len, &qend, &tend))
        return r;
    if (n_pairs == 0) return TA_OK;
    std::lock_guard<std::mutex> lock(ctx->mu);
    TA_HIP(ctx, hipSetDevice(ctx->device));
    ta_affine_plan* pl = nullptr;
    if (int r = ta_affine_plan_create(ctx, n_pairs, qlen, tlen, type, match, mismatch, gap_open, gap_extend,
                                      want_cigar, 0, &pl))
        return r;
    const int rc = host_batch(ctx, n_pairs, qb, qoff, qlen, tbytes, toff, tlen, qend, tend, want_cigar, score,
                              target_begin, arena, arena_bytes, cigar_off, cigar_len,
                              ta_affine_plan_cigar_slots_bytes(pl),
                              [&](const ta_device_io* io, hipStream_t s) { return ta_affine_plan_execute(pl, io, s); });
    ta_affine_plan_destroy(pl);
    return rc;
}

}  // extern "C"
