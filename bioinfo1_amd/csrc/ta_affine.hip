// bioinfo1_amd/csrc/ta_affine.hip -- the affine-gap extension on gfx950
// (BASELINE config 5: "affine gaps + full CIGAR traceback"): fill and
// traceback kernels and the ta_affine_plan host driver of
// include/team_align_c.h.
//
// The reference has no affine-gap Align (team_alignment.cpp:25-28 is a linear
// indel); the semantics are DEFINED in oracle/affine_oracle.c (Gotoh E/F/H
// with the reference's strict-> tie order MATCH > INSERT > DELETE, '-' free
// gap steps, the reference's boundaries, goals, local clamp and argmax, walk,
// semi-global tail and RLE).  With gap_open == 0 every result equals
// team::Align with gap = gap_extend (tests/test_affine*.py).
//
// Layout.  Same geometry as the linear int32 fill
// (ta_kernels.hip): one wave64 per pair, lane l owns 16 consecutive query rows
// of a 1024-row pass, lanes sweep the target columns with a one-step lane skew
// and pass their last row's H and F down with DPP wave_shr:1 (the row-0 "up"
// and "diag" of lane l are lane l-1's last row one and two steps earlier).
// Each lane keeps H and E (the horizontal-gap state, which moves along its own
// rows) for its 16 rows in VGPRs; F (vertical) moves down the rows inside the
// step.  Per cell the kernel writes 4 bits as four 16-row bit planes, one
// uint2 per (pass, step, lane) -- 512 coalesced bytes per step:
//   .x = D plane << 16 | I plane   (source, local canonical M/I/D/STOP as the
//                                   linear kernels' Code; global/semi raw
//                                   compares where D wins)
//   .y = F-ext plane << 16 | E-ext plane
// row r of a lane's stripe at bit 15 - r of each plane.  Passes hand their
// bottom row's (H, F) to the next pass through a boundary row in HBM.
// The traceback walks the three-state machine one cell per iteration on the
// SALU with a 64-step tile of the lane stripe's codes held in two VGPRs, and
// writes runs through the shared RunWriter (ta_device.h).
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/team_align_c.h"
#include "ta_context.h"
#include "ta_device.h"
#include "ta_host_batch.h"
#include "ta_planner.h"
#include "ta_packed.h"

namespace ta {
namespace {

constexpr int kNeg = -(1 << 29);  // E(i,0), F(0,j): never wins (|values| < 2^26)

struct AffArgs {
    const uint32_t* order;  // plan order; this launch handles order[begin .. begin+count)
    uint32_t begin, count;
    const uint8_t* qbytes;
    const uint64_t* qoff;
    const uint32_t* qlen;
    const uint8_t* tbytes;
    const uint64_t* toff;
    const uint32_t* tlen;
    int match, mismatch, open, extend;
    uint2* ptrs;              // chunk workspace, one uint2 per (pass, step, lane)
    const uint64_t* ptr_off;  // per pair, uint2 entries from ptrs
    int2* bnd;                // chunk pass-boundary rows: (H, F) per column
    const uint64_t* bnd_off;  // per pair, int2 entries from bnd
    int32_t* score;
    uint32_t* target_begin;
    uint32_t* goal_i;
    uint32_t* goal_j;
    char* slots;
    const uint64_t* slot_off;
    uint64_t* cigar_start;
    uint32_t* cigar_len;
    const uint32_t* count_dev;  // non-null: wave count read on the device (the dual fill's hand-back list)
    uint32_t* fb_list;          // dual fill: couples handed back to the int32 fill ('-' in a query)
    uint32_t* fb_count;
    // dual fill, one wave per (couple, pass): ticket t is pass
    // t / count of couple t % count (pass-major), n_tasks = count * the chunk's
    // largest pass count; passes hand their bottom row over tagged records
    uint32_t* ticket;  // zeroed before the launch
    uint32_t n_tasks;
    uint32_t epoch;    // tag base of this launch's records
    uint32_t* err;     // a poll gave up (never on a correct schedule)
    void* pout;        // PassOut[2] per (pass, couple): [(pass * count + w) * 2 + h]
    // the pipelined int32 fill of multi-pass singles (affine_pipe_kernel): per
    // single its first task, tasks in ticket order (single << 32 | pass),
    // pout = PassOut per task; ticket, n_tasks and err as above
    const uint32_t* task_off;
    const uint64_t* tasks64;
    uint32_t end_aligned;  // dual tickets: level = pass + (chunk passes - couple passes), not the pass
};

// 64 boundary entries per chunk: column 64k+lane+1.
__device__ __forceinline__ int2 load_bchunk2(const int2* B, uint32_t m, uint32_t k, int lane) {
    const uint32_t j = k * 64u + (uint32_t)lane + 1u;
    return j <= m ? B[j] : make_int2(0, kNeg);
}

// The pass boundary row (H, F per column).  A wave sweeping all of a pair's
// passes keeps it in place (B).  The pipelined fill (one wave per (pair,
// pass), affine_pipe_kernel) hands it over as two 8-byte records per column,
// tag << 32 | H and tag << 32 | F, two buffers by pass parity, relaxed
// agent-scope stores polled 64 columns at a time (as the linear int32 fill).
struct AffBnd {
    int2* B;
    uint64_t* rec_w;        // null: B (or the last pass)
    const uint64_t* rec_r;  // null: B (or pass 0)
    uint32_t tag_w, tag_r;
    uint32_t* err;
};

typedef __attribute__((address_space(1))) unsigned long long gu64a;

__device__ __forceinline__ int2 load_bnd2(const AffBnd& io, uint32_t m, uint32_t k, int lane) {
    if (!io.rec_r) return load_bchunk2(io.B, m, k, lane);
    const uint32_t j = k * 64u + (uint32_t)lane + 1u;
    const gu64a* r = (const gu64a*)(io.rec_r + 2ull * j);
    int2 v = make_int2(0, kNeg);
    for (uint32_t spins = 0;; ++spins) {
        bool ok = true;
        if (j <= m) {
            const uint64_t x = __hip_atomic_load(r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t y = __hip_atomic_load(r + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = (uint32_t)(x >> 32) == io.tag_r && (uint32_t)(y >> 32) == io.tag_r;
            v = make_int2((int)(uint32_t)x, (int)(uint32_t)y);
        }
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
        if (spins > (1u << 22)) {  // bounded: the kernel always ends
            if (lane == 0) atomicOr(io.err, 1u);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    return v;
}

// One pass = rows row_base+1 .. row_base+nrows against the whole target.
//   QDASH  some query row of this pass is '-' (its vertical gap steps are free)
//   ROWSEL semi-global last pass whose row n is not the last register
template <int MODE, bool CIGAR, bool QDASH, bool ROWSEL>
__device__ __forceinline__ PassOut aff_pass(const AffArgs& a, const uint8_t* Q, const uint8_t* T, uint32_t n,
                                            uint32_t m, uint32_t pass, bool last_pass, uint2* ptrs, const AffBnd& B,
                                            int lane) {
    constexpr int R = kRows;
    const int O = a.open, X = a.extend, OX = wadd(a.open, a.extend);
    const int MA = a.match, MI = a.mismatch;
    const uint32_t Tmax = pass_steps(m);
    const uint32_t row_base = pass * kPassRows;
    const uint32_t nrows = min((uint32_t)kPassRows, n - row_base);
    const uint32_t nl = (nrows + R - 1) / R;  // lanes in use
    const uint32_t nv = nrows - (nl - 1) * R;  // valid rows of lane nl-1
    const uint32_t vlim = (uint32_t)lane < nl - 1 ? R : ((uint32_t)lane == nl - 1 ? nv : 0u);
    const bool has_next = !last_pass;

    uint32_t qp[R / 4];  // the lane's 16 query bytes, 4 per register
#pragma unroll
    for (int k = 0; k < R / 4; ++k) {
        uint32_t w = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t i0 = row_base + (uint32_t)lane * R + 4 * k + b;
            w |= (i0 < n ? (uint32_t)Q[i0] : 0u) << (8 * b);
        }
        qp[k] = w;
    }
    auto qbyte = [&](int r) { return (qp[r >> 2] >> (8 * (r & 3))) & 0xFFu; };
    int H[R], E[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i = row_base + (uint32_t)lane * R + r + 1;
        H[r] = (MODE == kGlobal) ? wadd(O, wmul(i, X)) : 0;  // column 0
        E[r] = kNeg;
    }
    // per-row vertical gap constants ('-' rows are free)
    int goq[R], geq[R];
    if constexpr (QDASH) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const bool d = qbyte(r) == (uint32_t)'-';
            goq[r] = d ? 0 : OX;
            geq[r] = d ? 0 : X;
        }
    }
    // local argmax key = 16*h + (15 - r) on valid rows; invalid rows never win
    int kc[R];
    if constexpr (MODE == kLocal) {
#pragma unroll
        for (int r = 0; r < R; ++r) kc[r] = (uint32_t)r < vlim ? (R - 1 - r) : -(1 << 30);
    }
    const uint32_t i_above = row_base + (uint32_t)lane * R;  // row above the stripe
    int recvH = (MODE == kGlobal && i_above) ? wadd(O, wmul(i_above, X)) : 0;  // its column 0
    int recvF = kNeg, Flast = kNeg;
    int tc = 0;
    int bestkey = INT_MIN;
    uint32_t bestj = 0;
    int rowbest = INT_MIN;
    uint32_t rowbest_j = 0;

    uint32_t tcur = load_tchunk(T, m, 0, lane), tnext = load_tchunk(T, m, 1, lane);
    int2 bcur = make_int2(0, kNeg), bnext = make_int2(0, kNeg);
    if (pass > 0) {
        bcur = load_bnd2(B, m, 0, lane);
        bnext = load_bnd2(B, m, 1, lane);
    }
    const uint32_t steps = m + nl - 1;
    uint2* prow = CIGAR ? ptrs + (uint64_t)pass * Tmax * kWave : nullptr;

    auto step = [&](uint32_t t, auto masked_tag) {
        constexpr bool MASKED = decltype(masked_tag)::value;
        if ((t & 255u) == 0 && t) {
            tcur = tnext;
            tnext = load_tchunk(T, m, (t >> 8) + 1, lane);
        }
        int topH, topF;
        if (pass == 0) {  // row 0: the boundary (:89-92 with an affine gap)
            topH = (MODE == kGlobal) ? wadd(O, wmul(t + 1, X)) : 0;
            topF = kNeg;
        } else {
            if ((t & 63u) == 0 && t) {
                bcur = bnext;
                bnext = load_bnd2(B, m, (t >> 6) + 1, lane);
            }
            topH = rdlane(bcur.x, t & 63u);
            topF = rdlane(bcur.y, t & 63u);
        }
        const uint32_t word = (uint32_t)rdlane((int)tcur, (t >> 2) & 63u);
        const int newc = (int)((word >> ((t & 3u) * 8)) & 0xFFu);
        const int prev = recvH;
        recvH = wave_shr1(topH, H[R - 1]);
        recvF = wave_shr1(topF, Flast);
        tc = wave_shr1(newc, tc);

        const int j = (int)t - lane + 1;
        const bool active = !MASKED || (((uint32_t)lane < nl) & (j >= 1) & (j <= (int)m));
        uint32_t accD = 0, accI = 0, accE = 0, accF = 0;
        if (active) {
            const bool tdash = tc == '-';
            const int got = tdash ? 0 : OX, get = tdash ? 0 : X;  // horizontal gap step (t[j-1])
            auto score_of = [&](int r) { return (qbyte(r) == (uint32_t)tc) ? MA : MI; };
            int dnext = wadd(prev, score_of(0));
            int upH = recvH, upF = recvF;
            int stepkey = INT_MIN;
            static_for<0, R>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                const int old = H[r];
                const int diag = dnext;
                if constexpr (r + 1 < R) dnext = wadd(old, score_of(r + 1));
                const int eo = wadd(old, got), ee = wadd(E[r], get);
                const int e = max(eo, ee);
                const int fo = wadd(upH, QDASH ? goq[r] : OX), fe = wadd(upF, QDASH ? geq[r] : X);
                const int f = max(fo, fe);
                const int m1 = max(diag, e);
                const int h = (MODE == kLocal) ? max3_imm<0>(m1, f) : max(m1, f);
                if constexpr (CIGAR) {
                    const uint64_t mI = ballot(e > diag);  // INSERT beats MATCH only if strictly greater
                    const uint64_t mD = ballot(f > m1);    // DELETE only if strictly greater
                    uint64_t hi = mD, lo = mI;
                    if constexpr (MODE == kLocal) {
                        const uint64_t mS = ballot(h == 0);  // cost 0 ends the walk (:202)
                        hi |= mS;
                        lo = (mI & ~mD) | mS;
                    }
                    accD = shl1_add_lanebit(accD, hi);
                    accI = shl1_add_lanebit(accI, lo);
                    accE = shl1_add_lanebit(accE, ballot(ee > eo));  // extension strictly better
                    accF = shl1_add_lanebit(accF, ballot(fe > fo));
                }
                if constexpr (MODE == kLocal) stepkey = max(stepkey, (int)(((uint32_t)h << 4) + (uint32_t)kc[r]));
                E[r] = e;
                H[r] = h;
                upH = h;
                upF = f;
            });
            Flast = upF;
            if constexpr (MODE == kLocal) {
                if (stepkey > bestkey) {  // strict: the first column keeps a tie (:186)
                    bestkey = stepkey;
                    bestj = (uint32_t)j;
                }
            }
            if constexpr (MODE == kSemi) {
                if (last_pass) {  // row n is register nv-1 of lane nl-1
                    const int rv = ROWSEL ? select_row<R>(H, nv - 1) : H[R - 1];
                    if (rv > rowbest) {
                        rowbest = rv;
                        rowbest_j = (uint32_t)j;
                    }
                }
            }
            if (has_next && (uint32_t)lane == nl - 1) {
                if (B.rec_w) {
                    const uint64_t tg = (uint64_t)B.tag_w << 32;
                    __hip_atomic_store((gu64a*)(B.rec_w + 2ull * j), tg | (uint32_t)H[R - 1], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store((gu64a*)(B.rec_w + 2ull * j + 1), tg | (uint32_t)Flast, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    B.B[j] = make_int2(H[R - 1], Flast);
                }
            }
        }
        if constexpr (CIGAR) prow[t * kWave + lane] = make_uint2((accD << 16) | accI, (accF << 16) | accE);
    };
    const uint32_t ramp_end = min(nl - 1, steps);
    uint32_t t = 0;
    for (; t < ramp_end; ++t) step(t, std::true_type{});
    for (; t < m; ++t) step(t, std::false_type{});
    for (; t < steps; ++t) step(t, std::true_type{});

    PassOut o{INT_MIN, 0, 0, INT_MIN, 0, 0};
    if constexpr (MODE == kLocal) {
        // h first over lanes (the row tag only orders rows inside a lane), then the first lane
        const int hk = (uint32_t)lane < nl ? (bestkey >> 4) : INT_MIN;
        const int mx = wave_max(hk);
        const int fl = first_lane(hk == mx);
        const int key = rdlane(bestkey, fl);
        o.h = mx;
        o.i = row_base + (uint32_t)fl * R + (uint32_t)(R - 1 - (key & 15)) + 1;
        o.j = (uint32_t)rdlane((int)bestj, fl);
    } else if constexpr (MODE == kSemi) {
        // column m (H holds it now), i ascending, strict '>' (:265-270)
        int cv = INT_MIN;
        uint32_t cr = 0;
#pragma unroll
        for (int r = 0; r < R; ++r)
            if ((uint32_t)r < vlim && H[r] > cv) {
                cv = H[r];
                cr = r;
            }
        const int mx = wave_max(cv);
        const int fl = first_lane(cv == mx && vlim > 0);
        o.h = mx;
        o.i = row_base + (uint32_t)fl * R + (uint32_t)rdlane((int)cr, fl) + 1;
        o.j = m;
        if (last_pass) {
            o.row_h = rdlane(rowbest, nl - 1);
            o.row_j = (uint32_t)rdlane((int)rowbest_j, nl - 1);
        }
    } else {
        if (last_pass) o.corner = rdlane(select_row<R>(H, nv - 1), nl - 1);  // H(n, m)
    }
    return o;
}

template <int MODE, bool CIGAR>
__device__ __forceinline__ PassOut aff_pass_any(const AffArgs& a, const uint8_t* Q, const uint8_t* T, uint32_t n,
                                                uint32_t m, uint32_t pass, bool last_pass, uint2* ptrs,
                                                const AffBnd& B, int lane) {
    bool dash = false;
    const uint32_t row0 = pass * kPassRows + (uint32_t)lane * kRows;
#pragma unroll
    for (int r = 0; r < kRows; ++r) dash |= (row0 + r < n) && Q[row0 + r] == '-';
    const uint32_t nrows = min((uint32_t)kPassRows, n - pass * kPassRows);
    const bool rowsel = MODE == kSemi && last_pass && (nrows % kRows) != 0;
    if (__ballot(dash)) {
        if (MODE == kSemi && rowsel) return aff_pass<MODE, CIGAR, true, true>(a, Q, T, n, m, pass, last_pass, ptrs, B, lane);
        return aff_pass<MODE, CIGAR, true, false>(a, Q, T, n, m, pass, last_pass, ptrs, B, lane);
    }
    if (MODE == kSemi && rowsel) return aff_pass<MODE, CIGAR, false, true>(a, Q, T, n, m, pass, last_pass, ptrs, B, lane);
    return aff_pass<MODE, CIGAR, false, false>(a, Q, T, n, m, pass, last_pass, ptrs, B, lane);
}

template <int MODE, bool CIGAR>
__global__ __launch_bounds__(kBlock) void affine_fill_kernel(AffArgs a) {
    const int lane = threadIdx.x & 63;
    const uint32_t widx = wave_id();
    if (widx >= (a.count_dev ? *a.count_dev : a.count)) return;  // wave-uniform
    const uint32_t p = a.order[a.begin + widx];
    const uint32_t n = a.qlen[p], m = a.tlen[p];
    const int O = a.open, X = a.extend;
    if (n == 0 || m == 0) {  // closed forms of the empty loops (affine boundaries)
        if (lane == 0) {
            int score = 0;
            uint32_t gi = 0, gj = 0, tb = 0;
            if (MODE == kGlobal) {
                gi = n;
                gj = m;
                score = (n || m) ? wadd(O, wmul(n ? n : m, X)) : 0;
            } else if (MODE == kLocal) {
                tb = 1;
            } else {
                gj = (n == 0) ? m : 0;
            }
            a.score[p] = score;
            a.target_begin[p] = tb;
            a.goal_i[p] = gi;
            a.goal_j[p] = gj;
        }
        return;
    }
    const uint8_t* Q = a.qbytes + a.qoff[p];
    const uint8_t* T = a.tbytes + a.toff[p];
    const uint32_t passes = n_passes(n);
    uint2* ptrs = CIGAR ? a.ptrs + a.ptr_off[p] : nullptr;
    const AffBnd B{(passes > 1) ? a.bnd + a.bnd_off[p] : nullptr, nullptr, nullptr, 0, 0, nullptr};

    int best_h = (MODE == kSemi) ? 0 : INT_MIN;  // semi starts from (0,m), cost 0
    uint32_t best_i = 0, best_j = (MODE == kSemi) ? m : 0;
    int corner = 0;
    for (uint32_t pass = 0; pass < passes; ++pass) {
        const bool last_pass = pass + 1 == passes;
        const PassOut o = aff_pass_any<MODE, CIGAR>(a, Q, T, n, m, pass, last_pass, ptrs, B, lane);
        if (MODE != kGlobal && o.h > best_h) {  // strict: the upper pass wins ties
            best_h = o.h;
            best_i = o.i;
            best_j = o.j;
        }
        if (MODE == kSemi && last_pass && o.row_h > best_h) {  // row n after column m (:271-278)
            best_h = o.row_h;
            best_i = n;
            best_j = o.row_j;
        }
        if (MODE == kGlobal && last_pass) corner = o.corner;
        if (!last_pass) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // boundary row -> next pass
    }
    if (lane == 0) {
        a.score[p] = (MODE == kGlobal) ? corner : best_h;
        a.target_begin[p] = (MODE == kLocal) ? best_j + 1 : 0;  // :117-121 / :197-199 / :283-285
        a.goal_i[p] = (MODE == kGlobal) ? n : best_i;
        a.goal_j[p] = (MODE == kGlobal) ? m : best_j;
    }
}

// The pipelined int32 fill: one wave per (pair, pass) of a chunk's singles,
// pass-major tickets (the planner's single_tasks), so the pass a wave polls
// belongs to a wave that took an earlier ticket and is running; the passes'
// results are folded by affine_fill_combine_kernel (as affine_fill_kernel).
template <int MODE, bool CIGAR>
__global__ __launch_bounds__(kBlock) void affine_pipe_kernel(AffArgs a) {
    const int lane = threadIdx.x & 63;
    uint32_t tk = 0;
    if (lane == 0) tk = atomicAdd(a.ticket, 1u);
    tk = (uint32_t)__builtin_amdgcn_readfirstlane((int)tk);
    if (tk >= a.n_tasks) return;
    const uint64_t code = a.tasks64[a.task_off[a.begin] + tk];
    const uint32_t w = (uint32_t)(code >> 32), pass = (uint32_t)code;
    const uint32_t p = a.order[w];
    const uint32_t n = a.qlen[p], m = a.tlen[p];  // both > 0: empty pairs have no task
    const bool last_pass = pass + 1 == n_passes(n);
    uint64_t* rec = reinterpret_cast<uint64_t*>(a.bnd + a.bnd_off[p]);  // 2 buffers x 2 (m + 1) records
    const uint64_t rb = 2ull * ((uint64_t)m + 1);
    // tags: pass + 1 for pass p's row (never 0; the host zeroes the records before the launch)
    const AffBnd B{nullptr, last_pass ? nullptr : rec + (pass & 1u) * rb, pass ? rec + ((pass - 1u) & 1u) * rb : nullptr,
                   pass + 1u, pass, a.err};
    uint2* ptrs = CIGAR ? a.ptrs + a.ptr_off[p] : nullptr;
    const PassOut o = aff_pass_any<MODE, CIGAR>(a, a.qbytes + a.qoff[p], a.tbytes + a.toff[p], n, m, pass, last_pass,
                                                ptrs, B, lane);
    if (lane == 0) static_cast<PassOut*>(a.pout)[a.task_off[w] + pass] = o;
}

template <int MODE>
__global__ void affine_fill_combine_kernel(AffArgs a) {
    const uint32_t w = a.begin + blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= a.begin + a.count) return;
    const uint32_t p = a.order[w];
    const uint32_t n = a.qlen[p], m = a.tlen[p];
    const int O = a.open, X = a.extend;
    int score = 0;
    uint32_t gi = 0, gj = 0, tb = 0;
    if (n == 0 || m == 0) {  // closed forms of the empty loops (affine boundaries)
        if (MODE == kGlobal) {
            gi = n;
            gj = m;
            score = (n || m) ? wadd(O, wmul(n ? n : m, X)) : 0;
        } else if (MODE == kLocal) {
            tb = 1;
        } else {
            gj = (n == 0) ? m : 0;
        }
    } else {
        const PassOut* po = static_cast<const PassOut*>(a.pout) + a.task_off[w];
        const uint32_t passes = a.task_off[w + 1] - a.task_off[w];
        int best_h = (MODE == kSemi) ? 0 : INT_MIN, corner = 0;
        uint32_t best_i = 0, best_j = (MODE == kSemi) ? m : 0;
        for (uint32_t k = 0; k < passes; ++k) {
            const PassOut& o = po[k];
            if (MODE != kGlobal && o.h > best_h) {
                best_h = o.h;
                best_i = o.i;
                best_j = o.j;
            }
            if (MODE == kSemi && k + 1 == passes && o.row_h > best_h) {
                best_h = o.row_h;
                best_i = n;
                best_j = o.row_j;
            }
            if (MODE == kGlobal && k + 1 == passes) corner = o.corner;
        }
        score = (MODE == kGlobal) ? corner : best_h;
        tb = (MODE == kLocal) ? best_j + 1 : 0;
        gi = (MODE == kGlobal) ? n : best_i;
        gj = (MODE == kGlobal) ? m : best_j;
    }
    a.score[p] = score;
    a.target_begin[p] = tb;
    a.goal_i[p] = gi;
    a.goal_j[p] = gj;
}

// The three-state walk (oracle/affine_oracle.c): H-state follows the source
// code, E/F-state emits one I/D per cell and keeps going while the cell's
// extension bit is set.  One cell per iteration; the wave holds the codes of
// 64 consecutive steps of the current lane stripe (lane k: step tt0 + k).
template <int MODE>
__device__ __forceinline__ void aff_traceback_pair(const uint2* P, uint32_t n, uint32_t m, uint32_t gi, uint32_t gj,
                                                   char* slot, uint64_t cap, int lane, uint64_t* start_in_slot,
                                                   uint32_t* len) {
    RunWriter w{slot + cap, 0u, 0u, 0u, 0u, 0u, 0u, lane};
    if (MODE == kSemi && (gj != m || gi != n)) {  // :306-315 (the walk runs backwards: pushed first)
        if (gi == n) {
            if (m - gj) w.push('I', m - gj);
        } else if (gj == m && n - gi) {
            w.push('D', n - gi);
        }
    }
    const uint32_t Tmax = pass_steps(m);
    uint32_t i = gi, j = gj, state = 0;  // 0 H, 1 E, 2 F
    uint32_t tP = 0xFFFFFFFFu, tL = 0xFFFFFFFFu, tt0 = 0;
    uint32_t cx = 0, cy = 0;
    // every iteration moves or leaves H-state, so 2(n+m)+2 bounds a correct
    // walk; the bound (and the E/F edge checks) only keep a corrupt code from
    // spinning the wave
    for (uint32_t it = 0; it < 2u * (n + m) + 2u; ++it) {
        if ((state == 1 && j == 0) || (state == 2 && i == 0)) break;
        if (state == 0) {
            if (MODE == kLocal) {
                if (min(i, j) == 0) break;  // boundary cost 0 ends the walk (:202)
            } else {
                if (i == 0) {  // row 0: INSERT run (:89-92)
                    if (j) w.push('I', j);
                    break;
                }
                if (j == 0) {  // column 0: DELETE run (:83-86)
                    w.push('D', i);
                    break;
                }
            }
        }
        const uint32_t row = i - 1;
        const uint32_t ln = (row >> 4) & 63u, r = row & 15u, ps = row >> 10;
        const uint32_t t = (j - 1) + ln;
        if (ps != tP || ln != tL || t < tt0) {
            tP = ps;
            tL = ln;
            tt0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(max(t, 63u) - 63u));
            const uint32_t ts = tt0 + (uint32_t)lane;
            cx = cy = 0;
            if (ts < Tmax) {
                const uint2 v = P[((uint64_t)tP * Tmax + ts) * kWave + tL];
                cx = v.x;
                cy = v.y;
            }
        }
        const uint32_t kk = t - tt0;
        const uint32_t sh = 15u - r;
        const uint32_t x = (uint32_t)rdlane((int)cx, kk) >> sh, y = (uint32_t)rdlane((int)cy, kk) >> sh;
        if (state == 0) {
            const uint32_t dflag = (x >> 16) & 1u, iflag = x & 1u;
            if (MODE == kLocal && (dflag & iflag)) break;  // STOP: cost == 0 (:202)
            if (dflag) {
                state = 2;
            } else if (iflag) {
                state = 1;
            } else {
                // a whole M run at once: lane L holds step tt0 + L of this stripe, i.e. the
                // diagonal cell d = kk - L back (row r - d); the streak of M codes going down
                // from lane kk is the run (capped at the stripe's first row and the borders)
                const uint32_t v = (cx >> ((sh + (kk - (uint32_t)lane)) & 31u)) & 0x10001u;
                const uint32_t run = min(streak_down(ballot(v == 0u), kk), min(min(i, j), r + 1u));
                w.push('M', run);
                i -= run;
                j -= run;
            }
        } else if (state == 1) {
            w.push('I', 1);
            --j;
            state = (y & 1u) ? 1u : 0u;
        } else {
            w.push('D', 1);
            --i;
            state = ((y >> 16) & 1u) ? 2u : 0u;
        }
    }
    w.finish();
    *start_in_slot = cap - w.used;
    *len = w.used;
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void affine_traceback_kernel(AffArgs a) {
    const int lane = threadIdx.x & 63;
    const uint32_t widx = wave_id();
    if (widx >= a.count) return;
    const uint32_t p = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.order[a.begin + widx]);
    const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.qlen[p]);
    const uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.tlen[p]);
    const uint32_t gi = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.goal_i[p]);
    const uint32_t gj = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.goal_j[p]);
    uint64_t st;
    uint32_t len;
    aff_traceback_pair<MODE>(a.ptrs + a.ptr_off[p], n, m, gi, gj, a.slots + a.slot_off[p], cigar_slot_bytes(n, m),
                             lane, &st, &len);
    if (lane == 0) {
        a.cigar_start[p] = a.slot_off[p] + st;
        a.cigar_len[p] = len;
    }
}

// ---------------------------------------------------------------------------
// Pass hand-off of the packed affine fill.  Each pass of a couple runs on its
// own wave; pass p's bottom row goes to 8-byte records tag << 32 | packed
// value ([2j] = H of both pairs, [2j + 1] = F), written with relaxed
// agent-scope (sc1) stores by the lane holding row 1024(p+1); pass p+1 polls
// a 64-column chunk with sc1 loads until every record carries the tag it
// expects (the data is its own flag, as the flexible fill's, ta_flex.hip).
// Two buffers alternate by pass parity.
typedef __attribute__((address_space(1))) unsigned long long gu64a;

struct AffRec {
    uint64_t* w;        // this pass's bottom row (null on the last pass)
    const uint64_t* r;  // the previous pass's (null on pass 0)
    uint32_t tag_w, tag_r;
    uint32_t* err;
    // this wave's per-step operands of the current 64 steps (aff_dual_pass): entry k for
    // step 64c + k -- both pairs' mismatch tables, the row above (H, F) -- and the bytes
    uint4* lst;
    uint32_t* lstc;
};

// columns 64k + lane + 1 of the previous pass's bottom row: (H, F) packed
__device__ __forceinline__ uint2 aff_poll_chunk(const AffRec& rc, uint32_t m, uint32_t k, int lane) {
    const uint32_t j = k * 64u + (uint32_t)lane + 1u;
    const gu64a* r = (const gu64a*)(rc.r + 2ull * j);
    uint2 v = make_uint2(0, 0);
    for (uint32_t spins = 0;; ++spins) {
        bool ok = true;
        if (j <= m) {
            const uint64_t x = __hip_atomic_load(r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t y = __hip_atomic_load(r + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = (uint32_t)(x >> 32) == rc.tag_r && (uint32_t)(y >> 32) == rc.tag_r;
            v = make_uint2((uint32_t)x, (uint32_t)y);
        }
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
        if (spins > (1u << 22)) {  // bounded: the kernel always ends
            if (lane == 0) atomicOr(rc.err, 1u);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    return v;
}

// ---------------------------------------------------------------------------
// Packed two-pair affine fill (global / semi-global): two pairs of the same
// (n, m) per wave, pair A in bits 15:0 and pair B in bits 31:16 of every
// register, v_pk_* arithmetic.  Same geometry and the same 4-bit codes as
// affine_fill_kernel, so the traceback is shared.  Values are stored biased
// by -ma*j (H, E and F alike: S = V - ma*j), which turns the diagonal
// candidate into one v_pk_mad_i16 of the mismatch flag (ta_dual.hip) and the
// horizontal ones into adds of (go - ma, ge - ma); vertical steps keep the
// bias.  The -inf of E(i,0) / F(0,j) is replaced by H - K with K > |open| +
// |ext|: it loses every comparison there, as -inf does, and stays in range.
// Codes: every compare is the sign of a saturating packed difference, spread
// to bytes by v_perm and inserted by v_bfi (ta_packed.h): x = [D | I] planes
// from (f > m1, e > diag), y = [F-ext | E-ext] planes from (fe > fo, ee > eo).
// The host sends only couples whose every value provably fits int16
// (affine_fits_int16); a couple with '-' in a query goes back to the int32
// fill through fb_list.
// CLS: both queries hold only A, C, G, T -- mismatch flags by table lookup
// (ta_packed.h mismatch_table / row_selector), one v_perm per row.
template <int MODE, bool CIGAR, int NV, bool CLS>
__device__ __forceinline__ void aff_dual_pass(const AffArgs& a, const uint8_t* const (&Q)[2], const uint8_t* const (&T)[2],
                                              uint2* const (&ptrs)[2], const AffRec& rc, uint32_t n, uint32_t m,
                                              uint32_t pass, bool last_pass, bool tdash, int lane, PassOut (&out)[2]) {
    constexpr int R = kRows;
    const int ma = a.match, mi = a.mismatch, O = a.open, X = a.extend;
    const int OX = O + X;
    const int K = abs(O) + abs(X) + 2;  // E(i,0) = H(i,0) - K, F(0,j) = H(0,j) - K
    const uint32_t KD = rep16(mi - ma);
    // Values are S = V - ma*j + X*(j - i) (V = H, E or F): the vertical extension
    // fe = F above (no add), the vertical open H above + O; horizontal gains carry
    // X twice.  No '-' in these queries.
    const uint32_t GOQ = rep16(O);
    uint32_t ONE = 0x00010001u;
    asm volatile("" : "+s"(ONE));  // opaque: keeps v_pk_min_u16 (ta_packed.h)
    const uint32_t Tmax = pass_steps(m);
    const uint32_t row_base = pass * kPassRows;
    const uint32_t nrows = min((uint32_t)kPassRows, n - row_base);
    const uint32_t nl = (nrows + R - 1) / R;
    const bool has_next = !last_pass;
    const uint32_t nv_lane = (uint32_t)lane < nl - 1 ? R : ((uint32_t)lane == nl - 1 ? NV : 0);

    uint32_t q2[R], H2[R], E2[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i0 = row_base + (uint32_t)lane * R + r;  // row i0 + 1
        if constexpr (CLS) q2[r] = i0 < n ? row_selector(Q[0][i0], Q[1][i0]) : row_selector(0, 0);
        else q2[r] = i0 < n ? ((uint32_t)Q[0][i0] | ((uint32_t)Q[1][i0] << 16)) : 0u;
        const int h0 = ((MODE == kGlobal) ? O + (int)(i0 + 1) * X : 0) - X * (int)(i0 + 1);  // S of H(i, 0)
        H2[r] = rep16(h0);
        E2[r] = rep16(h0 - K);
    }
    const uint32_t ia = row_base + (uint32_t)lane * R;  // row above the stripe
    uint32_t recvH = rep16(((MODE == kGlobal && ia) ? O + (int)ia * X : 0) - X * (int)ia);  // S of H(ia, 0)
    uint32_t recvF = 0, Flast = 0;
    uint32_t tc2 = 0, tA = 0x01010101u, tB = 0x01010101u;
    uint32_t maj = rep16(-(ma - X) * lane);  // (ma - X)*j at t = -1 (semi: row n holds H = S + (ma - X)*j + X*n)
    const uint32_t MA2 = rep16(ma - X);
    uint32_t jj = rep16(-lane);
    uint32_t rowbest = rep16(-32768), rowbest_j = 0;

    // A step's wave-uniform operands come from one LDS read of a 64-entry list each lane
    // fills for its column every 64 steps, instead of v_readlane and SALU tables per step
    // (ta_dual.hip LST)
    uint32_t tnext[2];
    auto tbyte = [&](int h, uint32_t c) -> uint32_t {  // target byte of step 64c + lane
        const uint32_t k = c * 64u + (uint32_t)lane;
        return k < m ? (uint32_t)T[h][k] : 0u;
    };
#pragma unroll
    for (int h = 0; h < 2; ++h) tnext[h] = tbyte(h, 0);
    // the previous pass's bottom row, polled one 64-column chunk at a time just
    // before it is needed
    uint2 bcur = make_uint2(0, 0);
    if (pass > 0) bcur = aff_poll_chunk(rc, m, 0, lane);
    auto lst_fill = [&](uint32_t c) {
        uint32_t tH = bcur.x, tF = bcur.y;
        if (pass == 0) {  // row 0 (:89-92 with an affine gap): H(0,j) - ma*j; F(0,j) = -inf stand-in
            const int jt = (int)(c * 64u) + lane + 1;
            const int h0 = ((MODE == kGlobal) ? O + jt * X : 0) - ma * jt + X * jt;
            tH = rep16(h0);
            tF = rep16(h0 - K);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // (after the last chunk's reads)
        rc.lst[lane] = make_uint4(mismatch_table(tnext[0]), mismatch_table(tnext[1]), tH, tF);
        rc.lstc[lane] = tnext[0] | (tnext[1] << 16);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
        for (int h = 0; h < 2; ++h) tnext[h] = tbyte(h, c + 1);
    };
    lst_fill(0);
    const uint32_t steps = m + nl - 1;
    uint2* prow0 = CIGAR ? ptrs[0] + (uint64_t)pass * Tmax * kWave : nullptr;
    uint2* prow1 = CIGAR ? ptrs[1] + (uint64_t)pass * Tmax * kWave : nullptr;

    auto reload = [&](uint32_t t) {
        if (pass > 0) bcur = aff_poll_chunk(rc, m, t >> 6, lane);
        lst_fill(t >> 6);
    };
    auto step = [&](uint32_t t, auto masked_tag) {
        constexpr bool MASKED = decltype(masked_tag)::value;
        const uint4 e = rc.lst[t & 63u];  // (one address for the wave: a broadcast)
        const uint32_t prev = recvH;
        recvH = (uint32_t)wave_shr1((int)e.z, (int)H2[R - 1]);
        recvF = (uint32_t)wave_shr1((int)e.w, (int)Flast);
        if constexpr (CLS) {
            tA = (uint32_t)wave_shr1((int)e.x, (int)tA);
            tB = (uint32_t)wave_shr1((int)e.y, (int)tB);
            if (tdash) tc2 = (uint32_t)wave_shr1((int)rc.lstc[t & 63u], (int)tc2);
        } else {
            tc2 = (uint32_t)wave_shr1((int)rc.lstc[t & 63u], (int)tc2);
        }
        jj = pk_add(jj, ONE);
        if (MODE == kSemi) maj = pk_add(maj, MA2);

        const int j = (int)t - lane + 1;
        const bool active = !MASKED || (((uint32_t)lane < nl) & (j >= 1) & (j <= (int)m));
        uint32_t ax0 = 0, ax1 = 0, ay0 = 0, ay1 = 0;
        if (active) {
            uint32_t GOT = rep16(OX + X - ma), GET = rep16(2 * X - ma);  // horizontal, biased
            if (tdash) {  // a '-' target byte: the horizontal step is free
                const bool da = (tc2 & 0xFFFFu) == '-', db = (tc2 >> 16) == '-';
                GOT = ((uint32_t)(da ? X - ma : OX + X - ma) & 0xFFFFu) | ((uint32_t)(db ? X - ma : OX + X - ma) << 16);
                GET = ((uint32_t)(da ? X - ma : 2 * X - ma) & 0xFFFFu) | ((uint32_t)(db ? X - ma : 2 * X - ma) << 16);
            }
            auto e_of = [&](int r) {  // 0 on a match, 1 otherwise
                if constexpr (CLS) return mismatch_flags(tA, tB, q2[r]);
                else return pk_min_u16(q2[r] ^ tc2, ONE);
            };
            uint32_t dnext = pk_mad_i16(e_of(0), KD, prev);
            uint32_t upH = recvH, upF = recvF;
            static_for<0, R>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                const uint32_t old = H2[r];
                const uint32_t diag = dnext;
                if constexpr (r + 1 < R) dnext = pk_mad_i16(e_of(r + 1), KD, old);
                const uint32_t eo = pk_add(old, GOT), ee = pk_add(E2[r], GET);
                const uint32_t e = pk_max(eo, ee);
                const uint32_t fo = pk_add(upH, GOQ), fe = upF;
                const uint32_t f = pk_max(fo, fe);
                const uint32_t m1 = pk_max(diag, e);
                const uint32_t h = pk_max(m1, f);
                if (CIGAR) {
                    const uint32_t wi = pk_sub_sat(diag, e);  // sign: e > diag   (INSERT)
                    const uint32_t wd = pk_sub_sat(m1, f);    // sign: f > m1     (DELETE)
                    const uint32_t xe = pk_sub_sat(eo, ee);   // sign: ee > eo    (E extends)
                    const uint32_t xf = pk_sub_sat(fo, fe);   // sign: fe > fo    (F extends)
                    uint32_t& ax = (r < 8) ? ax0 : ax1;
                    uint32_t& ay = (r < 8) ? ay0 : ay1;
                    ax = bfi(0x01010101u << (7 - (r & 7)), sign_bytes(wd, wi), ax);
                    ay = bfi(0x01010101u << (7 - (r & 7)), sign_bytes(xf, xe), ay);
                }
                E2[r] = e;
                H2[r] = h;
                upH = h;
                upF = f;
            });
            Flast = upF;
            if (MODE == kSemi && (NV != R || last_pass)) {  // row n: H = S + ma*j, strict '>' (:271-278)
                const uint32_t v = pk_add(H2[NV - 1], maj);
                rowbest_j = bfi(half_mask(pk_sub_sat(rowbest, v)), jj, rowbest_j);
                rowbest = pk_max(rowbest, v);
            }
            if (has_next && (uint32_t)lane == nl - 1) {
                const uint64_t tg = (uint64_t)rc.tag_w << 32;
                gu64a* wr = (gu64a*)(rc.w + 2ull * j);
                __hip_atomic_store(wr, tg | H2[R - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(wr + 1, tg | Flast, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (CIGAR) {
            // 32-bit byte offset from the uniform row base (SGPR base + VGPR offset stores)
            const uint32_t off = (t * kWave + (uint32_t)lane) * 8u;
            *(uint2*)((char*)prow0 + off) =
                make_uint2(__builtin_amdgcn_perm(ax0, ax1, 0x06020400u), __builtin_amdgcn_perm(ay0, ay1, 0x06020400u));
            *(uint2*)((char*)prow1 + off) =
                make_uint2(__builtin_amdgcn_perm(ax0, ax1, 0x07030501u), __builtin_amdgcn_perm(ay0, ay1, 0x07030501u));
        }
    };
    const uint32_t ramp_end = min(nl - 1, steps);
    const uint32_t every = 64u;  // (the operand list's chunks)
    uint32_t t = 0, next_reload = every;
    auto run_steps = [&](uint32_t t_end, auto masked_tag) {
        while (t < t_end) {
            if (t == next_reload) {
                reload(t);
                next_reload += every;
            }
            const uint32_t blk = min(t_end, next_reload);
            for (; t < blk; ++t) step(t, masked_tag);
        }
    };
    run_steps(ramp_end, std::true_type{});
    run_steps(m, std::false_type{});
    run_steps(steps, std::true_type{});

#pragma unroll
    for (int h = 0; h < 2; ++h) {
        PassOut& o = out[h];
        o = PassOut{INT_MIN, 0, 0, INT_MIN, 0, 0};
        if (MODE == kSemi) {
            // column m: H = S + (ma - X)*m + X*i; first lane, then first row (:265-270)
            int cv = INT_MIN;
            uint32_t cr = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int sv = (h ? hi16(H2[r]) : lo16(H2[r])) + X * (int)(row_base + (uint32_t)lane * R + r + 1);
                if ((uint32_t)r < nv_lane && sv > cv) {
                    cv = sv;
                    cr = r;
                }
            }
            const int mx = wave_max(cv);
            const int fl = first_lane(cv == mx && nv_lane > 0);
            o.h = mx + (ma - X) * (int)m;
            o.i = row_base + (uint32_t)fl * R + (uint32_t)rdlane((int)cr, fl) + 1;
            o.j = m;
            if (last_pass) {
                const int rb = rdlane(h ? hi16(rowbest) : lo16(rowbest), nl - 1);
                o.row_h = rb == -32768 ? INT_MIN : rb + X * (int)n;  // -32768: never set
                o.row_j = (uint32_t)rdlane((int)(h ? (rowbest_j >> 16) : (rowbest_j & 0xFFFFu)), nl - 1);
            }
        } else if (last_pass) {
            int hv[R];
#pragma unroll
            for (int r = 0; r < R; ++r) hv[r] = h ? hi16(H2[r]) : lo16(H2[r]);
            o.corner = rdlane(select_row<R>(hv, nrows - (nl - 1) * R - 1), nl - 1) + (ma - X) * (int)m + X * (int)n;
        }
    }
}

template <int MODE, bool CIGAR, bool CLS>
__device__ __forceinline__ void aff_dual_pass_nv(const AffArgs& a, const uint8_t* const (&Q)[2],
                                                 const uint8_t* const (&T)[2], uint2* const (&ptrs)[2],
                                                 const AffRec& rc, uint32_t n, uint32_t m, uint32_t pass,
                                                 bool last_pass, bool tdash, int lane, PassOut (&out)[2]) {
    const uint32_t nrows = min((uint32_t)kPassRows, n - pass * kPassRows);
    const uint32_t nv = nrows - ((nrows + kRows - 1) / kRows - 1) * kRows;
    if (MODE == kGlobal || nv == kRows || !last_pass)
        return aff_dual_pass<MODE, CIGAR, kRows, CLS>(a, Q, T, ptrs, rc, n, m, pass, last_pass, tdash, lane, out);
#define TA_NV_CASE(k) \
    case k: return aff_dual_pass<MODE, CIGAR, k, CLS>(a, Q, T, ptrs, rc, n, m, pass, last_pass, tdash, lane, out);
    switch (nv) {
        TA_NV_CASE(1) TA_NV_CASE(2) TA_NV_CASE(3) TA_NV_CASE(4) TA_NV_CASE(5) TA_NV_CASE(6) TA_NV_CASE(7)
        TA_NV_CASE(8) TA_NV_CASE(9) TA_NV_CASE(10) TA_NV_CASE(11) TA_NV_CASE(12) TA_NV_CASE(13) TA_NV_CASE(14)
        default: TA_NV_CASE(15)
    }
#undef TA_NV_CASE
}

constexpr uint32_t kAffSkip = 0xFFFFFFFFu;  // PassOut.i of a couple handed to the int32 fill

// order: 2 pair ids per couple (same n and m, values within int16).  One wave
// per (couple, pass): a wave takes the next ticket, level-major (level = pass,
// or end-aligned pass + chunk passes - couple passes: ta_planner.cpp
// order_pass_tasks), so the pass it polls belongs to a wave that
// took an earlier ticket and is running -- every poll ends -- and a chunk of
// long couples (config 5: 2,048 couples x 10 passes) fills every wave slot
// instead of two per SIMD.  Each wave writes its pass's PassOut; a combine
// kernel folds them.
template <int MODE, bool CIGAR>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(5))) void affine_dual_fill_kernel(AffArgs a) {
    const int lane = threadIdx.x & 63;
    __shared__ uint4 lst_all[kWavesPerBlock * 64];  // (aff_dual_pass: the per-step operands)
    __shared__ uint32_t lstc_all[kWavesPerBlock * 64];
    uint32_t tk = 0;
    if (lane == 0) tk = atomicAdd(a.ticket, 1u);
    tk = (uint32_t)__builtin_amdgcn_readfirstlane((int)tk);
    if (tk >= a.n_tasks) return;
    const uint32_t level = tk / a.count, w = tk - level * a.count;
    uint32_t p[2];
    p[0] = a.order[2 * (a.begin + w)];
    p[1] = a.order[2 * (a.begin + w) + 1];
    const uint32_t n = a.qlen[p[0]], m = a.tlen[p[0]];
    const uint32_t passes = n_passes(n);
    const uint32_t shift = a.end_aligned ? a.n_tasks / a.count - passes : 0u;
    if (level < shift) return;
    const uint32_t pass = level - shift;
    if (pass >= passes) return;
    PassOut* po = static_cast<PassOut*>(a.pout) + 2ull * ((uint64_t)pass * a.count + w);
    const uint8_t* Q[2];
    const uint8_t* T[2];
    uint2* ptrs[2];
    bool tdash = false, qdash = false, qother = false;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        Q[h] = a.qbytes + a.qoff[p[h]];
        T[h] = a.tbytes + a.toff[p[h]];
        ptrs[h] = CIGAR ? a.ptrs + a.ptr_off[p[h]] : nullptr;
        for (uint32_t k = (uint32_t)lane; k < m; k += 64) tdash |= T[h][k] == '-';
        for (uint32_t k = (uint32_t)lane; k < n; k += 64) {
            const uint32_t c = Q[h][k];
            qdash |= c == '-';
            qother |= !is_acgt(c);
        }
    }
    const bool cls = __ballot(qother) == 0;
    if (__ballot(qdash)) {  // per-row vertical gap constants: the int32 fill takes the couple (pass 0 hands it over)
        if (lane == 0) {
            if (pass == 0) {
                // a self-coupled pair (p[0] == p[1]) is handed back once
                const uint32_t k = (p[1] != p[0]) ? 2u : 1u;
                const uint32_t at = atomicAdd(a.fb_count, k);
                a.fb_list[at] = p[0];
                if (k == 2) a.fb_list[at + 1] = p[1];
            }
            po[0].i = kAffSkip;
            po[1].i = kAffSkip;
        }
        return;
    }
    tdash = __ballot(tdash) != 0;
    const bool last_pass = pass + 1 == passes;
    AffRec rc;
    uint64_t* rec = reinterpret_cast<uint64_t*>(a.bnd + a.bnd_off[p[0]]);  // 2 buffers x 2(m+1) records
    const uint64_t rb = 2ull * (m + 1);
    rc.w = last_pass ? nullptr : rec + (pass & 1u) * rb;
    rc.r = pass ? rec + ((pass - 1u) & 1u) * rb : nullptr;
    // never 0, unique per launch and pass (passes < 64: affine_fits_int16); the
    // host zeroes the records before each launch
    rc.tag_w = a.epoch * 64u + pass + 1u;
    rc.tag_r = a.epoch * 64u + pass;
    rc.err = a.err;
    rc.lst = lst_all + (threadIdx.x >> 6) * 64;
    rc.lstc = lstc_all + (threadIdx.x >> 6) * 64;
    PassOut o[2];
    if (cls) aff_dual_pass_nv<MODE, CIGAR, true>(a, Q, T, ptrs, rc, n, m, pass, last_pass, tdash, lane, o);
    else aff_dual_pass_nv<MODE, CIGAR, false>(a, Q, T, ptrs, rc, n, m, pass, last_pass, tdash, lane, o);
    if (lane == 0) {
        po[0] = o[0];
        po[1] = o[1];
    }
}

// After the packed fill: fold each couple's per-pass results in pass order
// (semi: the upper pass wins ties on column m, then row n strictly above,
// :265-278; global: the last pass's corner).
template <int MODE>
__global__ void affine_dual_combine_kernel(AffArgs a) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= a.count) return;
    const PassOut* po = static_cast<const PassOut*>(a.pout);
    if (po[2ull * w].i == kAffSkip) return;
    const uint32_t p0 = a.order[2 * (a.begin + w)];
    const uint32_t n = a.qlen[p0], m = a.tlen[p0], passes = n_passes(n);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t p = a.order[2 * (a.begin + w) + h];
        int best_h = (MODE == kSemi) ? 0 : INT_MIN, corner = 0;  // semi starts from (0,m), cost 0
        uint32_t best_i = 0, best_j = (MODE == kSemi) ? m : 0;
        for (uint32_t k = 0; k < passes; ++k) {
            const PassOut& o = po[2ull * ((uint64_t)k * a.count + w) + h];
            if (MODE == kSemi && o.h > best_h) {
                best_h = o.h;
                best_i = o.i;
                best_j = o.j;
            }
            if (MODE == kSemi && k + 1 == passes && o.row_h > best_h) {
                best_h = o.row_h;
                best_i = n;
                best_j = o.row_j;
            }
            if (MODE == kGlobal && k + 1 == passes) corner = o.corner;
        }
        a.score[p] = (MODE == kGlobal) ? corner : best_h;
        a.target_begin[p] = 0;
        a.goal_i[p] = (MODE == kGlobal) ? n : best_i;
        a.goal_j[p] = (MODE == kGlobal) ? m : best_j;
    }
}

inline dim3 aff_grid(uint32_t waves) { return dim3((waves + kWavesPerBlock - 1) / kWavesPerBlock); }

hipError_t launch_affine_dual(int mode, bool cigar, const AffArgs& a, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    const dim3 g = aff_grid(a.n_tasks), b(kBlock), gc((a.count + 255) / 256), bc(256);
    switch (mode * 2 + (cigar ? 1 : 0)) {
        case kGlobal * 2: hipLaunchKernelGGL((affine_dual_fill_kernel<kGlobal, false>), g, b, 0, s, a); break;
        case kGlobal * 2 + 1: hipLaunchKernelGGL((affine_dual_fill_kernel<kGlobal, true>), g, b, 0, s, a); break;
        case kSemi * 2: hipLaunchKernelGGL((affine_dual_fill_kernel<kSemi, false>), g, b, 0, s, a); break;
        case kSemi * 2 + 1: hipLaunchKernelGGL((affine_dual_fill_kernel<kSemi, true>), g, b, 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    if (mode == kGlobal) hipLaunchKernelGGL(affine_dual_combine_kernel<kGlobal>, gc, bc, 0, s, a);
    else hipLaunchKernelGGL(affine_dual_combine_kernel<kSemi>, gc, bc, 0, s, a);
    return hipGetLastError();
}

hipError_t launch_affine_fill(int mode, bool cigar, const AffArgs& a, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    const dim3 g = aff_grid(a.count), b(kBlock);
    if (a.tasks64) {  // one wave per (pair, pass), then the fold of the passes
        const dim3 gt = aff_grid(a.n_tasks), gc((a.count + 255) / 256), bc(256);
#define TA_AFF_PIPE(M)                                                                                   \
    case M:                                                                                              \
        if (a.n_tasks) {                                                                                 \
            if (cigar) hipLaunchKernelGGL((affine_pipe_kernel<M, true>), gt, b, 0, s, a);                \
            else hipLaunchKernelGGL((affine_pipe_kernel<M, false>), gt, b, 0, s, a);                     \
        }                                                                                                \
        hipLaunchKernelGGL(affine_fill_combine_kernel<M>, gc, bc, 0, s, a);                              \
        break;
        switch (mode) {
            TA_AFF_PIPE(kGlobal)
            TA_AFF_PIPE(kLocal)
            TA_AFF_PIPE(kSemi)
            default: return hipErrorInvalidValue;
        }
#undef TA_AFF_PIPE
        return hipGetLastError();
    }
#define TA_AFF_FILL(M)                                                                   \
    case M:                                                                              \
        if (cigar) hipLaunchKernelGGL((affine_fill_kernel<M, true>), g, b, 0, s, a);     \
        else hipLaunchKernelGGL((affine_fill_kernel<M, false>), g, b, 0, s, a);          \
        break;
    switch (mode) {
        TA_AFF_FILL(kGlobal)
        TA_AFF_FILL(kLocal)
        TA_AFF_FILL(kSemi)
        default: return hipErrorInvalidValue;
    }
#undef TA_AFF_FILL
    return hipGetLastError();
}

hipError_t launch_affine_traceback(int mode, const AffArgs& a, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    const dim3 g = aff_grid(a.count), b(kBlock);
    switch (mode) {
        case kGlobal: hipLaunchKernelGGL(affine_traceback_kernel<kGlobal>, g, b, 0, s, a); break;
        case kLocal: hipLaunchKernelGGL(affine_traceback_kernel<kLocal>, g, b, 0, s, a); break;
        case kSemi: hipLaunchKernelGGL(affine_traceback_kernel<kSemi>, g, b, 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace
}  // namespace ta

// ---------------------------------------------------------------------------
// Host driver (the planning is ta_planner.cpp build_affine_plan).
struct ta_affine_plan {
    ta_context* ctx = nullptr;
    ta::AffinePlan h;
    void* own_block = nullptr;  // device arrays of a plan made by ta_affine_plan_create (one allocation)
    uint32_t *d_qlen = nullptr, *d_tlen = nullptr, *d_order = nullptr, *d_goal_i = nullptr, *d_goal_j = nullptr;
    uint32_t *d_singles = nullptr, *d_duals = nullptr;
    uint32_t* d_fb = nullptr;  // hand-back list [2 * couples], then one counter per chunk
    uint64_t *d_ptr_off = nullptr, *d_bnd_off = nullptr, *d_slot_off = nullptr;
    uint32_t *d_err = nullptr, *d_tickets = nullptr;  // packed fill: poll error word, one ticket counter per chunk
    void* d_pout = nullptr;                           // PassOut[2] per (pass, couple) of one chunk
    uint32_t* d_stask_off = nullptr;  // pipelined int32 fill: per single, its first task
    uint64_t* d_stasks = nullptr;     // ... its tasks in ticket order
    void* d_spout = nullptr;          // ... PassOut per task
};

namespace {

using ta_host::fail;

struct AffOffs {
    uint64_t qlen, tlen, order, singles, duals, stask_off, stasks, ptr_off, bnd_off, slot_off, err, tickets;  // uploaded
    uint64_t goal_i, goal_j, fb, pout, spout;                                                               // device-only
};

// PassOut[2] per (pass, couple) of the largest chunk (24-byte PassOut)
uint64_t aff_pout_bytes(const ta::AffinePlan& h) {
    uint64_t n = 0;
    for (const auto& ch : h.chunks) n = std::max<uint64_t>(n, 2ull * ch.dcount * ch.dpasses);
    return n * 24ull;
}

template <class T>
uint64_t avbytes(const std::vector<T>& v) {
    return v.size() * sizeof(T);
}

AffOffs aff_layout(const ta::AffinePlan& h, ta::BlockLayout& L) {
    AffOffs o{};
    o.qlen = L.add(avbytes(h.qlen));
    o.tlen = L.add(avbytes(h.tlen));
    o.order = L.add(avbytes(h.order));
    o.singles = L.add(avbytes(h.singles));
    o.duals = L.add(avbytes(h.duals));
    o.stask_off = L.add(avbytes(h.single_task_off));
    o.stasks = L.add(avbytes(h.single_tasks));
    o.ptr_off = L.add(avbytes(h.ptr_off));
    o.bnd_off = L.add(avbytes(h.bnd_off));
    o.slot_off = L.add(avbytes(h.slot_off));
    o.err = L.add(4);
    o.tickets = L.add(8ull * h.chunks.size());  // per chunk: packed, then pipelined int32
    return o;
}

void aff_layout_scratch(const ta::AffinePlan& h, ta::BlockLayout& L, AffOffs& o) {
    o.goal_i = L.add(4ull * h.n_pairs);
    o.goal_j = L.add(4ull * h.n_pairs);
    o.fb = L.add(4ull * (h.duals.size() + h.chunks.size()));
    o.pout = L.add(aff_pout_bytes(h));
    o.spout = L.add(h.single_tasks.size() * 24ull);
}

void aff_pack(const ta::AffinePlan& h, const AffOffs& o, uint8_t* base) {
    auto put = [&](uint64_t at, const auto& v) {
        if (!v.empty()) std::memcpy(base + at, v.data(), avbytes(v));
    };
    put(o.qlen, h.qlen);
    put(o.tlen, h.tlen);
    put(o.order, h.order);
    put(o.singles, h.singles);
    put(o.duals, h.duals);
    put(o.stask_off, h.single_task_off);
    put(o.stasks, h.single_tasks);
    put(o.ptr_off, h.ptr_off);
    put(o.bnd_off, h.bnd_off);
    put(o.slot_off, h.slot_off);
    std::memset(base + o.err, 0, 4);
    std::memset(base + o.tickets, 0, 8ull * h.chunks.size());
}

void aff_bind(ta_affine_plan* pl, uint8_t* d, const AffOffs& o) {
    auto u32 = [&](uint64_t at) { return reinterpret_cast<uint32_t*>(d + at); };
    auto u64 = [&](uint64_t at) { return reinterpret_cast<uint64_t*>(d + at); };
    pl->d_qlen = u32(o.qlen);
    pl->d_tlen = u32(o.tlen);
    pl->d_order = u32(o.order);
    pl->d_singles = u32(o.singles);
    pl->d_duals = u32(o.duals);
    pl->d_ptr_off = u64(o.ptr_off);
    pl->d_bnd_off = u64(o.bnd_off);
    pl->d_slot_off = u64(o.slot_off);
    pl->d_goal_i = u32(o.goal_i);
    pl->d_goal_j = u32(o.goal_j);
    pl->d_fb = u32(o.fb);
    pl->d_err = u32(o.err);
    pl->d_tickets = u32(o.tickets);
    pl->d_pout = d + o.pout;
    pl->d_stask_off = u32(o.stask_off);
    pl->d_stasks = u64(o.stasks);
    pl->d_spout = d + o.spout;
}

// the oracle's range (oracle_affine_in_range): every |value| < 2^26
bool affine_in_range(uint32_t n_pairs, const uint32_t* qlen, const uint32_t* tlen, int match, int mismatch,
                     int gap_open, int gap_extend) {
    uint64_t maxn = 0, maxm = 0;
    for (uint32_t p = 0; p < n_pairs; ++p) {
        maxn = std::max<uint64_t>(maxn, qlen[p]);
        maxm = std::max<uint64_t>(maxm, tlen[p]);
    }
    const long long pm = std::max({std::llabs(match), std::llabs(mismatch),
                                   std::llabs(gap_open) + std::llabs(gap_extend)});
    return (long long)(maxn + maxm + 2) * pm < (1ll << 26);
}

int affine_check_args(ta_context* ctx, uint32_t n_pairs, const uint32_t* qlen, const uint32_t* tlen, int type,
                      int match, int mismatch, int gap_open, int gap_extend) {
    if (!ctx) return TA_ERR_ARG;
    if (n_pairs && (!qlen || !tlen)) return fail(ctx, TA_ERR_ARG, "null argument");
    if (type != TA_GLOBAL && type != TA_LOCAL && type != TA_SEMI_GLOBAL)
        return fail(ctx, TA_ERR_BAD_TYPE, ta_status_string(TA_ERR_BAD_TYPE));
    if (!affine_in_range(n_pairs, qlen, tlen, match, mismatch, gap_open, gap_extend))
        return fail(ctx, TA_ERR_RANGE, ta_status_string(TA_ERR_RANGE));
    return TA_OK;
}

int affine_check_io(ta_affine_plan* pl, const ta_device_io* io) {
    if (!pl || !io) return TA_ERR_ARG;
    if (pl->h.n_pairs && (!io->query_off || !io->target_off || !io->score || !io->target_begin))
        return fail(pl->ctx, TA_ERR_ARG, "null device pointer");
    if (pl->h.want_cigar && pl->h.n_pairs && (!io->cigar_slots || !io->cigar_start || !io->cigar_len))
        return fail(pl->ctx, TA_ERR_ARG, "null cigar device pointer");
    return TA_OK;
}

int affine_exec_chunk(ta_affine_plan* pl, const ta_device_io* io, hipStream_t s, uint32_t c, bool fill, bool trace) {
    ta_context* ctx = pl->ctx;
    const ta::AffinePlan& h = pl->h;
    if (int r = ta_host::grow(ctx, ctx->ws_ptrs, h.ws_ptr_entries * sizeof(uint2))) return r;
    if (int r = ta_host::grow(ctx, ctx->ws_bnd, h.ws_bnd_entries * sizeof(int2))) return r;
    const auto& ch = h.chunks[c];
    ta::AffArgs a{};
    a.order = pl->d_order;
    a.begin = ch.begin;
    a.count = ch.count;
    a.qbytes = (const uint8_t*)io->query_bytes;
    a.qoff = io->query_off;
    a.qlen = pl->d_qlen;
    a.tbytes = (const uint8_t*)io->target_bytes;
    a.toff = io->target_off;
    a.tlen = pl->d_tlen;
    a.match = h.match;
    a.mismatch = h.mismatch;
    a.open = h.open;
    a.extend = h.extend;
    a.ptrs = (uint2*)ctx->ws_ptrs.p;
    a.ptr_off = pl->d_ptr_off;
    a.bnd = (int2*)ctx->ws_bnd.p;
    a.bnd_off = pl->d_bnd_off;
    a.score = io->score;
    a.target_begin = io->target_begin;
    a.goal_i = pl->d_goal_i;
    a.goal_j = pl->d_goal_j;
    a.slots = io->cigar_slots;
    a.slot_off = pl->d_slot_off;
    a.cigar_start = io->cigar_start;
    a.cigar_len = io->cigar_len;
    if (fill) {
        roctxRangePushA("ta affine fill");
        // pass hand-off records start zeroed (tags are small integers; the region may hold old codes)
        if ((ch.dcount && ch.dpasses > 1) || ch.spasses > 1)
            TA_HIP(ctx, hipMemsetAsync(ctx->ws_bnd.p, 0, ch.bnd_entries * sizeof(int2), s));
        if (ch.dcount) {  // packed couples, then the couples they hand back, on the same stream
            uint32_t* fb_list = pl->d_fb + 2ull * ch.dbegin;
            uint32_t* fb_count = pl->d_fb + h.duals.size() + c;
            TA_HIP(ctx, hipMemsetAsync(fb_count, 0, 4, s));
            ta::AffArgs d = a;
            d.order = pl->d_duals;
            d.begin = ch.dbegin;
            d.count = ch.dcount;
            d.fb_list = fb_list;
            d.fb_count = fb_count;
            // one wave per (couple, pass), tickets pass-major
            d.ticket = pl->d_tickets + c;
            d.n_tasks = ch.dcount * ch.dpasses;
            d.epoch = ++ctx->epoch & 0x3FFFFFFu;
            d.err = pl->d_err;
            d.pout = pl->d_pout;
            d.end_aligned = h.end_aligned ? 1u : 0u;
            TA_HIP(ctx, hipMemsetAsync(d.ticket, 0, 4, s));
            TA_HIP(ctx, ta::launch_affine_dual(h.type, h.want_cigar, d, s));
            ta::AffArgs f = a;
            f.order = fb_list;
            f.begin = 0;
            f.count = 2 * ch.dcount;
            f.count_dev = fb_count;
            TA_HIP(ctx, ta::launch_affine_fill(h.type, h.want_cigar, f, s));
        }
        ta::AffArgs sa = a;
        sa.order = pl->d_singles;
        sa.begin = ch.sbegin;
        sa.count = ch.scount;
        if (ch.spasses > 1) {  // one wave per (pair, pass), tickets pass-major
            sa.task_off = pl->d_stask_off;
            sa.tasks64 = pl->d_stasks;
            sa.ticket = pl->d_tickets + h.chunks.size() + c;
            sa.n_tasks = h.single_task_off[ch.sbegin + ch.scount] - h.single_task_off[ch.sbegin];
            sa.err = pl->d_err;
            sa.pout = pl->d_spout;
            TA_HIP(ctx, hipMemsetAsync(sa.ticket, 0, 4, s));
        }
        TA_HIP(ctx, ta::launch_affine_fill(h.type, h.want_cigar, sa, s));
        roctxRangePop();
    }
    if (trace && h.want_cigar) {
        roctxRangePushA("ta affine traceback");
        TA_HIP(ctx, ta::launch_affine_traceback(h.type, a, s));
        roctxRangePop();
    }
    return TA_OK;
}

int affine_exec(ta_affine_plan* pl, const ta_device_io* io, hipStream_t s, uint32_t chunk, bool fill, bool trace) {
    ta_context* ctx = pl->ctx;
    TA_HIP(ctx, hipSetDevice(ctx->device));
    if (int r = ta_host::stream_enter(ctx, s)) return r;
    const uint32_t c0 = chunk == UINT32_MAX ? 0 : chunk;
    const uint32_t c1 = chunk == UINT32_MAX ? (uint32_t)pl->h.chunks.size() : chunk + 1;
    for (uint32_t c = c0; c < c1; ++c)
        if (int r = affine_exec_chunk(pl, io, s, c, fill, trace)) return r;
    return ta_host::stream_leave(ctx, s);
}

struct AffineHostPlan final : ta_host::HostPlan {
    ta_affine_plan* pl;
    AffOffs o{};
    explicit AffineHostPlan(ta_affine_plan* p) : pl(p) {}
    void layout(ta::BlockLayout& L) override { o = aff_layout(pl->h, L); }
    void pack(uint8_t* base) override { aff_pack(pl->h, o, base); }
    void layout_device_only(ta::BlockLayout& L) override { aff_layout_scratch(pl->h, L, o); }
    void bind(uint8_t* dev) override { aff_bind(pl, dev, o); }
    int execute(const ta_device_io* io, hipStream_t s) override {
        return affine_exec(pl, io, s, UINT32_MAX, true, true);
    }
    uint64_t slots_bytes() const override { return pl->h.slots_bytes; }
    uint64_t err_offset() const override {
        return pl->h.duals.empty() && pl->h.single_tasks.empty() ? UINT64_MAX : o.err;
    }
    const char* err_message(uint32_t) const override {
        return "affine fill: a pass hand-off poll timed out; results of this batch are invalid";
    }
};

}  // namespace

extern "C" {

void ta_affine_plan_destroy(ta_affine_plan* pl) {
    if (!pl) return;
    if (pl->own_block) {
        (void)hipSetDevice(pl->ctx->device);
        (void)hipFree(pl->own_block);
    }
    delete pl;
}

int ta_affine_plan_create(ta_context* ctx, uint32_t n_pairs, const uint32_t* qlen, const uint32_t* tlen, int type,
                          int match, int mismatch, int gap_open, int gap_extend, int want_cigar, uint64_t budget,
                          uint32_t flags, ta_affine_plan** out) {
    if (!out) return TA_ERR_ARG;
    *out = nullptr;
    if (int r = affine_check_args(ctx, n_pairs, qlen, tlen, type, match, mismatch, gap_open, gap_extend)) return r;
    TA_HIP(ctx, hipSetDevice(ctx->device));
    auto* pl = new ta_affine_plan();
    pl->ctx = ctx;
    ta::build_affine_plan(pl->h, n_pairs, qlen, tlen, type, match, mismatch, gap_open, gap_extend, want_cigar != 0,
                          budget ? budget : ta_host::default_budget(ctx), flags, 4 * ctx->cu_count);
    ta::BlockLayout L;
    AffOffs o = aff_layout(pl->h, L);
    const uint64_t upload = L.bytes;
    aff_layout_scratch(pl->h, L, o);
    std::vector<uint8_t> host(upload);
    aff_pack(pl->h, o, host.data());
    hipError_t e = hipMalloc(&pl->own_block, std::max<uint64_t>(L.bytes, 256));
    if (e == hipSuccess) e = hipMemcpy(pl->own_block, host.data(), upload, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        ta_affine_plan_destroy(pl);
        return fail(ctx, TA_ERR_DEVICE, std::string("ta_affine_plan_create: ") + hipGetErrorString(e));
    }
    aff_bind(pl, static_cast<uint8_t*>(pl->own_block), o);
    *out = pl;
    return TA_OK;
}

uint64_t ta_affine_plan_cigar_slots_bytes(const ta_affine_plan* pl) { return pl ? pl->h.slots_bytes : 0; }

int ta_affine_plan_check(ta_affine_plan* pl) {
    if (!pl) return TA_ERR_ARG;
    if (pl->h.duals.empty() && pl->h.single_tasks.empty()) return TA_OK;
    uint32_t err = 0;
    TA_HIP(pl->ctx, hipSetDevice(pl->ctx->device));
    TA_HIP(pl->ctx, hipMemcpy(&err, pl->d_err, 4, hipMemcpyDeviceToHost));
    if (!err) return TA_OK;
    TA_HIP(pl->ctx, hipMemset(pl->d_err, 0, 4));
    return fail(pl->ctx, TA_ERR_DEVICE,
                "affine fill: a pass hand-off poll timed out; results of this plan are invalid");
}
uint64_t ta_affine_plan_workspace_bytes(const ta_affine_plan* pl) {
    return pl ? pl->h.ws_ptr_entries * sizeof(uint2) + pl->h.ws_bnd_entries * sizeof(int2) : 0;
}
uint32_t ta_affine_plan_chunks(const ta_affine_plan* pl) { return pl ? (uint32_t)pl->h.chunks.size() : 0; }
uint32_t ta_affine_plan_dual_pairs(const ta_affine_plan* pl) { return pl ? (uint32_t)pl->h.duals.size() : 0; }

int ta_affine_plan_pair_chunks(const ta_affine_plan* pl, uint32_t* chunk_of_pair) {
    if (!pl || !chunk_of_pair) return TA_ERR_ARG;
    for (uint32_t c = 0; c < (uint32_t)pl->h.chunks.size(); ++c) {
        const auto& ch = pl->h.chunks[c];
        for (uint32_t k = ch.begin; k < ch.begin + ch.count; ++k) chunk_of_pair[pl->h.order[k]] = c;
    }
    return TA_OK;
}

int ta_affine_plan_execute(ta_affine_plan* pl, const ta_device_io* io, void* stream) {
    if (int r = affine_check_io(pl, io)) return r;
    std::lock_guard<std::mutex> lock(pl->ctx->mu);
    return affine_exec(pl, io, (hipStream_t)stream, UINT32_MAX, true, true);
}

int ta_affine_plan_execute_fill(ta_affine_plan* pl, const ta_device_io* io, void* stream, uint32_t chunk) {
    if (int r = affine_check_io(pl, io)) return r;
    if (chunk >= pl->h.chunks.size()) return pl->h.n_pairs ? TA_ERR_ARG : TA_OK;
    std::lock_guard<std::mutex> lock(pl->ctx->mu);
    return affine_exec(pl, io, (hipStream_t)stream, chunk, true, false);
}

int ta_affine_plan_execute_traceback(ta_affine_plan* pl, const ta_device_io* io, void* stream, uint32_t chunk) {
    if (int r = affine_check_io(pl, io)) return r;
    if (chunk >= pl->h.chunks.size()) return pl->h.n_pairs ? TA_ERR_ARG : TA_OK;
    std::lock_guard<std::mutex> lock(pl->ctx->mu);
    return affine_exec(pl, io, (hipStream_t)stream, chunk, false, true);
}

int ta_align_batch_affine(ta_context* ctx, uint32_t n_pairs, const char* qb, const uint64_t* qoff,
                          const uint32_t* qlen, const char* tbytes, const uint64_t* toff, const uint32_t* tlen,
                          int type, int match, int mismatch, int gap_open, int gap_extend, int want_cigar,
                          int32_t* score, uint32_t* target_begin, char* arena, uint64_t arena_bytes,
                          uint64_t* cigar_off, uint32_t* cigar_len) {
    uint64_t qend = 0, tend = 0;
    if (int r = ta_host::check_host_batch(ctx, type, n_pairs, qb, qoff, qlen, tbytes, toff, tlen, want_cigar, arena,
                                          cigar_off, cigar_len, &qend, &tend))
        return r;
    if (n_pairs == 0) return TA_OK;
    if (int r = affine_check_args(ctx, n_pairs, qlen, tlen, type, match, mismatch, gap_open, gap_extend)) return r;
    std::lock_guard<std::mutex> lock(ctx->mu);
    TA_HIP(ctx, hipSetDevice(ctx->device));
    ta_affine_plan pl;
    pl.ctx = ctx;
    ta::build_affine_plan(pl.h, n_pairs, qlen, tlen, type, match, mismatch, gap_open, gap_extend, want_cigar != 0,
                          ta_host::batch_budget(ctx, n_pairs, qlen, tlen, want_cigar, sizeof(uint2)), 0,
                          4 * ctx->cu_count);
    AffineHostPlan hp(&pl);
    return ta_host::host_batch(ctx, hp, n_pairs, qb, qoff, qlen, tbytes, toff, tlen, qend, tend, want_cigar, score,
                               target_begin, arena, arena_bytes, cigar_off, cigar_len);
}

}  // extern "C"
