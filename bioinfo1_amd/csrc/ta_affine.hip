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

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/team_align_c.h"
#include "ta_context.h"
#include "ta_device.h"

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
};

// 64 boundary entries per chunk: column 64k+lane+1.
__device__ __forceinline__ int2 load_bchunk2(const int2* B, uint32_t m, uint32_t k, int lane) {
    const uint32_t j = k * 64u + (uint32_t)lane + 1u;
    return j <= m ? B[j] : make_int2(0, kNeg);
}

// One pass = rows row_base+1 .. row_base+nrows against the whole target.
//   QDASH  some query row of this pass is '-' (its vertical gap steps are free)
//   ROWSEL semi-global last pass whose row n is not the last register
template <int MODE, bool CIGAR, bool QDASH, bool ROWSEL>
__device__ __forceinline__ PassOut aff_pass(const AffArgs& a, const uint8_t* Q, const uint8_t* T, uint32_t n,
                                            uint32_t m, uint32_t pass, bool last_pass, uint2* ptrs, int2* B,
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
        bcur = load_bchunk2(B, m, 0, lane);
        bnext = load_bchunk2(B, m, 1, lane);
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
                bnext = load_bchunk2(B, m, (t >> 6) + 1, lane);
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
            if (has_next && (uint32_t)lane == nl - 1) B[j] = make_int2(H[R - 1], Flast);
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
                                                uint32_t m, uint32_t pass, bool last_pass, uint2* ptrs, int2* B,
                                                int lane) {
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
    if (widx >= a.count) return;  // wave-uniform
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
    int2* B = (passes > 1) ? a.bnd + a.bnd_off[p] : nullptr;

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
        if (!last_pass) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");  // boundary row -> next pass
    }
    if (lane == 0) {
        a.score[p] = (MODE == kGlobal) ? corner : best_h;
        a.target_begin[p] = (MODE == kLocal) ? best_j + 1 : 0;  // :117-121 / :197-199 / :283-285
        a.goal_i[p] = (MODE == kGlobal) ? n : best_i;
        a.goal_j[p] = (MODE == kGlobal) ? m : best_j;
    }
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
                w.push('M', 1);
                --i;
                --j;
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

inline dim3 aff_grid(uint32_t waves) { return dim3((waves + kWavesPerBlock - 1) / kWavesPerBlock); }

hipError_t launch_affine_fill(int mode, bool cigar, const AffArgs& a, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    const dim3 g = aff_grid(a.count), b(kBlock);
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
// Host driver.
struct ta_affine_plan {
    ta_context* ctx = nullptr;
    uint32_t n_pairs = 0;
    int type = 0, match = 0, mismatch = 0, open = 0, extend = 0;
    bool want_cigar = false;
    std::vector<uint32_t> order;  // pairs by descending cells: the big ones start first
    std::vector<uint64_t> ptr_off, bnd_off, slot_off;
    struct Chunk {
        uint32_t begin, count;  // plan order
        uint64_t ptr_entries, bnd_entries;
    };
    std::vector<Chunk> chunks;
    uint64_t slots_bytes = 0, ws_ptr_entries = 0, ws_bnd_entries = 0;
    uint32_t *d_qlen = nullptr, *d_tlen = nullptr, *d_order = nullptr, *d_goal_i = nullptr, *d_goal_j = nullptr;
    uint64_t *d_ptr_off = nullptr, *d_bnd_off = nullptr, *d_slot_off = nullptr;
};

namespace {

int afail(ta_context* ctx, int code, const std::string& msg) {
    if (ctx) ctx->last_error = msg;
    return code;
}

#define TA_AHIP(ctx, expr)                                                                            \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            return afail((ctx), TA_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <class T>
int aupload(ta_context* ctx, T** dptr, const std::vector<T>& v) {
    if (v.empty()) return TA_OK;
    TA_AHIP(ctx, hipMalloc(reinterpret_cast<void**>(dptr), v.size() * sizeof(T)));
    TA_AHIP(ctx, hipMemcpy(*dptr, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return TA_OK;
}

int agrow(ta_context* ctx, ta_context::Buf& b, size_t bytes) {
    if (bytes <= b.cap) return TA_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    const size_t want = std::max<size_t>(bytes, 4096);
    TA_AHIP(ctx, hipMalloc(&b.p, want));
    b.cap = want;
    return TA_OK;
}

uint64_t affine_default_budget(const ta_context* ctx) {
    if (const char* e = std::getenv("TA_WORKSPACE_BYTES")) return std::strtoull(e, nullptr, 10);
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return 48ull << 30;
    const uint64_t avail = (uint64_t)free_b + ctx->ws_ptrs.cap + ctx->ws_bnd.cap;
    return std::max<uint64_t>(avail / 100 * 85, 1ull << 30);
}

}  // namespace

extern "C" {

void ta_affine_plan_destroy(ta_affine_plan* pl) {
    if (!pl) return;
    (void)hipSetDevice(pl->ctx->device);
    for (void* p : {(void*)pl->d_qlen, (void*)pl->d_tlen, (void*)pl->d_order, (void*)pl->d_goal_i,
                    (void*)pl->d_goal_j, (void*)pl->d_ptr_off, (void*)pl->d_bnd_off, (void*)pl->d_slot_off})
        if (p) (void)hipFree(p);
    delete pl;
}

int ta_affine_plan_create(ta_context* ctx, uint32_t n_pairs, const uint32_t* qlen, const uint32_t* tlen, int type,
                          int match, int mismatch, int gap_open, int gap_extend, int want_cigar, uint64_t budget,
                          ta_affine_plan** out) {
    if (!ctx || !out || (n_pairs && (!qlen || !tlen))) return afail(ctx, TA_ERR_ARG, "null argument");
    *out = nullptr;
    if (type != TA_GLOBAL && type != TA_LOCAL && type != TA_SEMI_GLOBAL)
        return afail(ctx, TA_ERR_BAD_TYPE, ta_status_string(TA_ERR_BAD_TYPE));
    uint64_t maxn = 0, maxm = 0;
    for (uint32_t p = 0; p < n_pairs; ++p) {
        maxn = std::max<uint64_t>(maxn, qlen[p]);
        maxm = std::max<uint64_t>(maxm, tlen[p]);
    }
    // the oracle's range (oracle_affine_in_range): every |value| < 2^26
    const long long pm = std::max({std::llabs(match), std::llabs(mismatch),
                                   std::llabs(gap_open) + std::llabs(gap_extend)});
    if ((long long)(maxn + maxm + 2) * pm >= (1ll << 26))
        return afail(ctx, TA_ERR_RANGE, ta_status_string(TA_ERR_RANGE));
    TA_AHIP(ctx, hipSetDevice(ctx->device));
    auto* pl = new ta_affine_plan();
    pl->ctx = ctx;
    pl->n_pairs = n_pairs;
    pl->type = type;
    pl->match = match;
    pl->mismatch = mismatch;
    pl->open = gap_open;
    pl->extend = gap_extend;
    pl->want_cigar = want_cigar != 0;
    pl->order.resize(n_pairs);
    std::iota(pl->order.begin(), pl->order.end(), 0u);
    std::stable_sort(pl->order.begin(), pl->order.end(), [&](uint32_t x, uint32_t y) {
        return (uint64_t)qlen[x] * tlen[x] > (uint64_t)qlen[y] * tlen[y];
    });
    pl->slot_off.assign(n_pairs, 0);
    uint64_t so = 0;
    for (uint32_t p = 0; p < n_pairs; ++p) {
        pl->slot_off[p] = so;
        so += ta::cigar_slot_bytes(qlen[p], tlen[p]);
    }
    pl->slots_bytes = so;
    if (!budget) budget = affine_default_budget(ctx);
    const uint64_t budget_entries = std::max<uint64_t>(budget / sizeof(uint2), 1);
    pl->ptr_off.assign(n_pairs, 0);
    pl->bnd_off.assign(n_pairs, 0);
    ta_affine_plan::Chunk c{0, 0, 0, 0};
    for (uint32_t k = 0; k < n_pairs; ++k) {
        const uint32_t p = pl->order[k];
        const uint64_t pe = pl->want_cigar ? ta::ptr_dwords(qlen[p], tlen[p]) : 0;
        const uint64_t be = ta::bnd_words(qlen[p], tlen[p]);
        if (c.count && c.ptr_entries + pe > budget_entries) {
            pl->chunks.push_back(c);
            c = {k, 0, 0, 0};
        }
        pl->ptr_off[p] = c.ptr_entries;
        pl->bnd_off[p] = c.bnd_entries;
        c.ptr_entries += pe;
        c.bnd_entries += be;
        ++c.count;
    }
    if (c.count) pl->chunks.push_back(c);
    for (const auto& ch : pl->chunks) {
        pl->ws_ptr_entries = std::max(pl->ws_ptr_entries, ch.ptr_entries);
        pl->ws_bnd_entries = std::max(pl->ws_bnd_entries, ch.bnd_entries);
    }
    std::vector<uint32_t> ql(qlen, qlen + n_pairs), tl(tlen, tlen + n_pairs);
    int rc = TA_OK;
    auto up = [&](int r) {
        if (rc == TA_OK) rc = r;
    };
    up(aupload(ctx, &pl->d_qlen, ql));
    up(aupload(ctx, &pl->d_tlen, tl));
    up(aupload(ctx, &pl->d_order, pl->order));
    up(aupload(ctx, &pl->d_ptr_off, pl->ptr_off));
    up(aupload(ctx, &pl->d_bnd_off, pl->bnd_off));
    up(aupload(ctx, &pl->d_slot_off, pl->slot_off));
    if (rc == TA_OK && n_pairs) {
        hipError_t e = hipMalloc(&pl->d_goal_i, n_pairs * 4ull);
        if (e == hipSuccess) e = hipMalloc(&pl->d_goal_j, n_pairs * 4ull);
        if (e != hipSuccess) rc = afail(ctx, TA_ERR_DEVICE, hipGetErrorString(e));
    }
    if (rc != TA_OK) {
        ta_affine_plan_destroy(pl);
        return rc;
    }
    *out = pl;
    return TA_OK;
}

uint64_t ta_affine_plan_cigar_slots_bytes(const ta_affine_plan* pl) { return pl ? pl->slots_bytes : 0; }
uint64_t ta_affine_plan_workspace_bytes(const ta_affine_plan* pl) {
    return pl ? pl->ws_ptr_entries * sizeof(uint2) + pl->ws_bnd_entries * sizeof(int2) : 0;
}
uint32_t ta_affine_plan_chunks(const ta_affine_plan* pl) { return pl ? (uint32_t)pl->chunks.size() : 0; }

static int affine_check_io(ta_affine_plan* pl, const ta_device_io* io) {
    if (!pl || !io) return TA_ERR_ARG;
    if (pl->n_pairs && (!io->query_off || !io->target_off || !io->score || !io->target_begin))
        return afail(pl->ctx, TA_ERR_ARG, "null device pointer");
    if (pl->want_cigar && pl->n_pairs && (!io->cigar_slots || !io->cigar_start || !io->cigar_len))
        return afail(pl->ctx, TA_ERR_ARG, "null cigar device pointer");
    return TA_OK;
}

static int affine_exec_chunk(ta_affine_plan* pl, const ta_device_io* io, hipStream_t s, uint32_t c, bool fill,
                             bool trace) {
    ta_context* ctx = pl->ctx;
    TA_AHIP(ctx, hipSetDevice(ctx->device));
    if (int r = agrow(ctx, ctx->ws_ptrs, pl->ws_ptr_entries * sizeof(uint2))) return r;
    if (int r = agrow(ctx, ctx->ws_bnd, pl->ws_bnd_entries * sizeof(int2))) return r;
    const auto& ch = pl->chunks[c];
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
    a.match = pl->match;
    a.mismatch = pl->mismatch;
    a.open = pl->open;
    a.extend = pl->extend;
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
    if (fill) TA_AHIP(ctx, ta::launch_affine_fill(pl->type, pl->want_cigar, a, s));
    if (trace && pl->want_cigar) TA_AHIP(ctx, ta::launch_affine_traceback(pl->type, a, s));
    return TA_OK;
}

int ta_affine_plan_execute(ta_affine_plan* pl, const ta_device_io* io, void* stream) {
    if (int r = affine_check_io(pl, io)) return r;
    for (uint32_t c = 0; c < pl->chunks.size(); ++c)
        if (int r = affine_exec_chunk(pl, io, (hipStream_t)stream, c, true, true)) return r;
    return TA_OK;
}

int ta_affine_plan_execute_fill(ta_affine_plan* pl, const ta_device_io* io, void* stream, uint32_t chunk) {
    if (int r = affine_check_io(pl, io)) return r;
    if (chunk >= pl->chunks.size()) return pl->n_pairs ? TA_ERR_ARG : TA_OK;
    return affine_exec_chunk(pl, io, (hipStream_t)stream, chunk, true, false);
}

int ta_affine_plan_execute_traceback(ta_affine_plan* pl, const ta_device_io* io, void* stream, uint32_t chunk) {
    if (int r = affine_check_io(pl, io)) return r;
    if (chunk >= pl->chunks.size()) return pl->n_pairs ? TA_ERR_ARG : TA_OK;
    return affine_exec_chunk(pl, io, (hipStream_t)stream, chunk, false, true);
}

}  // extern "C"
