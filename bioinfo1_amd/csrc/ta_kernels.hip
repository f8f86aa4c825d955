// bioinfo1_amd/csrc/ta_kernels.hip -- gfx950 kernels for the team::Align path.
//
// What they compute is team::Align (/root/reference/team_alignment/
// team_alignment.cpp:49-350) for a batch of independent pairs:
//   fill      -- the (n+1)x(m+1) int32 DP of :102-116 / :171-194 / :249-264
//                (strict-> tie order MATCH > INSERT > DELETE, local clamp at 0,
//                '-' makes a gap free), the goal cell of :117-121 / :186-199 /
//                :265-285, the score and target_begin; with CIGAR on it also
//                writes a 2-bit traceback code per cell to HBM.
//   traceback -- the parent walk of :123-138 / :201-217 / :286-315 (incl. the
//                semi-global trailing I/D), run-length encoded (:145-160) into
//                the pair's CIGAR slot.
//   compact   -- packs the per-pair CIGAR slots back to back (host batches).
//
// How: one wave64 per pair.  Lane l owns 16 consecutive query
// rows ("stripe"); lanes sweep the target columns with a one-step lane skew
// (lane l is at column t-l+1 at step t), so each lane's row-0 "up" and
// "diag" neighbours are lane l-1's last row one and two steps earlier.  They
// move with one DPP wave_shr:1 per step -- no LDS, no shuffles through memory.
// Target characters enter at lane 0 and ride the same shift.  The pointer
// bits of a cell come from VALU compares whose wave-wide lane masks are
// combined on the SALU (canonical code M/I/D/STOP) and accumulated per lane,
// 16 rows x 2 bits = one dword per lane per step, stored as one coalesced
// 256-byte row per step.  Queries longer than 1024 rows take several passes;
// the bottom row of a pass is handed to the next through a boundary row in HBM.
#include <algorithm>
#include <cstdlib>

#include "ta_device.h"
#include "ta_walk2.h"
#include "ta_walk_lane.h"
#include "ta_walk_band.h"

namespace ta {
namespace {

#ifdef TA_FILL_MODE
// A pair's results, wave-uniform: score, target_begin, goal cell and (walked)
// its CIGAR's first byte in the pair's slot and its length.
struct PairOut {
    int score;
    uint32_t tb, gi, gj;
    uint64_t cstart;
    uint32_t clen;
};

// Degenerate pairs (an empty query or target): closed forms of what the
// reference computes when one of its loops is empty.
template <int MODE>
__device__ __forceinline__ PairOut degenerate(int gap, uint32_t n, uint32_t m) {
    PairOut o{0, 0, 0, 0, 0, 0};
    if (MODE == kGlobal) {  // :117-121 goal (n,m); boundary cost (n or m)*gap
        o.gi = n;
        o.gj = m;
        o.score = n ? wmul(n, gap) : wmul(m, gap);
    } else if (MODE == kLocal) {  // max never set: goal (0,0), tb = 0+1
        o.tb = 1;
    } else {  // :265-278: (0,m) wins the column scan (cost 0); row scan never beats it
        o.gi = 0;
        o.gj = (n == 0) ? m : 0;
    }
    return o;
}

// The pass boundary row.  A wave that sweeps all of a pair's passes itself
// keeps it in place (B: one int32 per column, rewritten by every pass).  In
// the pipelined fill (one wave per (pair, pass), fill_pipe_kernel) pass p's
// bottom row goes to 8-byte records tag << 32 | H in the pair's region, two
// buffers by pass parity, written with relaxed agent-scope stores; pass p + 1
// polls 64 columns at a time until every record carries the tag it expects
// (the data is its own flag, as ta_flex.hip / ta_dual.hip).
struct BndIo {
    int32_t* B;
    uint64_t* rec_w;        // null: B (or the last pass)
    const uint64_t* rec_r;  // null: B (or pass 0)
    uint32_t tag_w, tag_r;
    uint32_t* err;
};

typedef __attribute__((address_space(1))) unsigned long long gu64k;

// columns 64k + lane + 1 of the previous pass's bottom row
__device__ __forceinline__ int load_bnd(const BndIo& io, uint32_t m, uint32_t k, int lane) {
    if (!io.rec_r) return load_bchunk(io.B, m, k, lane);
    const uint32_t j = k * 64u + (uint32_t)lane + 1u;
    const gu64k* r = (const gu64k*)(io.rec_r + j);
    int v = 0;
    for (uint32_t spins = 0;; ++spins) {
        bool ok = true;
        if (j <= m) {
            const uint64_t x = __hip_atomic_load(r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = (uint32_t)(x >> 32) == io.tag_r;
            v = (int)(uint32_t)x;
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

// One pass = rows row_base+1 .. row_base+nrows of the query against the whole
// target.  Compile-time specialisation:
//   NV     valid rows of the last lane in use (every register index static);
//   QDASH  some query row of this pass is '-' (free vertical gap): the per-row
//          gap is then recomputed per cell, otherwise it is the uniform `gap`;
//   SCALED (local, |scores| < 2^25): each register holds V = 32*H + c_r with
//          c_r = 16 - r.  The recurrence is unchanged up to per-row offsets
//          folded into the constants (diag/up gain -1 per row, +15 into row 0
//          from the lane above's row 15), the clamp becomes max(.., c_r), and
//          V itself is the argmax key: larger H first, then the smaller row.
template <int MODE, bool CIGAR, bool WIDE, int NV, bool QDASH>
__device__ __forceinline__ PassOut run_pass(const FillArgs& a, const uint8_t* Q, const uint8_t* T, uint32_t n,
                                            uint32_t m, uint32_t pass, bool last_pass, uint32_t* ptrs,
                                            const BndIo& B, int lane) {
    constexpr int R = kRows;
    constexpr bool SCALED = (MODE == kLocal) && !WIDE;
    constexpr int SC = SCALED ? 32 : 1;
    const int gap = a.gap;
    // score constants for rows >= 1 (row 0 gets +16 on diag and up when SCALED)
    const int MA = SC * a.match - (SCALED ? 1 : 0);
    const int MI = SC * a.mismatch - (SCALED ? 1 : 0);
    const int UPG = SC * gap - (SCALED ? 1 : 0);   // up gain, query char != '-'
    const int UPD = SCALED ? -1 : 0;                 // up gain, query char == '-'
    const int GTG = SC * gap;                        // left gain, target char != '-'
    const int init = (MODE == kGlobal) ? gap : 0;    // :58-74 (local/semi boundaries are 0)
    const uint32_t Tmax = pass_steps(m);
    const uint32_t row_base = pass * kPassRows;
    const uint32_t nrows = min((uint32_t)kPassRows, n - row_base);
    const uint32_t nl = (nrows + R - 1) / R;  // lanes in use; lane nl-1 holds NV valid rows
    const bool has_next = !last_pass;

    uint32_t qp[R / 4];  // the lane's 16 query bytes, 4 per register (compared with SDWA byte selects)
    int H[R];
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
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i0 = row_base + (uint32_t)lane * R + r;  // row i0+1
        H[r] = SCALED ? (R - r) : wmul(i0 + 1, init);           // column 0, :83-86
    }
    int recv = SCALED ? 1 : wmul(row_base + (uint32_t)lane * R, init);  // H[row above the stripe][0]
    int tc = 0;
    const uint32_t nv_lane = (uint32_t)lane < nl - 1 ? R : ((uint32_t)lane == nl - 1 ? NV : 0);

    int bestkey = 0;                  // local SCALED: best V (0 = none: every real V >= 1)
    uint32_t bestj = 0;
    int bh = INT_MIN;                 // local WIDE: unpacked (h, r, j)
    uint32_t br = 0, bj = 0;
    int rowbest = INT_MIN;            // semi: row n
    uint32_t rowbest_j = 0;

    uint32_t tcur = load_tchunk(T, m, 0, lane), tnext = load_tchunk(T, m, 1, lane);
    int bcur = 0, bnext = 0;
    if (pass > 0) {
        bcur = load_bnd(B, m, 0, lane);
        bnext = load_bnd(B, m, 1, lane);
    }
    const uint32_t steps = m + nl - 1;
    uint32_t* prow = CIGAR ? ptrs + (uint64_t)pass * Tmax * kWave : nullptr;

    // One step = one target column per lane (lane l at column t-l+1).
    // MASKED steps (the ramp-up / ramp-down of the lane skew) run the cell
    // update under the per-lane `active` exec mask; in the steady state every
    // lane in use is active and lanes >= nl compute throw-away values, so
    // the update runs unmasked and H is updated in place.
    auto step = [&](uint32_t t, auto masked_tag) {
        constexpr bool MASKED = decltype(masked_tag)::value;
        if ((t & 255u) == 0 && t) {
            tcur = tnext;
            tnext = load_tchunk(T, m, (t >> 8) + 1, lane);
        }
        int top;
        if (pass == 0) {
            top = SCALED ? 1 : wmul(t + 1, init);  // row 0, :89-92
        } else {
            if ((t & 63u) == 0 && t) {
                bcur = bnext;
                bnext = load_bnd(B, m, (t >> 6) + 1, lane);
            }
            top = rdlane(bcur, t & 63u);
        }
        const uint32_t word = (uint32_t)rdlane((int)tcur, (t >> 2) & 63u);
        const int newc = (int)((word >> ((t & 3u) * 8)) & 0xFFu);
        const int prev = recv;
        recv = wave_shr1(top, H[R - 1]);
        tc = wave_shr1(newc, tc);

        const int j = (int)t - lane + 1;
        const bool active = !MASKED || (((uint32_t)lane < nl) & (j >= 1) & (j <= (int)m));
        uint32_t accD = 0, accI = 0;  // the two bit planes (ta_internal.h Code)
        if (active) {
            const int gt = (tc == '-') ? 0 : GTG;  // indel(t[j-1])
#pragma unroll
            for (int k = 0; k < R / 4; ++k) asm volatile("" : "+v"(qp[k]));  // keep bytes packed (SDWA compares)
            // match_func :20-23 for row r against this column's target byte
            auto score_of = [&](int r) {
                const uint32_t qb = (qp[r >> 2] >> (8 * (r & 3))) & 0xFFu;
                return (qb == (uint32_t)tc) ? MA : MI;
            };
            // diag of the next row is formed from old H[r] before h_r is
            // written, so h_r can take H[r]'s register (no rotation copies)
            int dnext = wadd(SCALED ? wadd(prev, 16) : prev, score_of(0));
            int upv = SCALED ? wadd(recv, 16) : recv;
            static_for<0, R>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                const int old = H[r];
                const int diag = dnext;
                const int left = wadd(old, gt);
                if constexpr (r + 1 < R) dnext = wadd(old, score_of(r + 1));
                int upg = UPG;  // indel(q[i-1])
                if (QDASH) upg = (((qp[r >> 2] >> (8 * (r & 3))) & 0xFFu) == (uint32_t)'-') ? UPD : UPG;
                const int up = wadd(upv, upg);
                const int m1 = max(diag, left);
                int h;
                if (MODE == kLocal) h = SCALED ? max3_imm<R - r>(m1, up) : max3_imm<0>(m1, up);  // clamp, :185
                else h = max(m1, up);
                if (CIGAR) {
                    // wave-wide lane masks from the VALU compares, shifted
                    // into the D and I planes (row 0 ends up in bit 15).
                    // Local mode canonicalises on the SALU:
                    //   D = D | S,  I = (I & !D) | S   (M=00 I=01 D=10 STOP=11)
                    const uint64_t mD = ballot(up > m1);      // DELETE only if strictly greater
                    const uint64_t mI = ballot(left > diag);  // INSERT beats MATCH only if strictly greater
                    uint64_t hi = mD, lo = mI;
                    if (MODE == kLocal) {
                        const uint64_t mS = ballot(h == (SCALED ? (R - r) : 0));  // cost 0 ends the walk
                        hi |= mS;
                        lo = (mI & ~mD) | mS;
                    }
                    accD = shl1_add_lanebit(accD, hi);
                    accI = shl1_add_lanebit(accI, lo);
                }
                if (MODE == kLocal && WIDE) {
                    if ((uint32_t)r < nv_lane && (h > bh || (h == bh && (uint32_t)r < br))) {
                        bh = h;
                        br = r;
                        bj = (uint32_t)j;
                    }
                }
                H[r] = h;
                upv = h;
            });
            if (SCALED) {
                // step key = max V over the lane's valid rows (prefix max chain)
                int P[R];
                P[0] = H[0];
#pragma unroll
                for (int r = 1; r < R; ++r) P[r] = max(P[r - 1], H[r]);
                int sk = P[R - 1];
                if (NV != R) sk = ((uint32_t)lane == nl - 1) ? P[NV - 1] : sk;
                if (sk > bestkey) {  // strict: the first column keeps a tie (:186)
                    bestkey = sk;
                    bestj = (uint32_t)j;
                }
            }
            if (MODE == kSemi && (NV != R || last_pass)) {
                // row n is register NV-1 of lane nl-1 in the last pass
                if (H[NV - 1] > rowbest) {
                    rowbest = H[NV - 1];
                    rowbest_j = (uint32_t)j;
                }
            }
            if (has_next && (uint32_t)lane == nl - 1) {
                if (B.rec_w)
                    __hip_atomic_store((gu64k*)(B.rec_w + j), ((uint64_t)B.tag_w << 32) | (uint32_t)H[R - 1],
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else
                    B.B[j] = H[R - 1];
            }
        }
        if (CIGAR) {
            const uint32_t code = (accD << kDPlane) | accI;
            // (blocked layout: the couples a blk plan's dual fill hands back; one
            // dword per lane 64 bytes apart, rare enough to need no staging)
            if (a.blk) ptrs[blk_index(pass, t, (uint32_t)lane, blk_count(m))] = code;
            else prow[t * kWave + lane] = code;
        }
    };
    // lanes 0..nl-1 are all active for t in [nl-1, m-1]
    const uint32_t ramp_end = min(nl - 1, steps);
    uint32_t t = 0;
    for (; t < ramp_end; ++t) step(t, std::true_type{});
    for (; t < m; ++t) step(t, std::false_type{});
    for (; t < steps; ++t) step(t, std::true_type{});

    PassOut o{INT_MIN, 0, 0, INT_MIN, 0, 0};
    if (MODE == kLocal) {
        const int v = (uint32_t)lane >= nl ? INT_MIN : (WIDE ? bh : (bestkey ? (bestkey >> 5) : -1));
        const int mx = wave_max(v);
        const int fl = first_lane(v == mx);
        uint32_t r, j;
        if (!WIDE) {
            r = R - ((uint32_t)rdlane(bestkey, fl) & 31u);
            j = (uint32_t)rdlane((int)bestj, fl);
        } else {
            r = (uint32_t)rdlane((int)br, fl);
            j = (uint32_t)rdlane((int)bj, fl);
        }
        o.h = mx;
        o.i = row_base + (uint32_t)fl * R + r + 1;
        o.j = j;
    } else if (MODE == kSemi) {
        // column m (H holds it now), i ascending, strict '>' (:265-270)
        int cv = INT_MIN;
        uint32_t cr = 0;
#pragma unroll
        for (int r = 0; r < R; ++r)
            if ((uint32_t)r < nv_lane && H[r] > cv) {
                cv = H[r];
                cr = r;
            }
        const int mx = wave_max(cv);
        const int fl = first_lane(cv == mx && nv_lane > 0);
        o.h = mx;
        o.i = row_base + (uint32_t)fl * R + (uint32_t)rdlane((int)cr, fl) + 1;
        o.j = m;
        if (last_pass) {
            o.row_h = rdlane(rowbest, nl - 1);
            o.row_j = (uint32_t)rdlane((int)rowbest_j, nl - 1);
        }
    } else {
        if (last_pass) o.corner = rdlane(select_row<R>(H, nrows - (nl - 1) * R - 1), nl - 1);  // row n
    }
    return o;
}

template <int MODE, bool CIGAR, bool WIDE, bool QDASH>
__device__ __forceinline__ PassOut run_pass_nv(const FillArgs& a, const uint8_t* Q, const uint8_t* T, uint32_t n,
                                               uint32_t m, uint32_t pass, bool last_pass, uint32_t* ptrs,
                                               const BndIo& B, int lane) {
    const uint32_t nrows = min((uint32_t)kPassRows, n - pass * kPassRows);
    const uint32_t nv = nrows - ((nrows + kRows - 1) / kRows - 1) * kRows;
    // Global needs NV only for the corner cell (read with a runtime select);
    // local/semi specialise the step loop on NV.
    // (WIDE tracks the argmax per row with a runtime row bound: no NV needed)
    if (MODE == kGlobal || (MODE == kLocal && WIDE) || nv == kRows)
        return run_pass<MODE, CIGAR, WIDE, kRows, QDASH>(a, Q, T, n, m, pass, last_pass, ptrs, B, lane);
#define TA_NV_CASE(k) \
    case k: return run_pass<MODE, CIGAR, WIDE, k, QDASH>(a, Q, T, n, m, pass, last_pass, ptrs, B, lane);
    switch (nv) {
        TA_NV_CASE(1) TA_NV_CASE(2) TA_NV_CASE(3) TA_NV_CASE(4) TA_NV_CASE(5) TA_NV_CASE(6) TA_NV_CASE(7)
        TA_NV_CASE(8) TA_NV_CASE(9) TA_NV_CASE(10) TA_NV_CASE(11) TA_NV_CASE(12) TA_NV_CASE(13) TA_NV_CASE(14)
        default: TA_NV_CASE(15)
    }
#undef TA_NV_CASE
}

template <int MODE, bool CIGAR, bool WIDE>
__device__ __forceinline__ PassOut run_pass_any(const FillArgs& a, const uint8_t* Q, const uint8_t* T, uint32_t n,
                                                uint32_t m, uint32_t pass, bool last_pass, uint32_t* ptrs,
                                                const BndIo& B, int lane) {
    // does any query row of this pass hold '-' (free vertical gap)?
    bool dash = false;
    const uint32_t row0 = pass * kPassRows + (uint32_t)lane * kRows;
#pragma unroll
    for (int r = 0; r < kRows; ++r) dash |= (row0 + r < n) && Q[row0 + r] == '-';
#ifndef TA_ANALYSIS_NODASH  // analysis builds: drop the dash variant to read the common loop
    if (__ballot(dash)) return run_pass_nv<MODE, CIGAR, WIDE, true>(a, Q, T, n, m, pass, last_pass, ptrs, B, lane);
#endif
    return run_pass_nv<MODE, CIGAR, WIDE, false>(a, Q, T, n, m, pass, last_pass, ptrs, B, lane);
}

// The fill of one n x m pair by one wave (all passes), its goal cell and,
// when `walk`, its walk into `slot` (cigar_slot_bytes(n, m) bytes).  Q, T:
// the sequences; ptrs: the pair's code workspace; B: its pass boundary row.
template <int MODE, bool CIGAR, bool WIDE>
__device__ __forceinline__ PairOut fill_one(const FillArgs& a, uint32_t n, uint32_t m, const uint8_t* Q,
                                            const uint8_t* T, uint32_t* ptrs, int32_t* Bw, char* slot, bool walk,
                                            int lane) {
    const WalkSeq seq0{Q, T, 0, a.match, a.mismatch, a.gap};
    if (n == 0 || m == 0) {
        PairOut o = degenerate<MODE>(a.gap, n, m);
        if (CIGAR && walk) {
            // no cells: the walk is the closed-form boundary run (global/semi) or "1\0"
            const uint32_t gi = (MODE == kGlobal) ? n : 0, gj = (MODE == kGlobal || n == 0) ? m : 0;
            traceback_pair<MODE>(nullptr, n, m, MODE == kLocal ? 0 : gi, MODE == kLocal ? 0 : gj, slot,
                                 cigar_slot_bytes(n, m), lane, &o.cstart, &o.clen, seq0);
        }
        return o;
    }
    const uint32_t passes = n_passes(n);
    const BndIo B{Bw, nullptr, nullptr, 0, 0, nullptr};
    // running goal over passes (wave-uniform); semi starts from (0,m), cost 0
    int best_h = (MODE == kSemi) ? 0 : INT_MIN;
    uint32_t best_i = 0, best_j = (MODE == kSemi) ? m : 0;
    int corner = 0;
    for (uint32_t pass = 0; pass < passes; ++pass) {
        const bool last_pass = pass + 1 == passes;
        const PassOut o = run_pass_any<MODE, CIGAR, WIDE>(a, Q, T, n, m, pass, last_pass, ptrs, B, lane);
        if (MODE != kGlobal && o.h > best_h) {  // strict: the earlier (upper) pass wins ties
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
        // the next pass reads this pass's bottom row (written by this wave)
        if (!last_pass) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
    PairOut o{(MODE == kGlobal) ? corner : best_h, (MODE == kLocal) ? best_j + 1 : 0u,  // :117-121 / :197-199 / :283-285
              (MODE == kGlobal) ? n : best_i, (MODE == kGlobal) ? m : best_j, 0, 0};
    if (CIGAR && walk) {
        // this wave's pointer stores -> its own loads in the walk
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const WalkSeq seq{Q, T, best_h, a.match, a.mismatch, a.gap};
        traceback_pair<MODE>(ptrs, n, m, o.gi, o.gj, slot, cigar_slot_bytes(n, m), lane, &o.cstart, &o.clen, seq);
    }
    return o;
}

// fill_one for pair p of a plan chunk: per-pair arrays in, per-pair arrays out.
template <int MODE, bool CIGAR, bool WIDE>
__device__ __forceinline__ void fill_pair(const FillArgs& a, uint32_t p, int lane) {
    const uint32_t n = a.qlen[p], m = a.tlen[p];
    const bool walk = CIGAR && a.fused;
    uint32_t* ptrs = (CIGAR && n && m) ? a.ptrs + a.ptr_off[p] : nullptr;
    int32_t* B = (n_passes(n) > 1) ? a.bnd + a.bnd_off[p] : nullptr;
    char* slot = walk ? a.slots + a.slot_off[p] : nullptr;
    const PairOut o = fill_one<MODE, CIGAR, WIDE>(a, n, m, a.qbytes + a.qoff[p], a.tbytes + a.toff[p], ptrs, B, slot,
                                                  walk, lane);
    if (lane == 0) {
        a.score[p] = o.score;
        a.target_begin[p] = o.tb;
        a.goal_i[p] = o.gi;
        a.goal_j[p] = o.gj;
        if (walk) {
            a.cigar_start[p] = a.slot_off[p] + o.cstart;
            a.cigar_len[p] = o.clen;
        }
    }
}

template <int MODE, bool CIGAR, bool WIDE>
__global__ __launch_bounds__(kBlock) void fill_kernel(FillArgs a) {
    const int lane = threadIdx.x & 63;
    const uint32_t widx = wave_id();
    if (widx >= (a.count_dev ? *a.count_dev : a.count)) return;  // wave-uniform
    fill_pair<MODE, CIGAR, WIDE>(a, a.order ? a.order[a.begin + widx] : a.begin + widx, lane);
}

// The pipelined int32 fill: one wave per (pair, pass) of a chunk's singles
// (order = the plan's singles).  A wave takes the next ticket; the tasks are
// pass-major (every pair's pass 0, then every pass 1, ...; the planner's
// single_tasks), so pass p - 1 of its pair belongs to a wave that took an
// earlier ticket and is running: every poll ends.  The walk runs in the
// traceback kernel after fill_combine_kernel has folded the passes.
template <int MODE, bool CIGAR, bool WIDE>
__global__ __launch_bounds__(kBlock) void fill_pipe_kernel(FillArgs a) {
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
    uint64_t* rec = reinterpret_cast<uint64_t*>(a.bnd + a.bnd_off[p]);  // 2 buffers x (m + 1) records
    const uint64_t rb = (uint64_t)m + 1;
    // tags: pass + 1 for pass p's row (never 0; the host zeroes the records before the launch)
    const BndIo B{nullptr, last_pass ? nullptr : rec + (pass & 1u) * rb, pass ? rec + ((pass - 1u) & 1u) * rb : nullptr,
                  pass + 1u, pass, a.err};
    uint32_t* ptrs = CIGAR ? a.ptrs + a.ptr_off[p] : nullptr;
    const PassOut o = run_pass_any<MODE, CIGAR, WIDE>(a, a.qbytes + a.qoff[p], a.tbytes + a.toff[p], n, m, pass,
                                                      last_pass, ptrs, B, lane);
    if (lane == 0) static_cast<PassOut*>(a.pout)[a.task_off[w] + pass] = o;
}

// After the pipelined fill: fold each pair's per-pass results in pass order
// as fill_one does (the upper pass wins ties; semi: row n after column m).
template <int MODE>
__global__ void fill_combine_kernel(FillArgs a) {
    const uint32_t w = a.begin + blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= a.begin + a.count) return;
    const uint32_t p = a.order[w];
    const uint32_t n = a.qlen[p], m = a.tlen[p];
    PairOut r;
    if (n == 0 || m == 0) {
        r = degenerate<MODE>(a.gap, n, m);
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
        r = PairOut{(MODE == kGlobal) ? corner : best_h, (MODE == kLocal) ? best_j + 1 : 0u,
                    (MODE == kGlobal) ? n : best_i, (MODE == kGlobal) ? m : best_j, 0, 0};
    }
    a.score[p] = r.score;
    a.target_begin[p] = r.tb;
    a.goal_i[p] = r.gi;
    a.goal_j[p] = r.gj;
}

#if TA_FILL_CIGAR
// ---- the low-latency server (ta_internal.h ServeArgs; host side ta_server.cpp)
// A relaxed system-scope load (bypasses the GPU caches; no cache invalidation):
// the poll reads with it, and one acquire fence follows a detected request.
__device__ __forceinline__ uint32_t sys_load(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- small pairs: R = 1, 2 or 4 query rows per lane (n <= 64R), all in LDS.
// The batch fill gives a lane 16 rows; for one lone pair that makes every step
// a 16-row dependent chain on an otherwise idle CU (a 5x9 pair: ~11 us of fill
// and walk, 200x200 ~170 us).  Here lane l owns rows lR + 1 .. lR + R and steps
// along the anti-diagonals (lane l at column t - l + 1 at step t; up and diag
// of its first row arrive from lane l - 1's last row by DPP wave_shr:1 as in
// the batch fill), with the reference's int32 cell rule verbatim
// (team_alignment.cpp:102-116 / :172-194 / :250-263: strict '>' in the order
// MATCH, INSERT, DELETE; '-' free gaps; the local clamp and first strict
// row-major maximum; the semi-global column-m then row-n goal).  Codes: 2 bits
// per cell (M 0, I 1, D 2, local cost 0 = STOP 3), 16 / R steps per dword,
// [step / (16 / R)][lane] in LDS.  The walk (:123-138, :201-217, :286-315) runs
// on uniform values reading LDS, the RLE is formatted lane-parallel (:145-160,
// "1\0" for an empty op string) and goes straight into the host slot.
constexpr uint32_t kSmallQ = 256, kSmallT = 1024;
constexpr uint32_t kSmallCodeDw = 68 * kWave;  // (steps x R) / 16 dwords per lane <= 68
struct SmallLds {
    uint32_t codes[kSmallCodeDw];
    uint32_t runs[kSmallT + 64 + 4];  // at most n + m runs (n + m <= 1,088 for every admitted shape)
    uint8_t q[kSmallQ];
    uint8_t t[kSmallT];
    char text[2 * (kSmallT + 64) + 16];
};
// Rows per lane for an n x m pair (0: not a small pair): the fewest with
// n <= 64R whose codes fit (m + ceil(n / R) - 1) * R <= 1,088.
__device__ __forceinline__ uint32_t small_rows(uint32_t n, uint32_t m) {
    if (n == 0 || m == 0 || m > kSmallT) return 0;
    for (uint32_t R = 1; R <= 4; R <<= 1)
        if (n <= 64u * R && (m + (n + R - 1) / R - 1) * R <= 16u * 68u) return R;
    return 0;
}

template <int MODE, int R>
__device__ __forceinline__ PairOut serve_small(const FillArgs& a, uint32_t n, uint32_t m, bool want, SmallLds& L,
                                               char* out_text, int lane) {
    constexpr uint32_t SPD = 16 / R;  // steps per code dword
    const int ma = a.match, mi = a.mismatch, gap = a.gap;
    const int init = (MODE == kGlobal) ? gap : 0;  // :62-74
    const uint32_t l = (uint32_t)lane;
    const uint32_t nl = (n + R - 1) / R;  // lanes in use
    uint32_t qb[R];
    int upg[R], H[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i0 = l * R + r;  // row i0 + 1
        qb[r] = L.q[min(i0, n - 1u)];
        upg[r] = (qb[r] == (uint32_t)'-') ? 0 : gap;  // indel(query[i-1]), :25-28
        H[r] = wmul(i0 + 1u, init);                    // H(i, 0), :83-86; kept while the lane is idle
    }
    int recv = 0;  // lane 0's first diag is H(0, 0) = 0
    // local: the lane's best cell (row-major first: larger h, then smaller row, then smaller j)
    int bh = INT_MIN, rb = INT_MIN;
    uint32_t br = 0, bj = 0, rbj = 0, acc = 0;
    const uint32_t rn = (n - 1u) % R;  // row n's register in lane (n - 1) / R
    const uint32_t steps = m + nl - 1u;
    uint32_t tnext = L.t[min(0u - l, m - 1u) & 0x3FFu];
    for (uint32_t t = 0; t < steps; ++t) {
        int dg = recv;                                // H(row above, j - 1)
        recv = wave_shr1(wmul(t + 1u, init), H[R - 1]);  // H(row above, j); lane 0: row 0, :89-92
        const uint32_t tb = tnext;
        tnext = L.t[min(t + 1u - l, m - 1u) & 0x3FFu];  // next column's target byte (clamped, unused when idle)
        const int j = (int)t - lane + 1;
        uint32_t c4 = 0;
        if (l < nl && j >= 1 && j <= (int)m) {
            int up_in = recv;
            const int lg = tb == (uint32_t)'-' ? 0 : gap;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t i0 = l * R + r;
                const int old = H[r];
                if (i0 < n) {
                    const int diag = wadd(dg, qb[r] == tb ? ma : mi);  // match_func, :20-23
                    const int left = wadd(old, lg);
                    const int up = wadd(up_in, upg[r]);
                    int h = diag;
                    uint32_t c = 0;
                    if (left > h) {
                        h = left;
                        c = 1;
                    }
                    if (up > h) {
                        h = up;
                        c = 2;
                    }
                    if (MODE == kLocal) {
                        if (h < 0) h = 0;  // :185
                        if (h == 0) c = 3;  // the walk stops here (:202)
                        if (h > bh || (h == bh && (uint32_t)r < br)) {  // :186 in row-major order
                            bh = h;
                            br = r;
                            bj = (uint32_t)j;
                        }
                    }
                    if (MODE == kSemi && i0 == n - 1u && h > rb) {  // row n, :272-278
                        rb = h;
                        rbj = (uint32_t)j;
                    }
                    H[r] = h;
                    c4 |= c << (2u * r);
                }
                dg = old;  // the next row's diag: this row's value one column left
                up_in = H[r];
            }
        }
        acc |= c4 << (2u * R * (t % SPD));
        if (t % SPD == SPD - 1u || t + 1u == steps) {
            L.codes[(t / SPD) * kWave + l] = acc;
            acc = 0;
        }
    }
    PairOut o{0, 0, n, m, 0, 0};
    if (MODE == kGlobal) {
        int hn = H[0];
#pragma unroll
        for (int r = 1; r < R; ++r) hn = ((uint32_t)r == rn) ? H[r] : hn;
        o.score = rdlane(hn, (n - 1u) / R);  // H(n, m)
    } else if (MODE == kLocal) {
        // best h, then the smallest row: lanes hold ascending rows
        const int mx = wave_max(l < nl ? bh : INT_MIN);
        const int fl = first_lane(l < nl && bh == mx);
        o.score = mx;
        o.gi = (uint32_t)fl * R + (uint32_t)rdlane((int)br, (uint32_t)fl) + 1u;
        o.gj = (uint32_t)rdlane((int)bj, (uint32_t)fl);
        o.tb = o.gj + 1u;  // :197-199
    } else {
        // column m from row 0 (cost 0), strict '>' (:265-271), then row n (:272-278)
        int cv = INT_MIN;
        uint32_t cr = 0;
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (l * R + r < n && H[r] > cv) {
                cv = H[r];
                cr = r;
            }
        const int mx = wave_max(cv);
        int best = 0;
        o.gi = 0;
        o.gj = m;
        if (mx > best) {
            best = mx;
            const int fl = first_lane(cv == mx);
            o.gi = (uint32_t)fl * R + (uint32_t)rdlane((int)cr, (uint32_t)fl) + 1u;
        }
        const int rbv = rdlane(rb, (n - 1u) / R);
        if (rbv > best) {
            best = rbv;
            o.gi = n;
            o.gj = (uint32_t)rdlane((int)rbj, (n - 1u) / R);
        }
        o.score = best;
    }
    if (!want) return o;
    __syncthreads();  // the code dwords of every lane
    // the walk, end to start (uniform; LDS broadcast reads), as runs (op | count << 2)
    uint32_t nr = 0, op = 4u, cnt = 0;
    auto push = [&](uint32_t o2, uint32_t k) {
        if (o2 == op) {
            cnt += k;
        } else {
            if (cnt) L.runs[nr++] = op | (cnt << 2);
            op = o2;
            cnt = k;
        }
    };
    uint32_t i = o.gi, jj = o.gj;
    if (MODE == kSemi && (jj != m || i != n)) {  // the trailing I / D of :306-315 end the string
        if (i == n) push(1u, m - jj);
        else if (jj == m) push(2u, n - i);
    }
    auto code_at = [&](uint32_t ci, uint32_t cj) {
        const uint32_t ln = (ci - 1u) / R, r = (ci - 1u) % R, st = cj + ln - 1u;
        return (L.codes[(st / SPD) * kWave + ln] >> (2u * (R * (st % SPD) + r))) & 3u;
    };
    if (MODE == kLocal) {
        while (i >= 1u && jj >= 1u) {  // cost > 0 (boundary cells cost 0)
            const uint32_t c = code_at(i, jj);
            if (c == 3u) break;
            push(c, 1u);
            i -= (c != 1u) ? 1u : 0u;
            jj -= (c != 2u) ? 1u : 0u;
        }
    } else {
        while (i > 0u || jj > 0u) {
            if (i == 0u) {  // row 0: parent INSERT (:88-92)
                push(1u, jj);
                break;
            }
            if (jj == 0u) {  // column 0: parent DELETE (:82-86)
                push(2u, i);
                break;
            }
            const uint32_t c = code_at(i, jj);
            push(c, 1u);
            i -= (c != 1u) ? 1u : 0u;
            jj -= (c != 2u) ? 1u : 0u;
        }
    }
    if (cnt) L.runs[nr++] = op | (cnt << 2);
    // RLE text, forward order = the runs in reverse, 64 runs per round
    uint32_t used = 0;
    if (nr == 0) {
        if (lane == 0) {
            L.text[0] = '1';
            L.text[1] = '\0';
        }
        used = 2;
    }
    for (uint32_t base = 0; base < nr; base += 64u) {
        const uint32_t f = base + l;
        const bool act = f < nr;
        const uint32_t v = act ? L.runs[nr - 1u - f] : 0u;
        uint32_t c = v >> 2;
        const uint32_t digits = 1u + (c >= 10u) + (c >= 100u) + (c >= 1000u) + (c >= 10000u);
        const uint32_t len = act ? digits + 1u : 0u;
        uint32_t incl = len;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, d, 64);
            if (lane >= d) incl += y;
        }
        if (act) {
            char* p = L.text + used + incl - len;
            for (int d = (int)digits - 1; d >= 0; --d) {
                p[d] = (char)('0' + c % 10u);
                c /= 10u;
            }
            p[digits] = (char)((0x44494Du >> (8u * (v & 3u))) & 0xFFu);  // 'M', 'I', 'D'
        }
        used += (uint32_t)__shfl((int)incl, 63, 64);
    }
    __syncthreads();
    for (uint32_t k = l; k < used; k += 64u) out_text[k] = L.text[k];
    o.clen = used;
    return o;
}

// One request of slot s: copy the bytes into HBM, fill + walk, results back.
// The request header and the first KB of each sequence come in one round trip
// over PCIe (lanes 0-5 the header words, the others query bytes; a second load
// per lane the target); longer sequences follow in a second round.  Small
// pairs stay in LDS (serve_small).
template <int MODE>
__device__ __forceinline__ void serve_one(const ServeArgs& sa, uint32_t s, char* slot, uint32_t seq, int lane,
                                          uint64_t t0, SmallLds& L) {
    ServeHdr* hd = reinterpret_cast<ServeHdr*>(slot);
    const uint32_t* req = reinterpret_cast<const uint32_t*>(slot);
    const FillArgs& fa = sa.fa;
    uint8_t* dq = const_cast<uint8_t*>(fa.qbytes) + (uint64_t)s * kSrvQMax;
    uint8_t* dt = const_cast<uint8_t*>(fa.tbytes) + (uint64_t)s * kSrvTMax;
    // lanes 0-5: words 1..6 (n, m, match, mismatch, gap, want_cigar); lanes 6-63: query bytes [0, 928)
    uint4 qv = make_uint4(0, 0, 0, 0), tv;
    uint32_t w = 0;
    if (lane < 6) w = sys_load(req + 1 + lane);
    else qv = *reinterpret_cast<const uint4*>(slot + kSrvQOff + 16u * (uint32_t)(lane - 6));
    tv = *reinterpret_cast<const uint4*>(slot + kSrvTOff + 16u * (uint32_t)lane);  // target bytes [0, 1024)
    const uint32_t n = (uint32_t)rdlane((int)w, 0), m = (uint32_t)rdlane((int)w, 1);
    FillArgs a = fa;
    a.match = rdlane((int)w, 2);
    a.mismatch = rdlane((int)w, 3);
    a.gap = rdlane((int)w, 4);
    const bool want = rdlane((int)w, 5) != 0;
    uint64_t t1 = t0, t2 = t0;  // phase clocks (100 MHz): request + bytes into HBM, fill + walk
    uint32_t status = TA_OK;
    PairOut o{0, 0, 0, 0, 0, 0};
    char* cslot = a.slots + (uint64_t)s * ((cigar_slot_bytes(kSrvQMax, kSrvTMax) + 255) & ~255ull);
    if (n > kSrvQMax || m > kSrvTMax) {
        status = TA_ERR_ARG;  // (the host never posts such a pair)
    } else if (const uint32_t R = small_rows(n, m)) {
        if (lane >= 6 && lane < 6 + (int)(kSmallQ / 16)) *reinterpret_cast<uint4*>(L.q + 16u * (uint32_t)(lane - 6)) = qv;
        *reinterpret_cast<uint4*>(L.t + 16u * (uint32_t)lane) = tv;
        __syncthreads();
        t1 = wall_clock64();
        if (R == 1) o = serve_small<MODE, 1>(a, n, m, want, L, slot + kSrvCOff, lane);
        else if (R == 2) o = serve_small<MODE, 2>(a, n, m, want, L, slot + kSrvCOff, lane);
        else o = serve_small<MODE, 4>(a, n, m, want, L, slot + kSrvCOff, lane);
        t2 = wall_clock64();
    } else {
        if (lane >= 6) *reinterpret_cast<uint4*>(dq + 16u * (uint32_t)(lane - 6)) = qv;
        *reinterpret_cast<uint4*>(dt + 16u * (uint32_t)lane) = tv;
        for (uint32_t k = 928u + 16u * (uint32_t)lane; k < n; k += 1024u)
            *reinterpret_cast<uint4*>(dq + k) = *reinterpret_cast<const uint4*>(slot + kSrvQOff + k);
        for (uint32_t k = 1024u + 16u * (uint32_t)lane; k < m; k += 1024u)
            *reinterpret_cast<uint4*>(dt + k) = *reinterpret_cast<const uint4*>(slot + kSrvTOff + k);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // this wave's stores -> its own loads
        t1 = wall_clock64();
        uint32_t* ptrs = fa.ptrs + (uint64_t)s * ptr_dwords(kSrvQMax, kSrvTMax);
        int32_t* B = fa.bnd + (uint64_t)s * bnd_words(kSrvQMax, kSrvTMax);
        o = fill_one<MODE, true, false>(a, n, m, dq, dt, ptrs, B, cslot, want, lane);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        t2 = wall_clock64();
        if (want)
            for (uint32_t k = (uint32_t)lane; k < o.clen; k += 64u) slot[kSrvCOff + k] = cslot[o.cstart + k];
    }
    const uint64_t t3 = wall_clock64();
    if (lane == 0) {
        hd->score = o.score;
        hd->target_begin = o.tb;
        hd->cigar_len = want ? o.clen : 0u;
        hd->status = status;
        hd->pad1[0] = (uint32_t)(t1 - t0);  // diagnostics (ta_server_last_times), 10 ns units
        hd->pad1[1] = (uint32_t)(t2 - t1);
        hd->pad1[2] = (uint32_t)(t3 - t2);
    }
    // `done` by a system-scope release store: the results and CIGAR bytes (this
    // wave's earlier stores) are visible to the host before it -- one fence (a
    // separate __threadfence_system before it cost ~1.3 µs on top)
    if (lane == 0) hd->pad1[3] = 0u;
    if (lane == 0) __hip_atomic_store(&hd->done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One wave per slot (block).  Polls its slot's `seq`, the stop flag and the
// heartbeat in one round trip; exits on stop, or when the heartbeat has not
// moved for hb_timeout (the host process is gone or hung): every wave ends.
template <int MODE>
__global__ __launch_bounds__(kWave) void serve_kernel(ServeArgs sa) {
    const int lane = (int)threadIdx.x;
    const uint32_t s = blockIdx.x;
    char* slot = sa.host + (uint64_t)s * kSrvStride;
    const uint32_t* seqp = reinterpret_cast<const uint32_t*>(slot);
    __shared__ SmallLds lds;
    // resume from the last finished request: one posted while no kernel ran is served now
    uint32_t last = (uint32_t)rdlane((int)(lane == 0 ? sys_load(&reinterpret_cast<const ServeHdr*>(slot)->done) : 0u), 0);
    uint32_t hb_last = 0;
    uint64_t t_hb = wall_clock64();
    for (;;) {
        const uint32_t v = lane == 0 ? sys_load(seqp)
                                     : (lane == 1 ? sys_load(&sa.ctl->stop)
                                                  : (lane == 2 ? sys_load(&sa.ctl->heartbeat) : 0u));
        const uint32_t seq = (uint32_t)rdlane((int)v, 0), stop = (uint32_t)rdlane((int)v, 1),
                       hb = (uint32_t)rdlane((int)v, 2);
        if (seq != last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the request's bytes were written before seq
            serve_one<MODE>(sa, s, slot, seq, lane, wall_clock64(), lds);
            last = seq;
            t_hb = wall_clock64();
            continue;
        }
        if (stop) break;
        const uint64_t now = wall_clock64();
        if (hb != hb_last) {
            hb_last = hb;
            t_hb = now;
        } else if (now - t_hb > sa.hb_timeout) {
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}
#endif  // TA_FILL_CIGAR

#endif  // TA_FILL_MODE

#ifdef TA_TU_MISC
template <int MODE>
#ifndef TA_TB_WPE
#define TA_TB_WPE 8  // waves per SIMD the traceback kernel is compiled for
#endif
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(TA_TB_WPE))) void traceback_kernel(TraceArgs a) {
    // Wave-strided over the pairs (one wave per pair: the grid covers them all).
    const int lane = threadIdx.x & 63;
    const uint32_t stride = gridDim.x * kWavesPerBlock;
    for (uint32_t widx = wave_id(); widx < a.count; widx += stride) {
        const uint32_t p = a.order ? a.order[a.begin + widx] : a.begin + widx;
        const uint32_t n = a.qlen[p], m = a.tlen[p];
        uint64_t st;
        uint32_t len;
        const WalkSeq seq{a.qbytes + a.qoff[p], a.tbytes + a.toff[p], MODE == kLocal ? a.score[p] : 0, a.match,
                          a.mismatch, a.gap};
        traceback_pair<MODE>(a.ptrs + a.ptr_off[p], n, m, a.goal_i[p], a.goal_j[p], a.slots + a.slot_off[p],
                             cigar_slot_bytes(n, m), lane, &st, &len, seq, a.blk != 0);
        if (lane == 0) {
            a.cigar_start[p] = a.slot_off[p] + st;
            a.cigar_len[p] = len;
        }
    }
}

// Local walks, 64/G pairs per wave (ta_walk2.h).
template <int G>
__global__ __launch_bounds__(kBlock) void traceback_group_kernel(TraceArgs a) {
    const uint32_t widx = wave_id();
    if ((64u / G) * widx >= a.count) return;
    traceback_group_local<G>(a, widx, threadIdx.x & 63);
}

// Local walks, one lane per pair stepping cell by cell, 64/G pairs per
// one-wave block (ta_walk_lane.h).
template <int G>
__global__ __launch_bounds__(kWave) void traceback_lane_kernel(TraceArgs a) {
    __shared__ uint32_t lds[(64 / G) * kLwGroupDw];
    traceback_lane_local<G>(a, lds, (int)threadIdx.x);
}

// Local walks of blocked-layout plans, one lane per pair, 64 per one-wave
// block (ta_walk_band.h).
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(1, 1))) void traceback_band_kernel(TraceArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kWave * kBwRegion + kBwStageBytes];
    const int lane = (int)threadIdx.x;
    traceback_band_local(a, lds, lane);
    // then the pairs the dual fill handed back ('-' bytes; usually none), one
    // wave per pair in the one-pair walk over the blocked layout -- here rather
    // than in a launch of its own, whose count only the device knows
    if (a.fb_count) {
        const uint32_t nfb = *a.fb_count;
        for (uint32_t w = blockIdx.x; w < nfb; w += gridDim.x) {
            const uint32_t p = a.fb_order[w];
            const uint32_t n = a.qlen[p], m = a.tlen[p];
            uint64_t st;
            uint32_t len;
            const WalkSeq seq{a.qbytes + a.qoff[p], a.tbytes + a.toff[p], a.score[p], a.match, a.mismatch, a.gap};
            traceback_pair<kLocal>(a.ptrs + a.ptr_off[p], n, m, a.goal_i[p], a.goal_j[p], a.slots + a.slot_off[p],
                                   cigar_slot_bytes(n, m), lane, &st, &len, seq, true);
            if (lane == 0) {
                a.cigar_start[p] = a.slot_off[p] + st;
                a.cigar_len[p] = len;
            }
        }
    }
}

// ... and their runs into CIGAR text, one wave per pair.
__global__ __launch_bounds__(kBlock) void format_runs_kernel(TraceArgs a) {
    const uint32_t w = wave_id();
    if (w >= a.count) return;
    format_runs(a, a.order ? a.order[a.begin + w] : a.begin + w, threadIdx.x & 63);
}

__global__ __launch_bounds__(kBlock) void compact_kernel(CompactArgs a) {
    const int lane = threadIdx.x & 63;
    const uint32_t p = wave_id();
    if (p >= a.n_pairs) return;
    const char* src = a.slots + a.cigar_start[p];
    char* dst = a.dst + a.dst_off[p];
    const uint32_t len = a.cigar_len[p];
    for (uint32_t k = (uint32_t)lane; k < len; k += 64u) dst[k] = src[k];
}

#endif  // TA_TU_MISC

inline dim3 grid_for(uint32_t waves) { return dim3((waves + kWavesPerBlock - 1) / kWavesPerBlock); }

}  // namespace

// Each fill mode is its own translation unit (build.sh compiles this file
// once per TA_FILL_MODE in parallel); TA_TU_MISC holds the rest.
#ifdef TA_FILL_MODE
// One translation unit per (mode, cigar) pair: build.sh compiles this file
// six times in parallel with -DTA_FILL_MODE=m -DTA_FILL_CIGAR=c.
template <>
hipError_t launch_fill_mode<TA_FILL_MODE, (TA_FILL_CIGAR != 0)>(bool wide, const FillArgs& a, hipStream_t s) {
    constexpr int MODE = TA_FILL_MODE;
    constexpr bool CIGAR = TA_FILL_CIGAR != 0;
    if (!a.count) return hipSuccess;
    const dim3 g = grid_for(a.count), b(kBlock);
    if (a.tasks64) {  // one wave per (pair, pass), then the fold of the passes
        if (a.n_tasks) {
            const dim3 gt = grid_for(a.n_tasks);
            if (MODE == kLocal && wide) hipLaunchKernelGGL((fill_pipe_kernel<MODE, CIGAR, MODE == kLocal>), gt, b, 0, s, a);
            else hipLaunchKernelGGL((fill_pipe_kernel<MODE, CIGAR, false>), gt, b, 0, s, a);
        }
        hipLaunchKernelGGL(fill_combine_kernel<MODE>, dim3((a.count + 255) / 256), dim3(256), 0, s, a);
        return hipGetLastError();
    }
    // WIDE only changes the local argmax; other modes use one instantiation.
    if (MODE == kLocal && wide) hipLaunchKernelGGL((fill_kernel<MODE, CIGAR, MODE == kLocal>), g, b, 0, s, a);
    else hipLaunchKernelGGL((fill_kernel<MODE, CIGAR, false>), g, b, 0, s, a);
    return hipGetLastError();
}
#if TA_FILL_CIGAR
template <>
hipError_t launch_serve_mode<TA_FILL_MODE>(const ServeArgs& a, uint32_t slots, hipStream_t s) {
    hipLaunchKernelGGL(serve_kernel<TA_FILL_MODE>, dim3(slots), dim3(kWave), 0, s, a);
    return hipGetLastError();
}
#endif
#endif

#ifdef TA_TU_MISC
#ifndef TA_LW_G
#define TA_LW_G 16
#endif
hipError_t launch_fill(int mode, bool cigar, bool wide, const FillArgs& a, hipStream_t s) {
    switch (mode * 2 + (cigar ? 1 : 0)) {
        case 0: return launch_fill_mode<kGlobal, false>(wide, a, s);
        case 1: return launch_fill_mode<kGlobal, true>(wide, a, s);
        case 2: return launch_fill_mode<kLocal, false>(wide, a, s);
        case 3: return launch_fill_mode<kLocal, true>(wide, a, s);
        case 4: return launch_fill_mode<kSemi, false>(wide, a, s);
        case 5: return launch_fill_mode<kSemi, true>(wide, a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_dual(int mode, bool cigar, const FillArgs& a, hipStream_t s) {
    switch (mode * 2 + (cigar ? 1 : 0)) {
        case 0: return launch_dual_mode<kGlobal, false>(a, s);
        case 1: return launch_dual_mode<kGlobal, true>(a, s);
        case 2: return launch_dual_mode<kLocal, false>(a, s);
        case 3: return launch_dual_mode<kLocal, true>(a, s);
        case 4: return launch_dual_mode<kSemi, false>(a, s);
        case 5: return launch_dual_mode<kSemi, true>(a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_flex(int mode, bool cigar, const FillArgs& a, hipStream_t s) {
    switch (mode * 2 + (cigar ? 1 : 0)) {
        case 0: return launch_flex_mode<kGlobal, false>(a, s);
        case 1: return launch_flex_mode<kGlobal, true>(a, s);
        case 2: return launch_flex_mode<kLocal, false>(a, s);
        case 3: return launch_flex_mode<kLocal, true>(a, s);
        case 4: return launch_flex_mode<kSemi, false>(a, s);
        case 5: return launch_flex_mode<kSemi, true>(a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_traceback(int mode, const TraceArgs& a, hipStream_t s, int group) {
    if (!a.count) return hipSuccess;
    const dim3 g = grid_for(a.count), b(kBlock);
    if (mode == kLocal && group == 32) {
        hipLaunchKernelGGL(traceback_group_kernel<32>, grid_for((a.count + 1) / 2), b, 0, s, a);
        return hipGetLastError();
    }
    if (group == 64 && a.blk == 2) {  // recomputing walks over checkpoints (ta_walk_ck.hip), any mode
        const hipError_t e = launch_walk_ck(mode, a, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(format_runs_kernel, g, b, 0, s, a);
        return hipGetLastError();
    }
    if (mode == kLocal && group == 64) {  // band walks (blocked layout), one lane per pair
        hipLaunchKernelGGL(traceback_band_kernel, dim3((a.count + kWave - 1) / kWave), dim3(kWave), 0, s, a);
        hipLaunchKernelGGL(format_runs_kernel, g, b, 0, s, a);
        return hipGetLastError();
    }
    if (mode == kLocal && group == 16) {  // lane walks (TA_LW_G lanes per pair)
        constexpr int W = 64 / TA_LW_G;
        hipLaunchKernelGGL(traceback_lane_kernel<TA_LW_G>, dim3((a.count + W - 1) / W), dim3(kWave), 0, s, a);
        return hipGetLastError();
    }
    switch (mode) {
        case kGlobal: hipLaunchKernelGGL(traceback_kernel<kGlobal>, g, b, 0, s, a); break;
        case kLocal: hipLaunchKernelGGL(traceback_kernel<kLocal>, g, b, 0, s, a); break;
        case kSemi: hipLaunchKernelGGL(traceback_kernel<kSemi>, g, b, 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

#ifdef TA_LW_PROF
extern "C" int ta_lw_prof(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lw_prof), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(lw_prof), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

#ifdef TA_BW_PROF
extern "C" int ta_bw_prof(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(bw_prof), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(bw_prof), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

hipError_t launch_serve(int mode, const ServeArgs& a, uint32_t slots, hipStream_t s) {
    switch (mode) {
        case kGlobal: return launch_serve_mode<kGlobal>(a, slots, s);
        case kLocal: return launch_serve_mode<kLocal>(a, slots, s);
        case kSemi: return launch_serve_mode<kSemi>(a, slots, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_compact(const CompactArgs& a, hipStream_t s) {
    if (!a.n_pairs) return hipSuccess;
    hipLaunchKernelGGL(compact_kernel, grid_for(a.n_pairs), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}
#endif

}  // namespace ta
