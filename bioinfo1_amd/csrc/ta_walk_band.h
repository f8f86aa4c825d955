// bioinfo1_amd/csrc/ta_walk_band.h -- the local-mode traceback of plans in the
// blocked code layout (ta_layout.h blk_index): ONE LANE PER PAIR, 64 walks per
// one-wave block, every operand of a walk step in the lane's own LDS region,
// then one wave per pair formats the runs into the CIGAR slot.
//
// Same walk as traceback_pair<kLocal> (ta_device.h) and the lane walk
// (ta_walk_lane.h): from the goal, while the current cell's cost is > 0
// (team_alignment.cpp:201-217), move to the parent its code names (D wins over
// I: the packed fill stores raw compares), the cost tracked exactly (a cell
// with cost > 0 is unclamped, so its parent's cost is its own minus the step's
// score, :20-28).  For gap <= 0 and sequences without '-' (the planner and the
// dual fill's per-pair flag route everything else to the fallback walk), a
// gap move never lowers the cost, so the walk can only end right after a
// diagonal move.
//
// A column resolves the D run above the current cell inside its stripe from
// ONE code dword (the D plane shifted so that the current row is bit 0:
// trailing ones), then the M or I move at the row the run stops on; an
// iteration reads kBwCols columns' operands in one batch of LDS reads and walks
// them while the moves stay in the stripe.  A walk follows its stripe (16 rows)
// along the steps, which in the blocked layout are contiguous: a stripe's
// 64-step window is 4 x 64 bytes.  Each walker stages the windows of the
// stripes ahead of it -- predicted along the diagonal from its current cell --
// into a ring of 4 slots (stripe & 3).  A slot is addressed by position alone
// (codes at step & 63, target bytes at their address & 127), and carries its
// stripe and window start in a header read beside the data, so a step needs no
// per-slot bookkeeping in registers.  Staging runs in rounds of kBwRound
// iterations: a round issues the next stripe's loads (codes into registers,
// query and target pieces by LDS-DMA), walks, and commits the stripe to its
// slot at its end, so no walker waits on memory unless its path left its
// predicted window (it then sits out until its stripe is restaged around its
// actual cell).  Every walked column leaves an event (D-run length, move) in an
// LDS list per walker that goes to HBM 32 at a time; format_runs_kernel merges
// the events into runs and writes the CIGAR text (the RunWriter layout,
// ta_device.h).
#pragma once

#include "ta_walk_lane.h"

namespace ta {
namespace {

#ifdef TA_BW_PROF
// experiment builds only: per-phase clock totals of the band walk
__device__ unsigned long long bw_prof[8];
#define BW_T(v) const uint64_t v = __builtin_readcyclecounter()
#define BW_ACC(k, d) bwp[k] += (d)
#else
#define BW_T(v)
#define BW_ACC(k, d)
#endif

constexpr int kBwSlots = 4;                       // stripe slots per walker (ring: stripe & 3)
#ifndef TA_BW_BLOCKS
#define TA_BW_BLOCKS 4
#endif
constexpr int kBwBlocks = TA_BW_BLOCKS;            // code window: 16-step blocks staged per stripe (3 or 4)
constexpr int kBwWin = 16 * kBwBlocks;             // ... its steps (the ring holds 64)
constexpr int kBwT = 64 * 4;                      // slot offset: target ring (128 bytes, by address & 127)
constexpr int kBwQ = kBwT + 128;                  // slot offset: the stripe's 16 query bytes
constexpr int kBwHdr = kBwQ + 16;                 // slot offset: header {stripe, window start step}
constexpr int kBwSlotB = 512;                     // bytes per slot
constexpr int kBwRunCap = 64;                     // event list: two halves of 32, leaving for HBM by halves
#ifndef TA_BW_COLS
#define TA_BW_COLS 2
#endif
constexpr int kBwCols = TA_BW_COLS;               // columns a walk iteration may move (1, 2 or 4)
#ifndef TA_BW_EVENTS
#define TA_BW_EVENTS 12
#endif
constexpr int kBwRound = TA_BW_EVENTS / kBwCols;  // walk iterations per staging round (<= 16 events)
#ifndef TA_BW_LOOK
#define TA_BW_LOOK 3
#endif
constexpr int kBwLook = TA_BW_LOOK;               // stripes staged ahead of the walk (<= kBwSlots - 1)
static_assert(kBwLook >= 1 && kBwLook < kBwSlots, "band walk lookahead");
constexpr int kBwRuns = kBwSlots * kBwSlotB;      // region offset of the run list
constexpr int kBwRegion = kBwRuns + kBwRunCap * 4 + 16;  // 2320 = 580 dwords (4 mod 32: spreads banks)
static_assert(kBwRegion % 16 == 0 && kBwHdr + 8 <= kBwSlotB, "band walk LDS layout");
// pending events (< 32 after a round's flush, + one round's, + one spare write) within the list
static_assert(31 + kBwRound * kBwCols + kBwCols - 1 < kBwRunCap, "band walk event list");

// Registers of one stripe staged in flight: 16 code pieces (4 blocks x 64
// bytes), 32 query bytes and 80 target bytes from 16-byte aligned addresses.
struct BwStage {
    uint4 c[4 * kBwBlocks];
};
// The query and target pieces go global -> LDS directly (LDS-DMA, lane-linear:
// piece k of lane l at stage + k * 1024 + 16 l), the codes through registers.
// (Register destinations for all 23 pieces left hipcc copying some of them at
// the branch merge, i.e. waiting for those loads in the middle of the issue.)
constexpr int kBwTPieces = kBwBlocks + 1;  // target pieces: the window's columns from an aligned start
constexpr int kBwStagePieces = 2 + kBwTPieces;  // + 2 query pieces
constexpr int kBwStageBytes = kBwStagePieces * kWave * 16;
typedef __attribute__((address_space(1))) const void* bw_gptr;
typedef __attribute__((address_space(3))) void* bw_lptr;
__device__ __forceinline__ void bw_dma16(const void* g, uint32_t lds) {
    __builtin_amdgcn_global_load_lds((bw_gptr)g, (bw_lptr)(uintptr_t)lds, 16, 0, 0);
}

typedef unsigned int bw_v4 __attribute__((ext_vector_type(4)));
typedef unsigned int bw_v2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) bw_v4 lds_u128;
typedef __attribute__((address_space(3))) bw_v2 lds_u64;
typedef __attribute__((address_space(3))) uint8_t lds_u8t;
__device__ __forceinline__ uint4 lds_ld128(uint32_t a) {
    const bw_v4 v = *(const lds_u128*)(uintptr_t)a;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void lds_st128(uint32_t a, uint4 v) {
    bw_v4 w;
    w.x = v.x, w.y = v.y, w.z = v.z, w.w = v.w;
    *(lds_u128*)(uintptr_t)a = w;
}
__device__ __forceinline__ bw_v2 lds_ld64(uint32_t a) { return *(const lds_u64*)(uintptr_t)a; }
__device__ __forceinline__ void lds_st64(uint32_t a, int x, int y) {
    bw_v2 w;
    w.x = (uint32_t)x, w.y = (uint32_t)y;
    *(lds_u64*)(uintptr_t)a = w;
}
__device__ __forceinline__ uint32_t lds_ld8(uint32_t a) { return *(const lds_u8t*)(uintptr_t)a; }

// Window of stripe h (global stripe index: pass * 64 + lane) centred on column
// ctr: 4 blocks from u0 = floor((ctr + ln - 24) / 16), clamped to the pass.
// Returns the window's first step; `ta16` the 16-byte aligned address of its
// target pieces.  The query and target pieces are 16-byte aligned and clamped
// to [first, last] piece that holds a valid byte (32-bit offsets from the
// pair's aligned base): a clamped piece is never read by the walk, and never
// a fault.
__device__ __forceinline__ int bw_issue(BwStage& st, uint32_t stage, const uint32_t* P, const uint8_t* Q,
                                        const uint8_t* T, uint32_t n, uint32_t m, uint32_t nb, int h, int ctr,
                                        uint32_t& qmis, uint32_t& ta16) {
    const uint32_t pass = (uint32_t)h >> 6, ln = (uint32_t)h & 63u;
    int u0 = (ctr + (int)ln - 24) >> 4;
    u0 = min(max(u0, 0), (int)nb - kBwBlocks);  // nb >= 4: pass_steps(m) >= 64
    const uint32_t* cp = P + blk_index(pass, 16u * (uint32_t)u0, ln, nb);
#pragma unroll
    for (int b = 0; b < kBwBlocks; ++b)
#pragma unroll
        for (int k = 0; k < 4; ++k)
            st.c[4 * b + k] = *reinterpret_cast<const uint4*>(cp + (uint64_t)b * (kWave * kBlkSteps) + 4 * k);
    // target: 80 bytes from the aligned piece holding the window's first column
    const int tm = (int)((uint32_t)(uintptr_t)T & 15u);
    const uint8_t* tb = T - tm;
    const int cw = 16 * u0 - (int)ln;  // the window's first column
    const int thi = (tm + (int)m - 1) & ~15;
    const int to = (tm + cw) & ~15;  // (floor; pieces outside the pair hold clamped copies, never read)
#pragma unroll
    for (int k = 0; k < kBwTPieces; ++k) bw_dma16(tb + min(max(to + 16 * k, 0), thi), stage + (2u + k) * (kWave * 16u));
    // ring positions follow the unclamped pieces' addresses
    ta16 = (uint32_t)(uintptr_t)tb + (uint32_t)to;
    // query: 32 bytes from the aligned piece holding row 16h
    // (pointer arithmetic from Q and T, not integer casts: keeps the loads global, not flat)
    const uint32_t qm = (uint32_t)(uintptr_t)Q & 15u;
    const uint8_t* qb = Q - qm;
    const uint32_t qo = (qm + 16u * (uint32_t)h) & ~15u, qhi = (qm + n - 1u) & ~15u;
    qmis = (qm + 16u * (uint32_t)h) & 15u;
    bw_dma16(qb + min(qo, qhi), stage);
    bw_dma16(qb + min(qo + 16u, qhi), stage + kWave * 16u);
    return 16 * u0;
}

// The staged stripe into its slot: codes at step & 63, target bytes at their
// address & 127, the 16 query bytes shifted to the slot's query field, and the
// header (stripe, first step) that tells a step whether its cell is inside.
__device__ __forceinline__ void bw_commit(const BwStage& st, uint32_t stl, uint32_t sb, uint32_t qmis, uint32_t ta16,
                                          int h, int w0) {
    // (stl: this lane's pieces in the LDS-DMA stage; every DMA of the round has landed)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    uint4 tq[kBwStagePieces];
#pragma unroll
    for (int k = 0; k < kBwStagePieces; ++k) tq[k] = lds_ld128(stl + (uint32_t)k * (kWave * 16u));
#pragma unroll
    for (int k = 0; k < 4 * kBwBlocks; ++k) lds_st128(sb + ((uint32_t)(w0 * 4 + 16 * k) & 255u), st.c[k]);
#pragma unroll
    for (int k = 0; k < kBwTPieces; ++k) lds_st128(sb + kBwT + ((ta16 + 16u * k) & 127u), tq[2 + k]);
    const uint32_t w[8] = {tq[0].x, tq[0].y, tq[0].z, tq[0].w, tq[1].x, tq[1].y, tq[1].z, tq[1].w};
    const uint32_t a = qmis >> 2, sh = qmis & 3u;
    uint32_t s[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint32_t v0 = w[i], v1 = w[i + 1], v2 = w[i + 2], v3 = i + 3 < 8 ? w[i + 3] : 0u;
        s[i] = a == 0 ? v0 : (a == 1 ? v1 : (a == 2 ? v2 : v3));
    }
    uint4 o;
    o.x = __builtin_amdgcn_alignbyte(s[1], s[0], sh);
    o.y = __builtin_amdgcn_alignbyte(s[2], s[1], sh);
    o.z = __builtin_amdgcn_alignbyte(s[3], s[2], sh);
    o.w = __builtin_amdgcn_alignbyte(s[4], s[3], sh);
    lds_st128(sb + kBwQ, o);
    lds_st64(sb + kBwHdr, h, w0);
}

// One half (32 events) of the walker's list to its event words in HBM.
__device__ __forceinline__ void bw_runs_out(uint32_t src, uint32_t* dst) {
#pragma unroll
    for (int k = 0; k < 8; ++k) *reinterpret_cast<uint4*>(dst + 4 * k) = lds_ld128(src + 16u * k);
}

// The local walks of pairs 64 * blockIdx.x + lane (one wave per block).  One
// event per walked column to a.runs: the D run's length above bit 16, the move
// after it in bits 1:0 (0 M, 1 I, 3 none: the run left the stripe) and its
// count (here 1; the recomputing walk's I runs, ta_walk_ck.hip) in bits 15:2;
// their number to cigar_len (format_runs_kernel merges them into runs and
// replaces it by the text length).
__device__ __forceinline__ void traceback_band_local(const TraceArgs& a, uint8_t* lds, int lane) {
    const uint32_t k = 64u * blockIdx.x + (uint32_t)lane;
    bool has = k < a.count;
    const uint32_t p = has ? (a.order ? a.order[a.begin + k] : a.begin + k) : 0u;
    if (has && a.pflag && a.pflag[p] == 1) has = false;  // '-' bytes: the fallback walk (traceback_kernel)
    uint32_t n = 0, m = 0, gi = 0, gj = 0;
    int H = 0;
    const uint32_t* P = a.ptrs;
    const uint8_t* Q = a.qbytes;
    const uint8_t* T = a.tbytes;
    uint32_t* rout = a.runs;
    if (has) {
        n = a.qlen[p];
        m = a.tlen[p];
        gi = a.goal_i[p];
        gj = a.goal_j[p];
        H = a.score[p];
        P += a.ptr_off[p];
        Q += a.qoff[p];
        T += a.toff[p];
        rout += band_runs_off(a.slot_off[p]);  // (16-byte aligned: bw_runs_out)
    }
    const uint32_t nb = blk_count(m);
    const int ma = a.match, mi = a.mismatch, gap = a.gap;
    const uint32_t reg = lds_addr(lds) + (uint32_t)lane * kBwRegion;
    const uint32_t rl = reg + kBwRuns;  // event list: 64 entries, two halves of 32
    const uint32_t stage = lds_addr(lds) + kWave * kBwRegion, stl = stage + 16u * (uint32_t)lane;
    const uint32_t tlow = (uint32_t)(uintptr_t)T;  // target byte c lives at ring (tlow + c) & 127
    bool live = has && H > 0;           // a positive score has its goal at i, j >= 1
    int g = live ? (int)((gi - 1u) >> 4) : 0, r = live ? (int)((gi - 1u) & 15u) : 0, c = live ? (int)gj - 1 : 0;
    // every slot's header invalid (stripe -1)
#pragma unroll
    for (int s = 0; s < kBwSlots; ++s) lds_st64(reg + s * kBwSlotB + kBwHdr, -1, 0);
    // the goal's stripe, staged at once
    if (live) {
        BwStage st;
        uint32_t qmis = 0, ta16 = 0;
        const int w0 = bw_issue(st, stage, P, Q, T, n, m, nb, g, c - r + 8, qmis, ta16);
        bw_commit(st, stl, reg + ((uint32_t)g & 3u) * kBwSlotB, qmis, ta16, g, w0);
    }
    int lo = g;                 // lowest stripe staged or in flight
    bool stalled = false;
    uint32_t nr = 0u, nout = 0u;  // events listed, events in HBM
#ifdef TA_BW_PROF
    uint64_t bwp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    // the scores in VGPRs (a select reads at most one SGPR besides its mask)
    int mav = ma, miv = mi, gapv = gap;
    asm volatile("" : "+v"(mav), "+v"(miv), "+v"(gapv));
    BW_T(t_begin);
    while (ballot(live)) {
        // ---- staging round: issue the next stripe's loads (they land while this
        // round's walk iterations run), commit them at the round's end
        BW_T(t1);
        int h = -1, ctr = 0;
        if (live) {
            if (stalled) {  // the walk left its window: restage its stripe around the current cell
                h = g;
                ctr = c - r + 8;
            } else if (lo > g - kBwLook && lo > 0) {  // the next stripe ahead, on the diagonal
                h = lo - 1;
                ctr = c - r + 8 - 16 * (g - h);
            }
        }
        BwStage st;
        uint32_t qmis = 0, ta16 = 0;
        int pend_w0 = 0;
        const bool pend = h >= 0;
        if (pend) {
            pend_w0 = bw_issue(st, stage, P, Q, T, n, m, nb, h, ctr, qmis, ta16);
            lo = min(lo, h);
        }
        // a full half of the event list to HBM (at most TA_BW_EVENTS events per round)
        if (nr - nout >= 32u) {
            bw_runs_out(rl + ((nout & 32u) << 2), rout + nout);
            nout += 32u;
        }
        BW_T(t2);
        BW_ACC(1, t2 - t1);
        BW_ACC(5, 1);
        // ---- walk iterations, branch-free: every lane computes all kBwCols
        // columns and writes all their events (an event past the count is
        // overwritten later; the list never holds more than 50 pending), and only
        // the lanes whose cell is inside their staged window keep the results.
        // The LDS reads of a step go out together: the codes and target bytes of
        // columns c .. c - kBwCols + 1; column k is walked when column k - 1's
        // move stayed in the stripe (an M or I move: the next cell is in column
        // c - k), the walk goes on and step t - k is inside the window.  A walk
        // that leaves its window stops there until its stripe is restaged.
#pragma unroll
        for (int it = 0; it < kBwRound; ++it) {
#ifdef TA_BW_PROF
            bwp[6] += (live && stalled) ? 1 : 0;
            bwp[7] += (live && !stalled) ? 1 : 0;
#endif
            const uint32_t ln = (uint32_t)g & 63u, t = (uint32_t)c + ln;
            const uint32_t sb = reg + (((uint32_t)g & 3u) << 9);
            const uint32_t tr = sb + kBwT, tc = tlow + (uint32_t)c;
            bw_v2 hd = lds_ld64(sb + kBwHdr);
            uint4 q4 = lds_ld128(sb + kBwQ);
            uint32_t xs[kBwCols], tbs[kBwCols];
#pragma unroll
            for (int k = 0; k < kBwCols; ++k) {
                xs[k] = lds_ld32(sb + (((t - (uint32_t)k) & 63u) << 2));
                tbs[k] = lds_ld8(tr + ((tc - (uint32_t)k) & 127u));
            }
            // (keeps the reads together ahead of their uses)
            asm volatile("" : "+v"(hd), "+v"(q4.x), "+v"(q4.y), "+v"(q4.z), "+v"(q4.w));
#pragma unroll
            for (int k = 0; k < kBwCols; ++k) asm volatile("" : "+v"(xs[k]), "+v"(tbs[k]));
            const bool inwin = (int)hd.x == g && t - hd.y < (uint32_t)kBwWin;
            const bool ok = live && !stalled && inwin;
            stalled = stalled || (live && !inwin);
            // one column: the D run from row rr up (bit planes, ta_internal.h Code:
            // row rr's D at 31 - rr), then the M or I move at the row it stops on
            // (none when the run leaves the stripe at its top); its event is the D
            // run's length above bit 16, the move in bits 1:0 (3: none), its count (1) between
            auto column = [&](uint32_t xc, uint32_t tbc, int rr, int& dH, uint32_t& ev, int& nrow, bool& top) {
                const uint32_t dp = xc >> (31 - rr);
                const int kd = (int)__builtin_ctz(~dp);  // <= rr + 1
                const int rp = rr - kd;
                top = rp < 0;
                const uint32_t ib = __builtin_amdgcn_ubfe(xc, (uint32_t)(15 - rp), 1u);  // (offset mod 32)
                const uint32_t sel = (uint32_t)rp & 7u;
                const uint32_t qlo = __builtin_amdgcn_perm(q4.y, q4.x, sel), qhi = __builtin_amdgcn_perm(q4.w, q4.z, sel);
                uint32_t qb = ((rp & 8) ? qhi : qlo) & 0xFFu;
                // (computed in every lane: hipcc would branch around the query
                // read for the lanes whose run left the stripe)
                asm volatile("" : "+v"(qb));
                const int sc = (qb == tbc) ? mav : miv;
                const int mv = top ? 0 : (ib ? gapv : sc);
                dH = __mul24(kd, gapv) + mv;
                ev = ((uint32_t)kd << 16) | 4u | (top ? 3u : ib);
                nrow = (top || ib) ? rp : rp - 1;
            };
            bool take = ok, prev_top = false;
            int rr = r, Hc = H, nrowf = r, dc = 0;  // (no column taken: the cell stays)
            uint32_t ne = 0u;
#pragma unroll
            for (int k = 0; k < kBwCols; ++k) {
                int dH, nrow;
                uint32_t ev;
                bool top;
                column(xs[k], tbs[k], rr & 15, dH, ev, nrow, top);
                lds_st32(rl + (((nr + (uint32_t)k) & 63u) << 2), ev);
                if (k > 0) take = take && !prev_top && rr >= 0 && Hc > 0 && t - (uint32_t)k - hd.y < (uint32_t)kBwWin;
                Hc = take ? Hc - dH : Hc;
                ne += take ? 1u : 0u;
                dc += (take && !top) ? 1 : 0;
                nrowf = take ? nrow : nrowf;
                prev_top = top;
                rr = nrow;
            }
            // the next cell: up the stripe (D run), left (I) or diagonal (M)
            c -= dc;
            H = Hc;
            nr += ne;
            g += nrowf >> 31;  // -1 when the row leaves the stripe's top
            r = nrowf & 15;    // (-1 -> 15)
            // (events of a walk <= its columns + stripe crossings <= m + n/16 + 1: the
            // cap never binds on a correct walk; it bounds the list and the loop)
            live = live && H > 0 && nr + kBwCols <= n + m + 1u;
        }
        BW_T(t3);
        BW_ACC(3, t3 - t2);
        // ---- the stripe loaded this round into its slot (the walk reads it from
        // the next round on); a stalled walk whose stripe this is goes on
        if (pend) {
            bw_commit(st, stl, reg + ((uint32_t)h & 3u) * kBwSlotB, qmis, ta16, h, pend_w0);
            if (h == g) stalled = false;
        }
        BW_T(t4);
        BW_ACC(0, t4 - t3);
    }
    BW_T(t_end);
    BW_ACC(4, t_end - t_begin);
#ifdef TA_BW_PROF
    // phases: per wave (lane 0); stall / walk iterations: summed over lanes
    if (lane == 0)
        for (int q = 0; q < 6; ++q) atomicAdd(&bw_prof[q], (unsigned long long)bwp[q]);
    atomicAdd(&bw_prof[6], (unsigned long long)bwp[6]);
    atomicAdd(&bw_prof[7], (unsigned long long)bwp[7]);
#endif
    // a walk stopped by the event cap with cost left would hand over a truncated
    // CIGAR: the plan's error word says so (never on a correct walk: the cap is
    // its columns plus stripe crossings)
    if (has && H > 0) atomicOr(a.err, kErrWalkCap);
    if (has) {
        // the rest of the list (fewer than 40 events, in list order)
        for (uint32_t j = nout; j < nr; ++j) rout[j] = lds_ld32(rl + ((j & 63u) << 2));
        a.cigar_len[p] = nr;  // the event count, for format_runs_kernel
    }
}

// Wave-wide inclusive scans in DPP (row_shr 1, 2, 4, 8 within each 16-lane row,
// then row_bcast 15 / 31 across rows): six VALU ops where __shfl_up steps are
// six ds_bpermute round trips.  Lanes without a source add 0 (max: INT_MIN).
__device__ __forceinline__ uint32_t bw_scan_add(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
}
__device__ __forceinline__ int bw_scan_max(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x111, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x112, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x114, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x118, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x142, 0xA, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x143, 0xC, 0xF, false));
    return v;
}
// lane l gets lane l + 1's v (lane 63: last63)
__device__ __forceinline__ int wave_shl1(int last63, int v) {
    return __builtin_amdgcn_update_dpp(last63, v, 0x130, 0xF, 0xF, false);
}

// Decimal digits of c (c < 2^32).
__device__ __forceinline__ uint32_t bw_digits(uint32_t c) {
    uint32_t d = 1u + (c >= 10u) + (c >= 100u) + (c >= 1000u) + (c >= 10000u);
    if (ballot(c >= 100000u))
        d += (c >= 100000u) + (c >= 1000000u) + (c >= 10000000u) + (c >= 100000000u) + (c >= 1000000000u);
    return d;
}

// "<count><op>" at q (digits first).
__device__ __forceinline__ void bw_put_run(char* q, uint32_t c, uint32_t op, uint32_t digits, bool act) {
    if (act) q[digits] = (char)((0x44494Du >> (8u * op)) & 0xFFu);  // 'M', 'I', 'D'
    for (uint32_t d = 0; ballot(act && d < digits); ++d) {
        if (act && d < digits) {
            const uint32_t qv = __umulhi(c, 0xCCCCCCCDu) >> 3;  // c / 10
            q[digits - 1u - d] = (char)('0' + (c - 10u * qv));
            c = qv;
        }
    }
}

// One wave per pair of a band-walked chunk: its events (walk order, i.e. the
// CIGAR's last run first) expanded into items -- the event's D run (when
// long 1+), then its move (when any, count times) -- and items of one op next to each other
// merged into runs, formatted right to left into the end of its slot, 64
// events per round (RunWriter's layout, ta_device.h; "1\0" for no move,
// :145-160).  A run still open at the end of a round is carried into the next.
__device__ __forceinline__ void format_runs(const TraceArgs& a, uint32_t p, int lane) {
    if (a.pflag && a.pflag[p] == 1) return;  // walked by the fallback walk (2: a flexible-fill pair, walked over checkpoints)
    const uint32_t n = a.qlen[p], m = a.tlen[p];
    const uint64_t cap = cigar_slot_bytes(n, m), soff = a.slot_off[p];
    const uint32_t* ev = a.runs + band_runs_off(soff);
    char* end = a.slots + soff + cap;
    const uint32_t E = a.cigar_len[p];
#ifdef TA_BW_DUMP
    // experiment builds only: the raw events, one byte each, as the "CIGAR"
    for (uint32_t k = (uint32_t)lane; k < E; k += 64u) a.slots[soff + k] = (char)ev[k];
    if (lane == 0) {
        a.cigar_start[p] = soff;
        a.cigar_len[p] = E;
    }
    return;
#endif
    uint32_t used = 0;
    if (E == 0) {
        if (lane == 0) {
            *(end - 2) = '1';
            *(end - 1) = '\0';
        }
        used = 2;
    }
    uint32_t cop = 3u, ccnt = 0u;  // the run carried from the previous round (op 3: none)
    // each round's events are loaded one round ahead: the text stores of a round
    // (char, which may alias anything) keep the compiler from hoisting the load
    uint32_t vnext = (uint32_t)lane < E ? ev[lane] : 0u;
    for (uint32_t base = 0; base < E; base += 64u) {
        const uint32_t k = base + (uint32_t)lane;
        const bool act = k < E;
        const uint32_t v = vnext;
        vnext = k + 64u < E ? ev[k + 64u] : 0u;
        const uint32_t kd = v >> 16, bc = (v >> 2) & 0x3FFFu, mop = act ? (v & 3u) : 3u;
        const bool va = kd > 0, vb = mop != 3u;      // item A: D x kd; item B: the move (M / I) x bc
        const uint32_t first = va ? 2u : mop;        // op of the event's first / last item (3: no item)
        const uint32_t last = vb ? mop : (va ? 2u : 3u);
        // the previous event's last op (lane 0: the carried run's), the next
        // event's first (lane 63: unused).  (Cross-lane moves stay out of any
        // select: inside `?:` one becomes a branch that masks lanes off, and a
        // masked-off source lane reads as 0.)
        const uint32_t plast = (uint32_t)wave_shr1((int)cop, (int)last);
        const uint32_t nfirst = (uint32_t)wave_shl1(3, (int)first);
        const bool ha = va && plast != 2u;                   // A starts a run
        const bool hb = vb && (va || plast != mop);          // B starts a run (always after an A)
        // item prefix sums: lane k's items end at pre_k; the carried count precedes lane 0
        const uint32_t tot = kd + (vb ? bc : 0u);
        const uint32_t pre = bw_scan_add(tot + (lane == 0 ? ccnt : 0u));
        const uint32_t preA = pre - (vb ? bc : 0u);  // through item A
        // the prefix just before the latest run head at or before each lane's end
        // (a max scan: prefixes grow); the carried run's head sits at prefix 0
        int hv = hb ? (int)(pre - bc) : (ha ? (int)(preA - kd) : -1);
        const int hmax = bw_scan_max(hv);
        const int hprev0 = wave_shr1(0, hmax);
        const int hprev = lane == 0 ? 0 : max(hprev0, 0);  // (lane 0 continues the carry: head at 0)
        const uint32_t sumA = preA - (uint32_t)(ha ? (int)(preA - kd) : hprev);
        const uint32_t sumB = pre - (uint32_t)(hb ? (int)(pre - bc) : hprev);
        // run ends: A before B, or before the next event's first item of another op;
        // lane 63's last item may continue into the next round
        const bool more = lane == 63 && base + 64u < E;  // (lane 63 of a non-final round)
        const bool nxt_diff = lane == 63 ? (base + 64u >= E) : nfirst != last;
        const bool ea = act && va && (vb || (!more && nxt_diff));
        const bool eb = act && vb && !more && nxt_diff;
        const uint32_t dA = bw_digits(sumA), dB = bw_digits(sumB);
        const uint32_t LA = ea ? dA + 1u : 0u, LB = eb ? dB + 1u : 0u;
        const uint32_t incl = bw_scan_add(LA + LB);
        // the carried run, when lane 0's first item does not continue it, ends first
        const uint32_t f0 = (uint32_t)__builtin_amdgcn_readlane((int)first, 0);
        if (cop != 3u && f0 != cop) {
            const uint32_t dg = bw_digits(ccnt);
            bw_put_run(end - used - (dg + 1u), ccnt, cop, dg, lane == 0);
            used += dg + 1u;
        }
        // lane k's texts: B (later in the walk) left of A
        char* q = end - used - incl;
        bw_put_run(q, sumB, mop, dB, eb);
        bw_put_run(q + LB, sumA, 2u, dA, ea);
        used += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        // carry lane 63's open run into the next round
        const bool cont = base + 64u < E;
        const uint32_t l63 = (uint32_t)__builtin_amdgcn_readlane((int)last, 63);
        const uint32_t s63 = (uint32_t)__builtin_amdgcn_readlane((int)(vb ? sumB : sumA), 63);
        cop = cont ? l63 : 3u;
        ccnt = cont ? s63 : 0u;
    }
    if (lane == 0) {
        a.cigar_start[p] = soff + cap - used;
        a.cigar_len[p] = used;
    }
}

}  // namespace
}  // namespace ta
