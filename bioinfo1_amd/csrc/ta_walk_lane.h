// bioinfo1_amd/csrc/ta_walk_lane.h -- the local-mode traceback as a serial
// walk: one lane per pair steps cell by cell through a tile of the code
// matrix staged in LDS, G lanes per pair (64 / G pairs per wave) load the
// tiles and format the CIGAR.
//
// Same walk as traceback_pair<kLocal> (ta_device.h) and walk_group_local
// (ta_walk2.h): from the goal, while the current cell's cost is > 0
// (team_alignment.cpp:201-217), move to the parent its code names (D wins
// over I, the raw compares of the packed fills), the cost tracked exactly
// (a cell with cost > 0 is unclamped, so its parent's cost is its own minus
// the step's score, :20-28).  The run walks resolve one run of one op per
// iteration for ~130 VALU instructions (config 2: ~440 runs of ~3 cells per
// pair); this walk costs ~35 per CELL but serves 64 / G pairs per
// instruction, and every per-cell operand is in LDS: the tile (8 stripes x 64
// steps of one pass, [step][stripe] dwords = the workspace's own 32-byte
// runs), the query bytes of its 128 rows and the target bytes of its 71
// columns with their indel costs (int8 beside each byte).  Runs go to an LDS
// list; the group formats 64 at a time, right to left into the slot
// (RunWriter's layout, ta_device.h).
//
// The walkers of a wave step together and leave the cell loop as soon as one
// of them needs the group: a tile reload (the walk left the tile at the top
// or the left), a full run list, or the end of its walk.
#pragma once

#include "ta_walk2.h"

namespace ta {
namespace {

#ifdef TA_LW_PROF
// experiment builds only: per-phase clock totals of the lane walk
__device__ unsigned long long lw_prof[8];
#define LW_T(v) const uint64_t v = __builtin_readcyclecounter()
#define LW_ACC(k, d) lwp[k] += (d)
#else
#define LW_T(v)
#define LW_ACC(k, d)
#endif

// 32-bit LDS byte addresses (the group's arrays are LDS; keeps the cell
// loop's address math in 32 bits)
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
template <typename T>
__device__ __forceinline__ uint32_t lds_addr(const T* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ uint32_t lds_ld32(uint32_t a) { return *(const lds_u32*)(uintptr_t)a; }
__device__ __forceinline__ uint32_t lds_ld16(uint32_t a) { return *(const lds_u16*)(uintptr_t)a; }
__device__ __forceinline__ void lds_st32(uint32_t a, uint32_t v) { *(lds_u32*)(uintptr_t)a = v; }

constexpr int kLwStripes = 8;                          // tile rows: 8 stripes = 128 query rows
#ifndef TA_LW_STEPS
#define TA_LW_STEPS 64
#endif
constexpr int kLwSteps = TA_LW_STEPS;                  // tile columns: 64 steps of the pass
#ifndef TA_LW_RUNS
#define TA_LW_RUNS 64
#endif
constexpr int kLwRunCap = TA_LW_RUNS;                  // runs listed before a flush
constexpr int kLwTileDw = kLwStripes * kLwSteps;       // 512 dwords
constexpr int kLwQEnt = kLwStripes * kRows;            // 128 query rows (u16: byte | indel cost << 8)
constexpr int kLwTEnt = kLwSteps + kLwStripes;         // 72 target columns (u16 likewise)
constexpr int kLwGroupDw = kLwTileDw + kLwQEnt / 2 + kLwTEnt / 2 + 1 + kLwRunCap + 7;  // +7: group bases on different banks

// Staging registers of one tile (per lane: its share of the loads).
template <int G>
struct LwStage {
    static constexpr int NL = 2 * kLwSteps / G;       // 16-byte pieces of codes
    static constexpr int NQ = kLwQEnt / G;            // query bytes
    static constexpr int NT = (kLwTEnt + G - 1) / G;  // target bytes
    uint4 v[NL];
    uint32_t q[NQ], t[NT];
};

// Issue the loads of the tile around the cell (row, col) = (i - 1, j - 1):
// stripes [L0, L0 + 8) of its pass (the cell's stripe 4..7 of them, L0 a
// multiple of 4 for 16-byte loads), steps [T0, T0 + 64) with the cell's step
// the last one (the walk only moves up and left), and set the tile
// coordinates of the cell: lr = row - rowbase in [0, 128), lc = col - cb in
// [0, 71], its step lc + (lr >> 4) - 7.  Every load comes from a clamped
// (valid) address, so a stage costs one memory latency.  All G lanes of the
// group.
template <int G>
__device__ __forceinline__ void lw_issue(int row, int col, int& rowbase, int& cb, int& lr, int& lc, uint32_t& T0,
                                         LwStage<G>& st, const uint32_t* P, const uint8_t* Q, const uint8_t* T,
                                         uint32_t n, uint32_t m, uint32_t li) {
    const uint32_t ln = ((uint32_t)row >> 4) & 63u, tP = (uint32_t)row >> 10;
    const uint32_t t = (uint32_t)col + ln;
    const uint32_t L0 = (max(ln, 4u) - 4u) & ~3u;
    const uint32_t Tmax = pass_steps(m);
    T0 = max(t, (uint32_t)kLwSteps - 1u) - (uint32_t)(kLwSteps - 1);
    rowbase = (int)(tP * (uint32_t)kPassRows + L0 * (uint32_t)kRows);
    cb = (int)T0 - (int)L0 - (kLwStripes - 1);
    lr = row - rowbase;
    lc = col - cb;
    // one 64-bit base per stage, 32-bit dword offsets per load (full-rate math)
    const uint32_t* Pp = P + ((uint64_t)tP * Tmax * kWave + L0);
#pragma unroll
    for (int k = 0; k < LwStage<G>::NL; ++k) {
        const uint32_t x = li + (uint32_t)G * k, ts = min(T0 + (x >> 1), Tmax - 1u);
        st.v[k] = *(const uint4*)(Pp + (ts * (uint32_t)kWave + 4u * (x & 1u)));
    }
#pragma unroll
    for (int k = 0; k < LwStage<G>::NQ; ++k) st.q[k] = Q[min((uint32_t)rowbase + li + (uint32_t)G * k, n - 1u)];
#pragma unroll
    for (int k = 0; k < LwStage<G>::NT; ++k)
        st.t[k] = T[(uint32_t)min(max(cb + (int)(li + (uint32_t)G * k), 0), (int)m - 1)];
}

// Write a staged tile into the group's LDS: codes ([step][stripe] dwords),
// query rows and target columns as u16 (byte | indel cost << 8).  Entries
// outside the pass or the sequences hold copies of clamped in-range loads: the
// walk reads only the cells of its path, which lie inside both.
template <int G>
__device__ __forceinline__ void lw_commit(const LwStage<G>& st, uint32_t* tile, uint16_t* qw, uint16_t* tw, int gap,
                                          uint32_t li) {
    const uint32_t gq = (uint32_t)gap & 0xFFu;
#pragma unroll
    for (int k = 0; k < LwStage<G>::NL; ++k) *(uint4*)(tile + 4u * (li + (uint32_t)G * k)) = st.v[k];
#pragma unroll
    for (int k = 0; k < LwStage<G>::NQ; ++k) {
        const uint32_t c = st.q[k];
        qw[li + (uint32_t)G * k] = (uint16_t)(c | ((c == '-' ? 0u : gq) << 8));
    }
#pragma unroll
    for (int k = 0; k < LwStage<G>::NT; ++k) {
        const uint32_t e = li + (uint32_t)G * k, c = st.t[k];
        if (e < (uint32_t)kLwTEnt) tw[e] = (uint16_t)(c | ((c == '-' ? 0u : gq) << 8));
    }
}

// Inclusive prefix sum over the G lanes of the group; G = 16 is one DPP row
// (row_shr 1, 2, 4, 8: four VALU ops instead of four ds_bpermute round trips).
template <int G>
__device__ __forceinline__ int lw_prefix(int v, uint32_t li) {
    if constexpr (G == 16) {
        v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
        v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
        v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
        v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
        return v;
    } else {
        return group_prefix<G>(v, li);
    }
}

// Format runs[0 .. nflush) (op 0/1/2 = M/I/D in bits 1:0, count above) right to
// left in front of the `used` bytes already written at the slot's end.
template <int G>
__device__ __forceinline__ void lw_flush(const uint32_t* runs, int nflush, char* end, uint32_t& used, uint32_t h,
                                         uint32_t li) {
    for (int base = 0; base < nflush; base += G) {
        const int e = base + (int)li;
        const bool act = e < nflush;
        const uint32_t v = act ? runs[e] : 0u;
        uint32_t c = v >> 2;
        // counts below 65,536 (every run of pairs shorter than that): five digit
        // tests and exact 24-bit reciprocal divisions, (c * 52429) >> 19 = c / 10
        const bool big = ballot(c >= 65536u) != 0;
        uint32_t digits = 1u + (c >= 10u) + (c >= 100u) + (c >= 1000u) + (c >= 10000u);
        if (big)
            digits += (c >= 100000u) + (c >= 1000000u) + (c >= 10000000u) + (c >= 100000000u) + (c >= 1000000000u);
        const uint32_t L = act ? digits + 1u : 0u;
        const uint32_t incl = (uint32_t)lw_prefix<G>((int)L, li);
        char* p = end - used - (incl - L) - 1;
        if (act) *p = (char)((0x44494Du >> (8u * (v & 3u))) & 0xFFu);  // 'M', 'I', 'D'
        for (uint32_t d = 0; ballot(act && d < digits); ++d) {
            const uint32_t q = big ? c / 10u : (__umul24(c, 52429u) >> 19);
            if (act && d < digits) p[-1 - (int)d] = (char)('0' + (c - q * 10u));
            c = q;
        }
        used += gread<G>(incl, h, G - 1);
    }
}

// The local walks of pairs W * blockIdx.x + h (W = 64 / G walkers, one wave
// per block), h = lane / G.  Every lane of a group holds its walker's state.
template <int G>
__device__ __forceinline__ void traceback_lane_local(const TraceArgs& a, uint32_t* lds, int lane) {
    constexpr int W = 64 / G;
    const uint32_t h = (uint32_t)lane / G, li = (uint32_t)lane % G;
    const uint32_t k = (uint32_t)W * blockIdx.x + h;
    const bool has = k < a.count;
    uint32_t* tile = lds + h * kLwGroupDw;
    uint16_t* qw = (uint16_t*)(tile + kLwTileDw);
    uint16_t* tw = qw + kLwQEnt;
    uint32_t* runs = (uint32_t*)(tw + kLwTEnt) + 1;  // runs[-1]: the first cell's deferred write
    const uint32_t p = has ? (a.order ? a.order[a.begin + k] : a.begin + k) : 0u;
    uint32_t n = 0, m = 0, gi = 0, gj = 0;
    int H = 0;
    uint64_t cap = 0, soff = 0;
    const uint32_t* P = a.ptrs;
    const uint8_t* Q = a.qbytes;
    const uint8_t* T = a.tbytes;
    if (has) {
        n = a.qlen[p];
        m = a.tlen[p];
        gi = a.goal_i[p];
        gj = a.goal_j[p];
        H = a.score[p];
        P += a.ptr_off[p];
        Q += a.qoff[p];
        T += a.toff[p];
        cap = cigar_slot_bytes(n, m);
        soff = a.slot_off[p];
    }
    char* end = a.slots + soff + cap;
    const int ma = a.match, mi = a.mismatch, gap = a.gap;
    const int posM = max(max(0, gap), max(ma, mi));  // no step lowers the cost by more
    int lr = 0, lc = 0, rowbase = 0, cb = 0;
    uint32_t T0 = 0;
    uint32_t op = 3u, cnt = 0u, used = 0u;
    int nr = -1;                        // runs[0 .. nr]: closed runs, then the open one
    bool live = has && H > 0;           // a positive score has its goal at i, j >= 1
    bool stage = live;                  // needs a tile around (row, col)
    int row = (int)gi - 1, col = (int)gj - 1;
    LwStage<G> st;
#ifdef TA_LW_PROF
    uint64_t lwp[5] = {0, 0, 0, 0, 0};
#endif
    LW_T(t_begin);
    while (ballot(live)) {
        LW_T(t0);
        if (ballot(stage)) {
            if (stage) {
                if (row < 0 || col < 0) {
                    live = false;  // (cannot happen: the cost of row / column 0 is 0)
                } else {
                    lw_issue<G>(row, col, rowbase, cb, lr, lc, T0, st, P, Q, T, n, m, li);
                    lw_commit<G>(st, tile, qw, tw, gap, li);
                }
                stage = false;
            }
        }
        LW_T(t1);
        LW_ACC(0, t1 - t0);
        const bool walk = live;
        if (walk) {
            // The cell loop: (lr, lc) is a tile cell with cost H > 0.  Its three
            // LDS reads are the only round trip per cell: the run entry of the
            // previous cell is written just before them (LDS completes in order),
            // and a cell whose successor provably stays inside the tile with a
            // positive cost and room in the run list (`safe`, from the state
            // before the reads) skips the exact exit test.  32-bit LDS byte
            // addresses (no 64-bit pointer math; full-rate 24-bit multiplies).
            const uint32_t tb = lds_addr(tile), qb = lds_addr(qw), tcb = lds_addr(tw), rb = lds_addr(runs);
            int mav = ma, miv = mi;  // held in VGPRs (a select reads at most one SGPR besides vcc)
            asm volatile("" : "+v"(mav), "+v"(miv));
            while (true) {
                lds_st32(rb + 4u * (uint32_t)nr, op | (cnt << 2));  // (every lane of the group: same value)
                const int s = lr >> 4;
                const uint32_t code = lds_ld32(tb + ((uint32_t)lc << 5) + __umul24((uint32_t)s, 36u) -
                                               4u * kLwStripes * (kLwStripes - 1));
                const uint32_t qv = lds_ld16(qb + ((uint32_t)lr << 1)), tv = lds_ld16(tcb + ((uint32_t)lc << 1));
                const bool safe = H > posM && lr >= 1 && lc + s - (kLwStripes - 1) >= 2 && nr < kLwRunCap - 2;
                // bit planes (ta_internal.h Code): row r's D bit at 31 - r, I bit at 15 - r
                const uint32_t x = (code >> ((uint32_t)~lr & 15u)) & 0x10001u;
                const uint32_t o = min(x, 2u);  // 0 M, 1 I, 2 D (D wins)
                lr -= (o != 1u) ? 1 : 0;
                lc -= (o != 2u) ? 1 : 0;
                const int sm = (((qv ^ tv) & 0xFFu) == 0u) ? mav : miv;
                const int sg = __builtin_amdgcn_sbfe((int)((o == 2u) ? qv : tv), 8, 8);
                H -= (o == 0u) ? sm : sg;
                const bool same = o == op;
                cnt = same ? cnt + 1u : 1u;
                nr += same ? 0 : 1;
                op = o;
                if (ballot(!safe)) {
                    const bool ok = H > 0 && lr >= 0 && lc + (lr >> 4) - (kLwStripes - 1) >= 0 && nr < kLwRunCap - 1;
                    if (ballot(!ok)) break;
                }
            }
            runs[nr] = op | (cnt << 2);
        }
        LW_T(t2);
        LW_ACC(1, t2 - t1);
        LW_ACC(4, 1);
        const bool fin = walk && H <= 0;
        const bool full = walk && !fin && nr >= kLwRunCap - 1;
        if (ballot(fin || full)) {
            if (fin || full) {
                lw_flush<G>(runs, fin ? nr + 1 : nr, end, used, h, li);
                if (full) {
                    if (li == 0) runs[0] = op | (cnt << 2);  // the open run moves to the front
                    nr = 0;
                }
            }
        }
        if (walk && !fin && (lr < 0 || lc + (lr >> 4) - (kLwStripes - 1) < 0)) {
            stage = true;  // left the tile at the top or the left
            row = rowbase + lr;
            col = cb + lc;
        }
        if (fin) live = false;
        LW_T(t3);
        LW_ACC(2, t3 - t2);
    }
    LW_T(t_end);
    LW_ACC(3, t_end - t_begin);
#ifdef TA_LW_PROF
    if (lane == 0)
        for (int q = 0; q < 5; ++q) atomicAdd(&lw_prof[q], (unsigned long long)lwp[q]);
#endif
    if (has) {
        if (used == 0u) {  // no move: RLE of an empty op string, "1" + '\0' (:145-160)
            if (li == 0) {
                *(end - 2) = '1';
                *(end - 1) = '\0';
            }
            used = 2u;
        }
        if (li == 0) {
            a.cigar_start[p] = soff + cap - used;
            a.cigar_len[p] = used;
        }
    }
}

}  // namespace
}  // namespace ta
