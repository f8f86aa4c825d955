// bioinfo1_amd/csrc/ta_walk_ck.hip -- the local walks of checkpoint plans
// (Plan::ck).  Their dual fill stored no codes, only each
// stripe's bottom row at every column and its 16 rows every 16 columns
// (ta_layout.h ck_row_index / ck_col_index); the walk recomputes the codes of
// the cells around its path.
//
// The walk is the band walk's (ta_walk_band.h) and traceback_pair<kLocal>'s:
// from the goal, while the cell's cost is > 0 (team_alignment.cpp:201-217),
// move to the parent the cell's raw compares name -- up when H(i-1, j) + gap
// beats max(diagonal, left), else left when H(i, j-1) + gap beats the
// diagonal, else the diagonal (the fill's compares, :102-116 / :171-194) --
// the cost tracked exactly (:20-28); with gap <= 0 and no '-' (the planner and
// the fill's hand-back flag route everything else elsewhere) it can only end
// right after a diagonal move.
//
// 8 lanes per pair (two rows of the stripe each), 8 pairs per wave.  A window
// is the 16 rows of the walk's stripe g over the columns c0 + 1 .. j, j the
// walk's column and c0 the stripe's nearest checkpoint at least kCkLead columns
// to its left (or column 0).  The lanes sweep the window's anti-diagonals in
// int32 from the checkpoint (left) and stripe g-1's stored bottom row (top),
// the up value from the lane above by DPP, and shift their rows' D, I and H = 0
// bits into registers; the rows go to LDS and the walk crosses the window one
// row per step: stop on a cell with H = 0, else the run of cells whose move is
// I (I set, D clear) as trailing ones, then the D or M move out of the row.
// It leaves through the window's top (stripe g - 1, same column) or its left
// edge (stripe g from the next checkpoint left).  Events as the band walk's,
// for format_runs_kernel: D run above bit 16, count of the move in bits 15:2,
// move in bits 1:0.  (16 lanes of one row each: 0.85 ms on config 2 against
// ... for 8 x 2, scripts/exp/gpu_ck.sh.)
#include "ta_device.h"
#include "ta_packed.h"

namespace ta {
namespace {

constexpr int kCkLead = 17;            // columns a window reaches left of the walk's column, at least
constexpr int kCkMaxW = kCkLead + 15;  // the widest window (checkpoints 16 columns apart)
// lanes per pair: 16 (a row of the stripe each) or 8 (two rows each)
#ifndef TA_CK_LANES
#define TA_CK_LANES 16
#endif
constexpr int kCkLanes = TA_CK_LANES;
constexpr int kCkRows = 16 / kCkLanes;      // rows per lane
constexpr int kCkPairs = kWave / kCkLanes;  // pairs per wave
static_assert(kCkLanes == 8 || kCkLanes == 16, "lanes per pair");
// sweep steps: W + lanes - 1, run in blocks of 8; two 32-bit words per row keep them all
constexpr int kCkMaxSteps = (kCkMaxW + kCkLanes - 1 + 7) / 8 * 8;
static_assert(kCkMaxSteps <= 64, "a window's steps fit a 64-bit row word");

struct CkGroup {
    // per row of the window, window column x at bit W - x: cells whose move is
    // I (I and not D), D bits, cells with H = 0 (the walk's end)
    uint4 row[16];
    int top[kCkMaxSteps + 8];        // H(16g, c0 + x) + gap, x = 0 .. W (the sweep reads up to x = K)
    uint8_t tb[16 + kCkMaxSteps + 8];  // target byte of window column x at [16 + x]
    uint8_t q[16];                   // query bytes of the stripe's rows
    uint32_t rec[16];                // the window's row steps: I run (bits 5:0), D move (8), run to the edge (9)
};

__device__ __forceinline__ void ck_wave_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

#ifdef TA_CK_PROF
// experiment builds only: per-phase clock totals (per wave) and counts
__device__ unsigned long long ck_prof[8];
#define CK_T(v) const uint64_t v = __builtin_readcyclecounter()
#define CK_ACC(k, d) ckp[k] += (d)
#else
#define CK_T(v)
#define CK_ACC(k, d)
#endif

// The pairs the dual fill handed back ('-' bytes; usually none), one wave per
// pair in the one-pair walk over their blocked codes -- here rather than in a
// launch of its own, whose count only the device knows.
__device__ __forceinline__ void ck_fallback_walks(const TraceArgs& a, int lane) {
    if (!a.fb_count) return;
    const uint32_t nfb = *a.fb_count;
    for (uint32_t w = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); w < nfb; w += gridDim.x * kWavesPerBlock) {
        const uint32_t q = a.fb_order[w];
        const uint32_t qn = a.qlen[q], qm = a.tlen[q];
        uint64_t st;
        uint32_t len;
        const WalkSeq seq{a.qbytes + a.qoff[q], a.tbytes + a.toff[q], a.score[q], a.match, a.mismatch, a.gap};
        traceback_pair<kLocal>(a.ptrs + a.ptr_off[q], qn, qm, a.goal_i[q], a.goal_j[q], a.slots + a.slot_off[q],
                               cigar_slot_bytes(qn, qm), lane, &st, &len, seq, true);
        if (lane == 0) {
            a.cigar_start[q] = a.slot_off[q] + st;
            a.cigar_len[q] = len;
        }
    }
}

__global__ __launch_bounds__(kBlock) void traceback_ck_kernel(TraceArgs a) {
    __shared__ CkGroup groups[kWavesPerBlock * kCkPairs];
    const int lane = (int)threadIdx.x & 63, lg = lane & (kCkLanes - 1), ra = kCkRows * lg;  // rows ra (, ra + 1)
    CkGroup& G = groups[threadIdx.x / kCkLanes];
    const uint32_t slot = (blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * kCkPairs + (uint32_t)(lane / kCkLanes);
    bool has = slot < a.count;
    const uint32_t p = has ? (a.order ? a.order[a.begin + slot] : a.begin + slot) : 0u;
    if (has && a.pflag && a.pflag[p]) has = false;  // '-' bytes: the fallback walk below
    uint32_t n = 0, m = 0;
    int i = 0, j = 0, H = 0;
    const uint16_t* P = nullptr;
    const uint8_t* Q = a.qbytes;
    const uint8_t* T = a.tbytes;
    uint32_t* rout = a.runs;
    if (has) {
        n = a.qlen[p];
        m = a.tlen[p];
        i = (int)a.goal_i[p];
        j = (int)a.goal_j[p];
        H = a.score[p];
        P = reinterpret_cast<const uint16_t*>(a.ptrs + a.ptr_off[p]);
        Q += a.qoff[p];
        T += a.toff[p];
        rout += band_runs_off(a.slot_off[p]);
    }
    const int ma = a.match, mi = a.mismatch, gap = a.gap;
    const int zstep = 1 - 16 * ma;
    const int off3 = has ? local_max3_offset(n, m, ma, mi, gap) : -1;  // the fill's frame (ck_decode)
    const int off = off3 >= 0 ? off3 : 0, dl = off3 >= 0 ? zstep + 16 : 0;
    const uint32_t nb = blk_count(m);
    const int sA = ma - gap, sB = mi - gap;  // diagonal gains net of the gap the values carry
    bool live = has && H > 0;                // a positive score has its goal at i, j >= 1
    // events listed; the pending I run (an I run continues across windows)
    uint32_t nev = 0, kI = 0;
    const uint32_t cap = 2 * (n + m) - 1;  // the walk's room (ta_internal.h band_runs_off)
    uint32_t windows = 0;
#ifdef TA_CK_PROF
    uint64_t ckp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    CK_T(t_begin);
    while (ballot(live)) {
        CK_T(t0);
        // ---- the window: stripe g, columns c0 + 1 .. j
        const int g = live ? (i - 1) >> 4 : 0, r = live ? (i - 1) & 15 : 0;
        const int l = g & 63, pass = g >> 6;
        const int e = j - kCkLead + l;
        // block (e >> 4) - 1's checkpoint column, or column 0 when that block ended
        // before the stripe's first column (16 (b + 1) - l <= 0: j <= 32 then)
        const int c0 = e >= 16 ? max((e >> 4) * 16 - l, 0) : 0;
        const int W = live ? j - c0 : 0;
        const int ir = 16 * g + ra + 1;  // this lane's first row
        const int lu = (g - 1) & 63, pu = (g - 1) >> 6;  // the stripe above (g >= 1)
        // every load of the window first (one wait for all), then the decodes
        constexpr int kTopQ = (kCkMaxW + kCkLanes) / kCkLanes, kTbQ = kCkMaxW / kCkLanes;
        const bool hl_ok = live && c0 > 0 && ir <= (int)n;
        // (two rows: two adjacent int16 of the checkpoint, one aligned dword)
        const uint32_t ck_at = hl_ok ? (uint32_t)ck_col_index(pass, (uint32_t)(e >> 4) - 1u, l, nb, ra) : 0u;
        const uint32_t v2 = !hl_ok ? 0u : (kCkRows == 2 ? *reinterpret_cast<const uint32_t*>(P + ck_at) : (uint32_t)P[ck_at]);
        int tr[kTopQ];
        uint32_t tbv[kTbQ];
#pragma unroll
        for (int q = 0; q < kTopQ; ++q) {
            const int x = lg + kCkLanes * q, col = c0 + x;
            tr[q] = (live && x <= W && g > 0 && col > 0) ? (int)(int16_t)P[ck_row_index(pu, (uint32_t)(col + lu - 1), lu, nb)] : 0;
        }
#pragma unroll
        for (int q = 0; q < kTbQ; ++q) {
            const int x = 1 + lg + kCkLanes * q;
            tbv[q] = (live && x <= W) ? T[c0 + x - 1] : 0u;
        }
        uint32_t qv[kCkRows];
        int gl[kCkRows];  // own H + gap: the next column's left candidates (H(row, c0) first)
#pragma unroll
        for (int h = 0; h < kCkRows; ++h) {
            qv[h] = (live && ir + h <= (int)n) ? Q[ir - 1 + h] : 0u;
            gl[h] = (hl_ok ? ck_decode((int)(int16_t)(v2 >> (16 * h)), off, zstep, dl, ir + h, c0, l) : 0) + gap;
        }
#pragma unroll
        for (int q = 0; q < kTopQ; ++q) {
            const int x = lg + kCkLanes * q, col = c0 + x;
            if (live && x <= W) G.top[x] = (g > 0 && col > 0 ? ck_decode(tr[q], off, zstep, dl, 16 * g, col, lu) : 0) + gap;
        }
#pragma unroll
        for (int q = 0; q < kTbQ; ++q) {
            const int x = 1 + lg + kCkLanes * q;
            if (live && x <= W) G.tb[16 + x] = (uint8_t)tbv[q];
        }
#pragma unroll
        for (int h = 0; h < kCkRows; ++h) G.q[ra + h] = (uint8_t)qv[h];
        ck_wave_sync();

        // ---- the sweep: step k, lane lg computes column x = k - lg + 1 of its rows
        const int K = ((wave_max(W > 0 ? W + r / kCkRows : 0) + 7) >> 3) << 3;
        CK_T(t1);
        CK_ACC(0, t1 - t0);
        CK_ACC(4, 1);
        CK_ACC(6, K);
        int upp = G.top[0];  // the previous step's up candidate of row ra (lane 0: H(16g, c0) + gap)
        uint32_t db[kCkRows][2], ib[kCkRows][2], zb[kCkRows][2];
#pragma unroll
        for (int h = 0; h < kCkRows; ++h)
            for (int w = 0; w < 2; ++w) db[h][w] = ib[h][w] = zb[h][w] = 0u;
        const uint8_t* tbl = &G.tb[17 - lg];
        const bool first = lg == 0;
        auto block = [&](int kb, auto ramp_tag, auto hi_tag) {
            constexpr bool RAMP = decltype(ramp_tag)::value;
            constexpr int HW = decltype(hi_tag)::value ? 1 : 0;
            int tv[8], bv[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                tv[s] = G.top[kb + s + 1];
                bv[s] = tbl[kb + s];
            }
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                // the first row: up from the lane above's last row (row_shr:1; a
                // group's first lane: the top row), diagonal = the previous step's up
                const int dpp = __builtin_amdgcn_update_dpp(tv[s], gl[kCkRows - 1], 0x111, 0xF, 0xF, false);
                int up = (kCkLanes == 16 || !first) ? dpp : tv[s];
                int dg = upp + ((uint32_t)bv[s] == qv[0] ? sA : sB);
                upp = up;
                int gn[kCkRows];
#pragma unroll
                for (int h = 0; h < kCkRows; ++h) {
                    if (h) {  // the next row: up = the row above's new value, diagonal = its previous one
                        dg = gl[h - 1] + ((uint32_t)bv[s] == qv[h] ? sA : sB);
                        up = gn[h - 1];
                    }
                    const int m1 = max(dg, gl[h]);
                    const int hn = max(max(m1, up), 0);
                    gn[h] = hn + gap;
                    // signs: D, I, H = 0
                    db[h][HW] = __builtin_amdgcn_alignbit(db[h][HW], (uint32_t)(m1 - up), 31);
                    ib[h][HW] = __builtin_amdgcn_alignbit(ib[h][HW], (uint32_t)(dg - gl[h]), 31);
                    zb[h][HW] = __builtin_amdgcn_alignbit(zb[h][HW], (uint32_t)(hn - 1), 31);
                }
                if (!RAMP || kb + s >= lg) {
#pragma unroll
                    for (int h = 0; h < kCkRows; ++h) gl[h] = gn[h];
                }
            }
        };
        for (int kb = 0; kb < K; kb += 8) {
            if (kb < kCkLanes) block(kb, std::true_type{}, std::false_type{});
            else if (kb < 32) block(kb, std::false_type{}, std::false_type{});
            else block(kb, std::false_type{}, std::true_type{});
        }
        // step k at bit K - 1 - k of the 64-bit row; column x = k - lg + 1 at bit W - x of
        // its window word (column 0, bit W, cleared: an I run stops at the window's edge)
        const uint32_t sh = (uint32_t)max(K - lg - W, 0), wmask = W >= 32 ? 0xFFFFFFFFu : (1u << W) - 1u;
        auto word = [&](const uint32_t (&v)[2]) -> uint32_t {
            const uint64_t u = K > 32 ? ((uint64_t)v[0] << (K - 32)) | v[1] : (uint64_t)v[0];
            return (uint32_t)(u >> sh) & wmask;
        };
#pragma unroll
        for (int h = 0; h < kCkRows; ++h) {
            const uint32_t wd = word(db[h]);
            G.row[ra + h] = make_uint4(word(ib[h]) & ~wd, wd, word(zb[h]), 0u);
        }
        ck_wave_sync();

        // ---- the walk across the window, one row per step: stop on a cell with
        // H = 0 (its cost, :20-28); else the I run from the current column (the
        // trailing ones of the I-only row word), then the D or M move out of the
        // row -- or, when the run reaches column c0, on in the next window.  The
        // loop keeps only what the next step depends on and lists each step's
        // record; the events are made from the records afterwards, in parallel.
        // (flags as 0 / 1 integers: compares into lane masks and back cost the
        // loop more than the arithmetic)
        int rr = r, x = W;
        uint32_t nrec = 0;
        const bool room = nev + 2u * (uint32_t)(r + 1) <= cap;  // (<= 2 events per row step)
        uint32_t wl = (live && room) ? 1u : 0u, zdone = 0;
        CK_T(t2);
        CK_ACC(1, t2 - t1);
        // Two steps per loop iteration with the row words read one step ahead
        // into alternating registers (a single one became a copy at the loop's
        // end, which waited for the read).
        auto row_step = [&](const uint4& w4) {
            const uint32_t pos = (uint32_t)(W - x);
            const uint32_t zero = (w4.z >> pos) & 1u;
            const uint32_t run = min((uint32_t)__builtin_ctzll((uint64_t)~(w4.x >> pos) | (1ull << 32)), (uint32_t)x);
            const uint32_t x1 = (uint32_t)x - run;
            const uint32_t edge = (x1 - 1u) >> 31, dmove = (w4.y >> ((pos + run) & 31u)) & 1u;  // (x1 >= 0)
            const uint32_t go = wl & (zero ^ 1u), mv = go & (edge ^ 1u);
            G.rec[nrec & 15] = run | (dmove << 8) | (edge << 9);
            nrec += go;
            x -= (int)(go * run + (mv & (dmove ^ 1u)));
            rr -= (int)mv;
            zdone |= wl & zero;
            wl = mv & ((uint32_t)~rr >> 31) & ((uint32_t)(x - 1) >> 31 ^ 1u);  // rr >= 0, x >= 1
        };
        uint4 wa = G.row[rr & 15], wb;
        while (ballot(wl != 0u)) {
            CK_ACC(5, 1);
            wb = G.row[(rr - 1) & 15];  // (the row a move up reaches)
            __builtin_amdgcn_sched_barrier(0);  // (issued here, not sunk to its use)
            row_step(wa);
            if (!ballot(wl != 0u)) break;
            wa = G.row[(rr - 1) & 15];
            __builtin_amdgcn_sched_barrier(0);
            row_step(wb);
        }
        ck_wave_sync();
        // events of the records, two per lane: an I run (with the run carried from
        // the previous window on the first record) and the D or M move; a record
        // that ran to the window's edge carries its run to the next window
        {
            uint32_t ev[4], ne = 0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t k = 2u * (uint32_t)lg + (uint32_t)h;
                const uint32_t rc = k < nrec ? G.rec[k] : 0x200u;  // (past the list: no event)
                const uint32_t runI = (rc & 63u) + (k == 0 ? kI : 0u);
                const bool ed = rc & 0x200u, iev = !ed && runI > 0;
                ev[2 * h] = (runI << 2) | 1u;
                ev[2 * h + 1] = (rc & 0x100u) ? ((1u << 16) | 3u) : 4u;  // D: a D run of 1, no move; M
                ne |= (iev ? 1u : 0u) << (2 * h);
                ne |= (ed ? 0u : 1u) << (2 * h + 1);
            }
            // exclusive prefix of the lane's event counts over the group's 8 lanes
            const uint32_t cnt = (uint32_t)__builtin_popcount(ne);
            uint32_t inc = cnt;
#pragma unroll
            for (int d = 1; d < kCkLanes; d <<= 1) {
                const uint32_t o = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (lane - d), (int)inc);
                inc += lg >= d ? o : 0u;
            }
            uint32_t at = nev + inc - cnt;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if ((ne >> e) & 1u) rout[at] = ev[e];
                at += (ne >> e) & 1u;
            }
            const uint32_t tot = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * ((lane & ~(kCkLanes - 1)) + kCkLanes - 1), (int)inc);
            // the carried I run: the last record's when it ran to the edge
            const uint32_t last = nrec ? G.rec[nrec - 1] : 0u;
            if (live) {
                kI = nrec ? ((last & 0x200u) ? (last & 63u) + (nrec == 1 ? kI : 0u) : 0u) : kI;
                nev += tot;
            }
        }
        CK_T(t3);
        CK_ACC(2, t3 - t2);
        if (live) {
            i = 16 * g + rr + 1;
            j = c0 + x;
            if (kI >= 8192u) {  // (an I run's count field is 14 bits; runs of one op merge in the text)
                if (lg == 0) rout[nev] = (kI << 2) | 1u;
                ++nev;
                kI = 0;
            }
            ++windows;
            const bool done = zdone || i < 1 || j < 1;  // row 0 / column 0: H = 0
            live = !done && room && windows <= n + m + 16u;
            H = done ? 0 : H;
        }
        ck_wave_sync();
    }
    CK_T(t_end);
    CK_ACC(3, t_end - t_begin);
#ifdef TA_CK_PROF
    if (lane == 0)
        for (int k = 0; k < 8; ++k) atomicAdd(&ck_prof[k], (unsigned long long)ckp[k]);
#endif
    if (has) {
        // (H: the goal's score until the walk reached a cell with H = 0; a walk
        // stopped by the event cap first -- never a correct one, its events <= n + m --
        // would hand over a truncated CIGAR: the plan's error word says so)
        if (H > 0) atomicOr(a.err, kErrWalkCap);
        if (lg == 0) a.cigar_len[p] = nev;  // the event count, for format_runs_kernel
    }
    ck_fallback_walks(a, lane);
}

// ---- Two pairs per lane (TA_CK_PACKED): the sweep in packed int16, 16 lanes
// (the 16 rows) per two pairs, 8 pairs per wave.  Each value is H + gap + B
// with B = mag + 1, so every value and candidate is a non-negative int16 below
// 0x7BFF (H <= 2047 in a dual plan, ta_planner.cpp fits_int16): the clamp and
// both maxima are one v_pk_maximum3_f16 (ta_packed.h pk_max3_pos).  (The gains
// stay v_pk_add_u16: a half past its window or of a finished pair holds
// anything, and a 32-bit add could carry it into the other.)  Each step's D, I and H = 0 signs of both pairs
// go into bit 7 - s of byte accumulators (sign_bytes + one bit insert, as the
// dual fill's codes); the sweep always runs 48 steps (W + r <= 47).  Then the
// lanes 0-7 of a group walk its first pair, 8-15 its second, as above.
constexpr int kCk2Steps = 48;
static_assert(kCkMaxW + 15 <= kCk2Steps, "packed sweep length");
struct Ck2Group {
    uint4 row[2][16];              // per pair and row: I-only, D, H = 0 window words
    uint32_t top[kCk2Steps + 8];   // per x: the two pairs' H(16g, c0 + x) + gap + B (int16 halves)
    uint32_t tb[16 + kCk2Steps + 8];  // per x (at 16 + x): the two pairs' target bytes (bytes 0 and 2)
    uint32_t rec[2][16];           // per pair: the window's row steps (as CkGroup.rec)
};

// Per-pair walk state, held by every lane of the pair's 16-lane group.
struct Ck2Pair {
    uint32_t p, n, m, nb;
    int i, j, H, off, dl;
    const uint16_t* P;
    const uint8_t* Q;
    const uint8_t* T;
    uint32_t* rout;
    uint32_t nev, kI, windows;
    bool has, live;
};

__global__ __launch_bounds__(kBlock) void traceback_ck2_kernel(TraceArgs a) {
    __shared__ Ck2Group groups[kWavesPerBlock * 4];
    // a latency-bound chain: beside the next batch's fill (align.DevicePipeline)
    // its instructions go first at the SIMD's issue arbiter
#ifndef TA_WALK_PRIO
#define TA_WALK_PRIO 3
#endif
    __builtin_amdgcn_s_setprio(TA_WALK_PRIO);
    const int lane = (int)threadIdx.x & 63, rw = lane & 15, hh = rw >> 3, lw = rw & 7;
    Ck2Group& G = groups[threadIdx.x >> 4];
    const int ma = a.match, mi = a.mismatch, gap = a.gap;
    const int zstep = 1 - 16 * ma;
    const int mag = max(max(max(ma, -ma), max(mi, -mi)), max(max(gap, -gap), 1));
    const int B = mag + 1;  // bias: values H + gap + B >= 1
    Ck2Pair S[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        Ck2Pair& c = S[h];
        const uint32_t slot = ((blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * 4 + (uint32_t)(lane >> 4)) * 2 + h;
        c.has = slot < a.count;
        c.p = c.has ? (a.order ? a.order[a.begin + slot] : a.begin + slot) : 0u;
        if (c.has && a.pflag && a.pflag[c.p]) c.has = false;  // '-' bytes: the fallback walk
        c.n = c.m = 0;
        c.i = c.j = c.H = 0;
        c.P = nullptr;
        c.Q = a.qbytes;
        c.T = a.tbytes;
        c.rout = a.runs;
        if (c.has) {
            c.n = a.qlen[c.p];
            c.m = a.tlen[c.p];
            c.i = (int)a.goal_i[c.p];
            c.j = (int)a.goal_j[c.p];
            c.H = a.score[c.p];
            c.P = reinterpret_cast<const uint16_t*>(a.ptrs + a.ptr_off[c.p]);
            c.Q += a.qoff[c.p];
            c.T += a.toff[c.p];
            c.rout += band_runs_off(a.slot_off[c.p]);
        }
        const int off3 = c.has ? local_max3_offset(c.n, c.m, ma, mi, gap) : -1;  // the fill's frame
        c.off = off3 >= 0 ? off3 : 0;
        c.dl = off3 >= 0 ? zstep + 16 : 0;
        c.nb = blk_count(c.m);
        c.live = c.has && c.H > 0;
        c.nev = c.kI = c.windows = 0;
    }
    // target bytes of both pairs share a dword per column: bytes 1 and 3 stay 0
    for (int k = rw; k < 16 + kCk2Steps + 8; k += 16) G.tb[k] = 0u;
    const uint32_t SA2 = rep16(ma - gap), GAP2 = rep16(gap), KD2 = rep16(mi - ma), B2 = rep16(B), Z2 = rep16(B + 1);
    uint32_t ONE = 0x00010001u;
    asm volatile("" : "+s"(ONE));  // (see ta_packed.h pk_min_u16)
    while (ballot(S[0].live || S[1].live)) {
        // ---- both pairs' windows: stripe g, columns c0 + 1 .. j (as traceback_ck_kernel)
        int g[2], r[2], c0[2], W[2], e[2], l[2];
        uint32_t gl2 = 0, q2 = 0;
        {
            int tr[2][3], hl[2];
            uint32_t tbv[2][2], qv[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const Ck2Pair& c = S[h];
                g[h] = c.live ? (c.i - 1) >> 4 : 0;
                r[h] = c.live ? (c.i - 1) & 15 : 0;
                l[h] = g[h] & 63;
                e[h] = c.j - kCkLead + l[h];
                c0[h] = e[h] >= 16 ? max((e[h] >> 4) * 16 - l[h], 0) : 0;
                W[h] = c.live ? c.j - c0[h] : 0;
                const int ir = 16 * g[h] + rw + 1, lu = (g[h] - 1) & 63, pu = (g[h] - 1) >> 6;
                const bool hl_ok = c.live && c0[h] > 0 && ir <= (int)c.n;
                hl[h] = hl_ok ? (int)(int16_t)c.P[ck_col_index(g[h] >> 6, (uint32_t)(e[h] >> 4) - 1u, l[h], c.nb, rw)] : 0;
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const int x = rw + 16 * q, col = c0[h] + x;
                    tr[h][q] = (c.live && x <= W[h] && g[h] > 0 && col > 0)
                                   ? (int)(int16_t)c.P[ck_row_index(pu, (uint32_t)(col + lu - 1), lu, c.nb)] : 0;
                }
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int x = 1 + rw + 16 * q;
                    tbv[h][q] = (c.live && x <= W[h]) ? c.T[c0[h] + x - 1] : 0u;
                }
                qv[h] = (c.live && ir <= (int)c.n) ? c.Q[ir - 1] : 0u;
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const Ck2Pair& c = S[h];
                const int ir = 16 * g[h] + rw + 1, lu = (g[h] - 1) & 63;
                const bool hl_ok = c.live && c0[h] > 0 && ir <= (int)c.n;
                const int lv = (hl_ok ? ck_decode(hl[h], c.off, zstep, c.dl, ir, c0[h], l[h]) : 0) + gap + B;
                gl2 |= ((uint32_t)lv & 0xFFFFu) << (16 * h);
                q2 |= qv[h] << (16 * h);
                uint16_t* tp = reinterpret_cast<uint16_t*>(G.top) + h;
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const int x = rw + 16 * q, col = c0[h] + x;
                    if (c.live && x <= W[h])
                        tp[2 * x] = (uint16_t)((g[h] > 0 && col > 0 ? ck_decode(tr[h][q], c.off, zstep, c.dl, 16 * g[h], col, lu) : 0) + gap + B);
                }
                uint8_t* tb8 = reinterpret_cast<uint8_t*>(G.tb) + 2 * h;
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int x = 1 + rw + 16 * q;
                    if (c.live && x <= W[h]) tb8[4 * (16 + x)] = (uint8_t)tbv[h][q];
                }
            }
        }
        ck_wave_sync();

        // ---- the sweep: 48 steps, lane rw computes column x = k - rw + 1 of its row of both pairs
        uint32_t upp = G.top[0];
        uint32_t adi[6], az[6];
        const uint32_t* tbl = &G.tb[17 - rw];
        auto block = [&](auto kb_tag) {
            constexpr int kb = decltype(kb_tag)::value;
            uint32_t tv[8], bv[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                tv[s] = G.top[kb + s + 1];
                bv[s] = tbl[kb + s];
            }
            uint32_t di = 0, zz = 0;
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp((int)tv[s], (int)gl2, 0x111, 0xF, 0xF, false);
                const uint32_t ef = pk_min_u16(q2 ^ bv[s], ONE);              // 0 match, 1 mismatch
                const uint32_t dg = pk_mad_i16(ef, KD2, pk_add(upp, SA2));  // H(r-1, x-1) + s + B
                const uint32_t m1 = pk_max(dg, gl2);
                const uint32_t hn = pk_max3_pos(m1, up, B2);                  // H + B (clamp at H = 0)
                const uint32_t gn = pk_add(hn, GAP2);
                // signs: D (up beats both), I (left beats the diagonal), H = 0
                const uint32_t mk = 0x01010101u << (7 - s);
                di = bfi(mk, sign_bytes(pk_sub(m1, up), pk_sub(dg, gl2)), di);
                const uint32_t zs = pk_sub(hn, Z2);
                zz = bfi(mk, sign_bytes(zs, zs), zz);
                if (kb >= 16 || kb + s >= rw) gl2 = gn;
                upp = up;
            }
            adi[kb / 8] = di;
            az[kb / 8] = zz;
        };
        block(std::integral_constant<int, 0>{});
        block(std::integral_constant<int, 8>{});
        block(std::integral_constant<int, 16>{});
        block(std::integral_constant<int, 24>{});
        block(std::integral_constant<int, 32>{});
        block(std::integral_constant<int, 40>{});
        // per pair: step k at bit 47 - k of a 48-bit row (block b's byte at bits
        // 8 (5 - b)), column x = k - rw + 1 at bit W - x of the window word
        auto word = [&](const uint32_t (&acc)[6], uint32_t bi, int h) -> uint32_t {
            const uint32_t sel = bi | ((4u + bi) << 8) | 0x0C0C0000u;  // [src1 byte, src0 byte, 0, 0]
            const uint32_t lo = (__builtin_amdgcn_perm(acc[2], acc[3], sel) << 16) | __builtin_amdgcn_perm(acc[4], acc[5], sel);
            const uint64_t u = ((uint64_t)__builtin_amdgcn_perm(acc[0], acc[1], sel) << 32) | lo;
            const uint32_t sh = (uint32_t)(kCk2Steps - rw - W[h]);
            return (uint32_t)(u >> sh) & (W[h] >= 32 ? 0xFFFFFFFFu : (1u << W[h]) - 1u);
        };
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t wd = word(adi, 2u + h, h);
            G.row[h][rw] = make_uint4(word(adi, (uint32_t)h, h) & ~wd, wd, word(az, (uint32_t)h, h), 0u);
        }
        ck_wave_sync();

        // ---- the walks: lanes 0-7 the group's first pair, 8-15 its second (as traceback_ck_kernel)
        Ck2Pair& c = S[0];  // (selected below: hh ? S[1] : S[0], field by field)
        const bool mlive = hh ? S[1].live : S[0].live;
        const int mr = hh ? r[1] : r[0], mW = hh ? W[1] : W[0], mg = hh ? g[1] : g[0], mc0 = hh ? c0[1] : c0[0];
        uint32_t mnev = hh ? S[1].nev : S[0].nev, mkI = hh ? S[1].kI : S[0].kI;
        const uint32_t mcap = 2 * ((hh ? S[1].n + S[1].m : S[0].n + S[0].m)) - 1;
        uint32_t* mrout = hh ? S[1].rout : S[0].rout;
        (void)c;
        int rr = mr, x = mW;
        uint32_t nrec = 0;
        const bool room = mnev + 2u * (uint32_t)(mr + 1) <= mcap;
        uint32_t wl = (mlive && room) ? 1u : 0u, zdone = 0;
        const uint4* rows = G.row[hh];
        uint32_t* recs = G.rec[hh];
        auto row_step = [&](const uint4& w4) {
            const uint32_t pos = (uint32_t)(mW - x);
            const uint32_t zero = (w4.z >> pos) & 1u;
            const uint32_t run = min((uint32_t)__builtin_ctzll((uint64_t)~(w4.x >> pos) | (1ull << 32)), (uint32_t)x);
            const uint32_t x1 = (uint32_t)x - run;
            const uint32_t edge = (x1 - 1u) >> 31, dmove = (w4.y >> ((pos + run) & 31u)) & 1u;
            const uint32_t go = wl & (zero ^ 1u), mv = go & (edge ^ 1u);
            recs[nrec & 15] = run | (dmove << 8) | (edge << 9);
            nrec += go;
            x -= (int)(go * run + (mv & (dmove ^ 1u)));
            rr -= (int)mv;
            zdone |= wl & zero;
            wl = mv & ((uint32_t)~rr >> 31) & ((uint32_t)(x - 1) >> 31 ^ 1u);
        };
        uint4 wa = rows[rr & 15], wb;
        while (ballot(wl != 0u)) {
            wb = rows[(rr - 1) & 15];
            __builtin_amdgcn_sched_barrier(0);
            row_step(wa);
            if (!ballot(wl != 0u)) break;
            wa = rows[(rr - 1) & 15];
            __builtin_amdgcn_sched_barrier(0);
            row_step(wb);
        }
        ck_wave_sync();
        {
            uint32_t ev[4], ne = 0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t k = 2u * (uint32_t)lw + (uint32_t)h;
                const uint32_t rc = k < nrec ? recs[k] : 0x200u;
                const uint32_t runI = (rc & 63u) + (k == 0 ? mkI : 0u);
                const bool ed = rc & 0x200u, iev = !ed && runI > 0;
                ev[2 * h] = (runI << 2) | 1u;
                ev[2 * h + 1] = (rc & 0x100u) ? ((1u << 16) | 3u) : 4u;
                ne |= (iev ? 1u : 0u) << (2 * h);
                ne |= (ed ? 0u : 1u) << (2 * h + 1);
            }
            const uint32_t cnt = (uint32_t)__builtin_popcount(ne);
            uint32_t inc = cnt;
#pragma unroll
            for (int d = 1; d < 8; d <<= 1) {
                const uint32_t o = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (lane - d), (int)inc);
                inc += lw >= d ? o : 0u;
            }
            uint32_t at = mnev + inc - cnt;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if ((ne >> q) & 1u) mrout[at] = ev[q];
                at += (ne >> q) & 1u;
            }
            const uint32_t tot = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * ((lane & ~7) + 7), (int)inc);
            const uint32_t last = nrec ? recs[nrec - 1] : 0u;
            if (mlive) {
                mkI = nrec ? ((last & 0x200u) ? (last & 63u) + (nrec == 1 ? mkI : 0u) : 0u) : mkI;
                mnev += tot;
            }
        }
        // the window's end: this half's pair, then both pairs' state in every lane
        int mi_ = hh ? S[1].i : S[0].i, mj = hh ? S[1].j : S[0].j, mH = hh ? S[1].H : S[0].H;
        uint32_t mwin = hh ? S[1].windows : S[0].windows;
        bool ml = mlive;
        if (mlive) {
            mi_ = 16 * mg + rr + 1;
            mj = mc0 + x;
            if (mkI >= 8192u) {
                if (lw == 0) mrout[mnev] = (mkI << 2) | 1u;
                ++mnev;
                mkI = 0;
            }
            ++mwin;
            const uint32_t mn = hh ? S[1].n : S[0].n, mm = hh ? S[1].m : S[0].m;
            const bool done = zdone || mi_ < 1 || mj < 1;
            ml = !done && room && mwin <= mn + mm + 16u;
            mH = done ? 0 : mH;
        }
        // (row_ror:8 within each 16-lane row: the other half's values)
        auto other = [](int v) { return __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false); };
        const int oi = other(mi_), oj = other(mj), oH = other(mH), onev = other((int)mnev), okI = other((int)mkI),
                  owin = other((int)mwin), ol = other(ml ? 1 : 0);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const bool mine = h == hh;
            S[h].i = mine ? mi_ : oi;
            S[h].j = mine ? mj : oj;
            S[h].H = mine ? mH : oH;
            S[h].nev = mine ? mnev : (uint32_t)onev;
            S[h].kI = mine ? mkI : (uint32_t)okI;
            S[h].windows = mine ? mwin : (uint32_t)owin;
            S[h].live = mine ? ml : (ol != 0);
        }
        ck_wave_sync();
    }
    {
        const Ck2Pair& c = hh ? S[1] : S[0];
        if (c.has) {
            if (c.H > 0) atomicOr(a.err, kErrWalkCap);
            if (lw == 0) a.cigar_len[c.p] = c.nev;
        }
    }
    ck_fallback_walks(a, lane);
}

}  // namespace

#ifdef TA_CK_PROF
extern "C" int ta_ck_prof(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ck_prof), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
    if (reset) {
        const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(ck_prof), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

#ifndef TA_CK_PACKED
#define TA_CK_PACKED 1
#endif
hipError_t launch_walk_ck(const TraceArgs& a, hipStream_t s) {
#if TA_CK_PACKED
    const uint32_t per_block = kWavesPerBlock * 8;
    hipLaunchKernelGGL(traceback_ck2_kernel, dim3((a.count + per_block - 1) / per_block), dim3(kBlock), 0, s, a);
#else
    const uint32_t per_block = kWavesPerBlock * kCkPairs;
    hipLaunchKernelGGL(traceback_ck_kernel, dim3((a.count + per_block - 1) / per_block), dim3(kBlock), 0, s, a);
#endif
    return hipGetLastError();
}

}  // namespace ta
