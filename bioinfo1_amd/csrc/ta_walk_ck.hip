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

namespace ta {
namespace {

constexpr int kCkLead = 17;            // columns a window reaches left of the walk's column, at least
constexpr int kCkMaxW = kCkLead + 15;  // the widest window (checkpoints 16 columns apart)
constexpr int kCkLanes = 8;            // lanes per pair, two rows of the stripe each
constexpr int kCkPairs = kWave / kCkLanes;  // pairs per wave
// sweep steps: W + 7 <= kCkMaxW + 7, run in blocks of 8; two 32-bit words per row keep them all
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

__global__ __launch_bounds__(kBlock) void traceback_ck_kernel(TraceArgs a) {
    __shared__ CkGroup groups[kWavesPerBlock * kCkPairs];
    const int lane = (int)threadIdx.x & 63, lg = lane & (kCkLanes - 1), ra = 2 * lg;  // rows ra, ra + 1
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
        // (rows ra, ra + 1: two adjacent int16 of the checkpoint, one aligned dword)
        const uint32_t v2 = hl_ok ? *reinterpret_cast<const uint32_t*>(P + ck_col_index(pass, (uint32_t)(e >> 4) - 1u, l, nb, ra)) : 0u;
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
        const uint32_t qa = (live && ir <= (int)n) ? Q[ir - 1] : 0u, qb = (live && ir < (int)n) ? Q[ir] : 0u;
        const int hla = hl_ok ? ck_decode((int)(int16_t)(v2 & 0xFFFFu), off, zstep, dl, ir, c0, l) : 0;  // H(ir, c0)
        const int hlb = hl_ok ? ck_decode((int)(int16_t)(v2 >> 16), off, zstep, dl, ir + 1, c0, l) : 0;
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
        G.q[ra] = (uint8_t)qa;
        G.q[ra + 1] = (uint8_t)qb;
        ck_wave_sync();

        // ---- the sweep: step k, lane lg computes column x = k - lg + 1 of rows ra, ra + 1
        const int K = ((wave_max(W > 0 ? W + (r >> 1) : 0) + 7) >> 3) << 3;
        CK_T(t1);
        CK_ACC(0, t1 - t0);
        CK_ACC(4, 1);
        CK_ACC(6, K);
        int ga = hla + gap, gb = hlb + gap;  // own H + gap: the next column's left candidates
        int upp = G.top[0];  // the previous step's up candidate of row ra (lane 0: H(16g, c0) + gap)
        uint32_t da0 = 0, da1 = 0, ia0 = 0, ia1 = 0, za0 = 0, za1 = 0;
        uint32_t db0 = 0, db1 = 0, ib0 = 0, ib1 = 0, zb0 = 0, zb1 = 0;
        const uint8_t* tbl = &G.tb[17 - lg];
        const bool first = lg == 0;
        auto block = [&](int kb, auto ramp_tag, auto hi_tag) {
            constexpr bool RAMP = decltype(ramp_tag)::value, HI = decltype(hi_tag)::value;
            int tv[8], bv[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                tv[s] = G.top[kb + s + 1];
                bv[s] = tbl[kb + s];
            }
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                // row ra: up from the lane above's row ra - 1 (row_shr:1; a group's first lane: the top row)
                const int dpp = __builtin_amdgcn_update_dpp(tv[s], gb, 0x111, 0xF, 0xF, false);
                const int upc = first ? tv[s] : dpp;
                const int dga = upp + ((uint32_t)bv[s] == qa ? sA : sB);
                const int m1a = max(dga, ga);
                const int hna = max(max(m1a, upc), 0);
                const int gan = hna + gap;
                // row ra + 1: up = row ra's new value, diagonal = row ra's previous one
                const int dgb = ga + ((uint32_t)bv[s] == qb ? sA : sB);
                const int m1b = max(dgb, gb);
                const int hnb = max(max(m1b, gan), 0);
                // signs: D, I, H = 0
                const uint32_t dsa = (uint32_t)(m1a - upc), isa = (uint32_t)(dga - ga), zsa = (uint32_t)(hna - 1);
                const uint32_t dsb = (uint32_t)(m1b - gan), isb = (uint32_t)(dgb - gb), zsb = (uint32_t)(hnb - 1);
                if constexpr (HI) {
                    da1 = __builtin_amdgcn_alignbit(da1, dsa, 31);
                    ia1 = __builtin_amdgcn_alignbit(ia1, isa, 31);
                    za1 = __builtin_amdgcn_alignbit(za1, zsa, 31);
                    db1 = __builtin_amdgcn_alignbit(db1, dsb, 31);
                    ib1 = __builtin_amdgcn_alignbit(ib1, isb, 31);
                    zb1 = __builtin_amdgcn_alignbit(zb1, zsb, 31);
                } else {
                    da0 = __builtin_amdgcn_alignbit(da0, dsa, 31);
                    ia0 = __builtin_amdgcn_alignbit(ia0, isa, 31);
                    za0 = __builtin_amdgcn_alignbit(za0, zsa, 31);
                    db0 = __builtin_amdgcn_alignbit(db0, dsb, 31);
                    ib0 = __builtin_amdgcn_alignbit(ib0, isb, 31);
                    zb0 = __builtin_amdgcn_alignbit(zb0, zsb, 31);
                }
                if (!RAMP || kb + s >= lg) {
                    ga = gan;
                    gb = hnb + gap;
                }
                upp = upc;
            }
        };
        for (int kb = 0; kb < K; kb += 8) {
            if (kb < 8) block(kb, std::true_type{}, std::false_type{});
            else if (kb < 32) block(kb, std::false_type{}, std::false_type{});
            else block(kb, std::false_type{}, std::true_type{});
        }
        // step k at bit K - 1 - k of the 64-bit row; column x = k - lg + 1 at bit W - x of
        // its window word (column 0, bit W, cleared: an I run stops at the window's edge)
        const uint32_t sh = (uint32_t)max(K - lg - W, 0), wmask = W >= 32 ? 0xFFFFFFFFu : (1u << W) - 1u;
        auto word = [&](uint32_t lo, uint32_t hi) -> uint32_t {
            const uint64_t u = K > 32 ? ((uint64_t)lo << (K - 32)) | hi : (uint64_t)lo;
            return (uint32_t)(u >> sh) & wmask;
        };
        const uint32_t wda = word(da0, da1), wdb = word(db0, db1);
        G.row[ra] = make_uint4(word(ia0, ia1) & ~wda, wda, word(za0, za1), 0u);
        G.row[ra + 1] = make_uint4(word(ib0, ib1) & ~wdb, wdb, word(zb0, zb1), 0u);
        ck_wave_sync();

        // ---- the walk across the window, one row per step: stop on a cell with
        // H = 0 (its cost, :20-28); else the I run from the current column (the
        // trailing ones of the I-only row word), then the D or M move out of the
        // row -- or, when the run reaches column c0, on in the next window.  The
        // loop keeps only what the next step depends on and lists each step's
        // record; the events are made from the records afterwards, in parallel.
        int rr = r, x = W;
        uint32_t nrec = 0;
        const bool room = nev + 2u * (uint32_t)(r + 1) <= cap;  // (<= 2 events per row step)
        bool wl = live && room, done = false;
        CK_T(t2);
        CK_ACC(1, t2 - t1);
        uint4 wnext = G.row[rr & 15];
        while (ballot(wl)) {
            CK_ACC(5, 1);
            const uint4 w4 = wnext;
            wnext = G.row[(rr - 1) & 15];  // (the row a move up reaches: read one step ahead)
            const uint32_t pos = (uint32_t)(W - x);
            const bool zero = (w4.z >> pos) & 1u;
            const uint32_t run = min((uint32_t)__builtin_ctzll((uint64_t)~(w4.x >> pos) | (1ull << 32)), (uint32_t)x);
            const int x1 = x - (int)run;
            const bool edge = x1 == 0, dmove = (w4.y >> ((pos + run) & 31u)) & 1u;
            const bool go = wl && !zero, mv = go && !edge;
            G.rec[nrec & 15] = run | (dmove ? 0x100u : 0u) | (edge ? 0x200u : 0u);
            nrec += go ? 1u : 0u;
            x = go ? (edge ? 0 : x1 - (dmove ? 0 : 1)) : x;
            rr = mv ? rr - 1 : rr;
            done = done || (wl && zero);
            wl = mv && rr >= 0 && x >= 1;
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
            done = done || i < 1 || j < 1;  // row 0 / column 0: H = 0
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
    // then the pairs the dual fill handed back ('-' bytes; usually none), one
    // wave per pair in the one-pair walk over their blocked codes
    if (a.fb_count) {
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

hipError_t launch_walk_ck(const TraceArgs& a, hipStream_t s) {
    const uint32_t per_block = kWavesPerBlock * kCkPairs;
    hipLaunchKernelGGL(traceback_ck_kernel, dim3((a.count + per_block - 1) / per_block), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace ta
