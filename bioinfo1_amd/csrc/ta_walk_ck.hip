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
// with gap <= 0 and no '-' (the planner and the fill's hand-back flag route
// everything else elsewhere) a gap move never lowers the cost, and the walk
// ends on the first cell with H = 0.
//
// A window is the 16 rows of the walk's stripe g over the columns c0 + 1 .. j,
// j the walk's column and c0 the stripe's nearest checkpoint at least kCkLead
// columns to its left (or column 0), so W = j - c0 <= 32.  Its operands: the
// checkpoint column (left), stripe g - 1's stored bottom row over c0 .. j
// (top), the target and query bytes.
//
// Geometry (r06): 8 lanes per two pairs, 16 pairs per wave.  Lane lg of a group
// holds rows 2 lg and 2 lg + 1 of its stripe for BOTH pairs of the group, packed
// in int16 halves (pair A low, pair B high).  The lanes sweep the window's
// anti-diagonals -- lane lg computes column x = k - lg + 1 at step k, W + 7
// steps -- the first row's up value from the lane above by DPP row_shr:1 (the
// group's first lane: the top row), the second row's from the first.  Values
// are H + gap + B with B = mag + 1, so every value and candidate is a
// non-negative int16 below 0x7BFF (H <= 2047 in a dual plan, ta_planner.cpp
// fits_int16): the clamp and both maxima are one v_pk_maximum3_f16
// (ta_packed.h pk_max3_pos).  Each step's D, I and H = 0 signs of both rows and
// both pairs (12 bits) go into three byte accumulators per 8 steps
// (sign_bytes + one bit insert, as the dual fill's codes).  Per pair and row
// three 32-bit words then go to LDS (column x at bit W - x): NI (cells whose
// move is NOT I-only), D, and H = 0.  The walk crosses the window one row per
// step (lanes 0-3 of a group: its first pair, 4-7: its second): stop on a
// cell with H = 0, else the run of I moves up to the first NI bit, then the D
// or M move up; it leaves through the top (stripe g - 1, same column) or, when
// the I run reaches c0, through the left edge (the same stripe, the next
// checkpoint left).  Each row step lists a record; the window's events for
// format_runs_kernel (D run above bit 16, count of the move in bits 15:2, move
// in bits 1:0) are made from the records by the pair's 4 lanes.
//
// r05's kernel (16 lanes per two pairs, one row each, 8 pairs per wave) swept
// a fixed 48 steps for 32 cells per lane; here 40 steps cover 64 cells per lane,
// and the walk's row steps and window loads serve 16 pairs per instruction
// instead of 8.
#include "ta_device.h"
#include "ta_packed.h"

namespace ta {
namespace {

constexpr int kCkLead = 17;            // columns a window reaches left of the walk's column, at least
constexpr int kCkMaxW = kCkLead + 15;  // the widest window (checkpoints 16 columns apart)
constexpr int kCkLanes = 8;            // lanes per group (two pairs, two rows per lane)
constexpr int kCkGroups = kWave / kCkLanes;
constexpr int kCkBlocks = 5;           // sweep blocks of 8 steps
static_assert(kCkMaxW + kCkLanes - 1 <= 8 * kCkBlocks, "a window's sweep fits the blocks");
static_assert(8 * kCkBlocks <= 40, "a row's steps fit 40 bits (one byte + one dword)");

struct CkGroup {
    uint32_t top[8 * kCkBlocks + 1];     // per x: both pairs' H(16g, c0 + x) + gap + B (int16 halves)
    // per x (at 8 + x): both pairs' gain tables of the target byte (TAB windows: .x pair
    // A's, .y pair B's, ckGainTable), else their target bytes (.x bits 7:0, 23:16)
    uint2 tb[8 + 8 * kCkBlocks + 1];
    // (after top / tb: the walk reads the row above row 0 -- up to 18 rows -- of
    // walkers that already left, from inside the group)
    uint2 row[2][16];                    // per pair and row: NI, D window words
    uint32_t rec[2][16];                 // per pair: the window's row steps
    uint8_t qb[2][16];                   // local: per pair, the query bytes of the stripe's rows
};
static_assert(offsetof(CkGroup, row) >= 18 * sizeof(uint2), "room above a walker's row 0");

// TAB windows (every query row of both pairs is A, C, G or T; ta_packed.h
// mismatch_table): the diagonal gain of a cell is a byte of its column's gain
// table -- byte k = (s - gap) + 128 for the query letter of class k, s = match
// when the target byte is that letter, else mismatch -- picked for both pairs by
// one v_perm with the row's selector (row_selector: pair A's byte in bits 7:0,
// B's in 23:16) and added as ONE 32-bit add3 with -128 * 65537.  Exact when both
// halves of the sum lie in [0, 2^16): true of every value the window holds for a
// column x <= W of its pair, and kept true past W by masking the top row and the
// rows past n to H = 0 (a borrow from pair A's half would change pair B's cell).
__device__ __forceinline__ uint32_t ck_gain_table(uint32_t c, int ua, int ub) {
    const uint32_t k = (c >> 1) & 3u;
    const bool hit = c == ((0x47544341u >> (8u * k)) & 0xFFu);  // 'A', 'C', 'T', 'G'
    const uint32_t t = (uint32_t)ub * 0x01010101u;
    return hit ? (t & ~(0xFFu << (8u * k))) | ((uint32_t)ua << (8u * k)) : t;
}

__device__ __forceinline__ void ck_wave_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// The pairs the dual fill handed back ('-' bytes; usually none), one wave per
// pair in the one-pair walk over their blocked codes -- here rather than in a
// launch of its own, whose count only the device knows.
template <int MODE>
__device__ __forceinline__ void ck_fallback_walks(const TraceArgs& a, int lane) {
    if (!a.fb_count) return;
    const uint32_t nfb = *a.fb_count;
    for (uint32_t w = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); w < nfb; w += gridDim.x * kWavesPerBlock) {
        const uint32_t q = a.fb_order[w];
        const uint32_t qn = a.qlen[q], qm = a.tlen[q];
        uint64_t st;
        uint32_t len;
        const WalkSeq seq{a.qbytes + a.qoff[q], a.tbytes + a.toff[q], a.score[q], a.match, a.mismatch, a.gap};
        traceback_pair<MODE>(a.ptrs + a.ptr_off[q], qn, qm, a.goal_i[q], a.goal_j[q], a.slots + a.slot_off[q],
                               cigar_slot_bytes(qn, qm), lane, &st, &len, seq, true);
        if (lane == 0) {
            a.cigar_start[q] = a.slot_off[q] + st;
            a.cigar_len[q] = len;
        }
    }
}

// DPP within a 4-lane quad (a walker's lanes): quad_perm(sel)
template <int SEL>
__device__ __forceinline__ uint32_t quad(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, SEL, 0xF, 0xF, false);
}

// Per-pair constants, held by every lane of the pair's group.
struct CkPair {
    uint32_t p, n, m, nb;
    int off, z, dl;  // the fill's frame (ta_layout.h ck_decode)
    bool fx;         // a pair of the flexible fill (pflag 2): its checkpoints hold H itself
    const uint16_t* P;
    const uint8_t* Q;
    const uint8_t* T;
    bool has;
};

// (<= 128 VGPRs: beside the next batch's fill -- 96 VGPRs a wave -- a walk wave then displaces
// one fill wave of its SIMD, not two)
template <int MODE>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void traceback_ck_kernel(TraceArgs a) {
    constexpr bool LOCAL = MODE == kLocal;
    __shared__ CkGroup groups[kWavesPerBlock * kCkGroups];
    __shared__ uint32_t gtab[256];  // per byte value: local: ck_gain_table; global / semi: mismatch_table
    // a latency-bound chain: beside the next batch's fill (align.DevicePipeline)
    // its instructions go first at the SIMD's issue arbiter (measured neutral)
    __builtin_amdgcn_s_setprio(3);
    const int lane = (int)threadIdx.x & 63, lg = lane & 7, hh = lg >> 2, lw = lg & 3;
    CkGroup& G = groups[threadIdx.x >> 3];
    const int ma = a.match, mi = a.mismatch, gap = a.gap;
    const int mag = max(max(max(ma, -ma), max(mi, -mi)), max(max(gap, -gap), 1));
    const int B = mag + 1;   // bias: values H + gap + B >= 1
    const int GB = gap + B;  // the value of a cell with H = 0
    // global / semi: the values are the fill's own S = H - ma j + gap (j - i) (ta_dual.hip,
    // int16 by fits_int16): the diagonal gain is (s - ma), the up one 0, the left one 2 gap - ma;
    // row 0 holds S(0, j) = R0 j, column 0 S(i, 0) = C0 i (:81-92)
    const int R0 = (MODE == kGlobal ? gap : 0) - ma + gap, C0 = MODE == kGlobal ? 0 : -gap;
    CkPair S[2];
    int ci[2], cj[2];        // the walk's current cell of each pair
    int hc[2];               // local: its H (the cost the walk carries)
    bool live[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        CkPair& c = S[h];
        const uint32_t slot = ((blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * kCkGroups + (uint32_t)(lane >> 3)) * 2 + h;
        c.has = slot < a.count;
        c.p = c.has ? (a.order ? a.order[a.begin + slot] : a.begin + slot) : 0u;
        // the fills' flag: 1 handed back ('-' bytes: the fallback walk), 2 the flexible fill's
        const uint32_t pf = (c.has && a.pflag) ? a.pflag[c.p] : 0u;
        if (pf == 1u) c.has = false;
        c.fx = pf == 2u;
        c.n = c.m = 0;
        c.P = reinterpret_cast<const uint16_t*>(a.ptrs);
        c.Q = a.qbytes;
        c.T = a.tbytes;
        ci[h] = cj[h] = 0;
        int H = 0;
        if (c.has) {
            c.n = a.qlen[c.p];
            c.m = a.tlen[c.p];
            ci[h] = (int)a.goal_i[c.p];
            cj[h] = (int)a.goal_j[c.p];
            H = LOCAL ? a.score[c.p] : min(ci[h], cj[h]);  // (global / semi: a walk to row 0 or column 0)
            c.P = reinterpret_cast<const uint16_t*>(a.ptrs + a.ptr_off[c.p]);
            c.Q += a.qoff[c.p];
            c.T += a.toff[c.p];
        }
        // the checkpoint fill's frame (ck_decode): the equal-gain one with three-input maxima
        const int off3 = (LOCAL && c.has && !c.fx) ? local_max3_offset(c.n, c.m, ma, mi, gap, true) : -1;
        c.off = off3 >= 0 ? off3 : 0;
        c.z = local_max3_z(ma, off3 >= 0);
        c.dl = off3 >= 0 ? c.z + 16 : 0;
        c.nb = blk_count(c.m);
        live[h] = c.has && H > 0;  // a positive score has its goal at i, j >= 1
        hc[h] = H;
    }
    // the walker's own pair (lanes 0-3: pair A, 4-7: pair B)
    const bool mhas = hh ? S[1].has : S[0].has;
    const uint32_t mp = hh ? S[1].p : S[0].p, mnm = hh ? S[1].n + S[1].m : S[0].n + S[0].m;
    uint32_t* const rout = a.runs + (mhas ? band_runs_off(a.slot_off[mp]) : 0);
    const uint32_t cap = 2 * mnm - 1;  // the walk's room (ta_internal.h band_runs_off)
    uint32_t nev = 0, kI = 0, windows = 0;       // events listed; the pending I run (across windows)
    bool mdone = !(hh ? live[1] : live[0]);      // (a pair with score 0 has nothing to walk)
    int mcost = hh ? hc[1] : hc[0];              // local: H of the walker's cell
    // runs of one op in events of at most 8192 (the count fields: 14 bits for I, 16 for D);
    // never past the pair's room (a walk moves >= 1 cell per event of its records, so with the
    // trailing and boundary runs its events stay <= n + m + 4 <= cap for n + m >= 3; a full
    // room marks the walk unfinished, the plan's error word)
    bool capped = false;
    auto emit = [&](bool ins, uint32_t c) {
        while (c) {
            const uint32_t k = min(c, 8192u);
            capped |= nev >= cap;
            if (lw == 0 && nev < cap) rout[nev] = ins ? (k << 2) | 1u : (k << 16) | 3u;
            nev += nev < cap ? 1u : 0u;
            c -= k;
        }
    };
    if (!LOCAL && mhas) {
        // semi-global: the goal's trailing run to column m / row n comes last in the CIGAR,
        // first in the walk (:306-315); a goal on row 0 / column 0 is only the boundary run
        const int gi = hh ? ci[1] : ci[0], gj = hh ? cj[1] : cj[0];
        const uint32_t n = hh ? S[1].n : S[0].n, m = hh ? S[1].m : S[0].m;
        if (MODE == kSemi && (uint32_t)gi == n && (uint32_t)gj < m) emit(true, m - (uint32_t)gj);
        else if (MODE == kSemi && (uint32_t)gj == m && (uint32_t)gi < n) emit(false, n - (uint32_t)gi);
        if (gi < 1) emit(true, (uint32_t)gj);
        else if (gj < 1) emit(false, (uint32_t)gi);
    }
    const uint32_t SA2 = rep16(ma - gap), GAP2 = rep16(gap), KD2 = rep16(mi - ma), B2 = rep16(B);
    const uint32_t GB2 = rep16(GB);
    uint32_t ONE = 0x00010001u;
    asm volatile("" : "+s"(ONE));  // (see ta_packed.h pk_min_u16)
    const bool first = lg == 0;
    // TAB windows need both gains (s - gap) in [-128, 127]
    const int ua = ma - gap + 128, ub = mi - gap + 128;
    const bool tab_ok = !LOCAL || ((uint32_t)ua < 256u && (uint32_t)ub < 256u);
    const uint32_t GL2 = rep16(2 * gap - ma), KE2 = rep16(mi - ma);  // (global / semi gains)
    gtab[threadIdx.x] = LOCAL ? ck_gain_table(threadIdx.x, ua, ub) : mismatch_table(threadIdx.x);  // (kBlock == 256)
    static_assert(kBlock == 256, "one gain table entry per thread");
    __syncthreads();
    uint32_t KN = swar_k(-128);
    asm volatile("" : "+s"(KN));
    uint32_t acc[2][kCkBlocks];
#pragma unroll
    for (int b = 0; b < kCkBlocks; ++b) acc[0][b] = acc[1][b] = 0u;

    while (ballot(live[0] || live[1])) {
        // ---- both pairs' windows: loads first (one wait for all), then the decodes
        int g[2], r[2], c0[2], W[2];
        uint32_t vl[2], vt[2][5], vb[2][4], vq[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const CkPair& c = S[h];
            g[h] = live[h] ? (ci[h] - 1) >> 4 : 0;
            r[h] = live[h] ? (ci[h] - 1) & 15 : 0;
            const int l = g[h] & 63;
            const int e = cj[h] - kCkLead + l;
            // block (e >> 4) - 1's checkpoint column, or column 0 when that block ended
            // before the stripe's first column (16 (b + 1) - l <= 0: j <= 32 then)
            c0[h] = e >= 16 ? max((e >> 4) * 16 - l, 0) : 0;
            W[h] = live[h] ? cj[h] - c0[h] : 0;
            // left: rows 2 lg, 2 lg + 1 of checkpoint column c0 (two adjacent int16, one dword)
            const bool hl = live[h] && c0[h] > 0;
            const uint32_t li = hl ? (uint32_t)ck_col_index((uint32_t)g[h] >> 6, (uint32_t)(e >> 4) - 1u, (uint32_t)l, c.nb,
                                                            2u * (uint32_t)lg) : 0u;
            vl[h] = *reinterpret_cast<const uint32_t*>(c.P + li);
            // top: stripe g - 1's bottom row at columns c0 + x, x = lg + 8q (its step c0 + x + lu - 1);
            // stripe 0 reads a dummy (its top row is row 0: H = 0)
            // (ck_row_index in int: step t0 is -1 for column 0 of lane 0 when lu = 0 -- a value
            // masked below, loaded from index 0 instead -- and then block -1 + 1 is step 15's)
            const bool ht = live[h] && g[h] > 0;
            const int gu = ht ? g[h] - 1 : 0, lu = gu & 63, pu = gu >> 6;
            const int t0 = ht ? c0[h] + lg + lu - 1 : 0, t1 = t0 + 8;
            const int base = ht ? pu * (int)c.nb * 2048 + lu * 16 : 0;
            const int i0 = base + (t0 >> 4) * 1024 + (t0 & 15), i1 = base + (t1 >> 4) * 1024 + (t1 & 15);
            vt[h][0] = c.P[max(i0, 0)];
            vt[h][1] = c.P[i1];
            vt[h][2] = c.P[i0 + 1024];  // (16 columns on: the next block, same step within it)
            vt[h][3] = c.P[i1 + 1024];
            vt[h][4] = c.P[i0 + 2048];
            // target bytes of columns x = 1 + lg + 8q (only x <= W: the last pair's bytes end the buffer)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int x = 1 + lg + 8 * q;
                vb[h][q] = x <= W[h] ? (uint32_t)c.T[c0[h] + x - 1] : 0u;
            }
            // query bytes of the lane's rows (rows past n: any byte, below the walk; pairs
            // not walking: 'A', which keeps a TAB window)
            const uint32_t ir = 16u * (uint32_t)g[h] + 2u * (uint32_t)lg;  // the first row - 1
            const uint32_t qn = c.n ? c.n - 1u : 0u;
            vq[h][0] = live[h] ? c.Q[min(ir, qn)] : 0x41u;
            vq[h][1] = live[h] ? c.Q[min(ir + 1u, qn)] : 0x41u;
        }
        // decodes (ta_layout.h ck_decode, plus gap + B): v = (s - off - z j + i - dl l) / 16 + gap + B
        // is exact in 16-bit wrap-around arithmetic ((s + C) mod 2^16 = 16 (H + gap + B) < 2^16),
        // so both pairs decode together: one packed add of C and one packed shift
        uint32_t gl0, gl1, q0, q1, mT = 0, mL0 = 0, mL1 = 0;
        bool acgt = true;
        {
            int CL[2], CT[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const CkPair& c = S[h];
                const int l = g[h] & 63, lu = (g[h] - 1) & 63;
                const int ir = 16 * g[h] + 2 * lg + 1;  // the lane's first row
                CL[h] = 16 * GB - c.off - c.z * c0[h] + ir - c.dl * l;
                CT[h] = 16 * GB - c.off - c.z * (c0[h] + lg) + 16 * g[h] - c.dl * lu;
                // (rows past n: H = 0 too, see ck_gain_table)
                const bool hl = live[h] && c0[h] > 0;
                mL0 |= (hl && ir <= (int)c.n) ? 0xFFFFu << (16 * h) : 0u;
                mL1 |= (hl && ir + 1 <= (int)c.n) ? 0xFFFFu << (16 * h) : 0u;
                mT |= (live[h] && g[h] > 0) ? 0xFFFFu << (16 * h) : 0u;
                acgt = acgt && is_acgt(vq[h][0]) && is_acgt(vq[h][1]);
            }
            const uint32_t cl = ((uint32_t)CL[0] & 0xFFFFu) | ((uint32_t)CL[1] << 16);
            const uint32_t ct = ((uint32_t)CT[0] & 0xFFFFu) | ((uint32_t)CT[1] << 16);
            const uint32_t l0 = __builtin_amdgcn_perm(vl[1], vl[0], 0x05040100u);  // row 2 lg of A, B
            const uint32_t l1 = __builtin_amdgcn_perm(vl[1], vl[0], 0x07060302u);  // row 2 lg + 1
            // column 0 (c0 = 0, x = 0): the boundary
            const uint32_t m0 = mT & (lg == 0 ? ((c0[0] > 0 ? 0xFFFFu : 0u) | (c0[1] > 0 ? 0xFFFF0000u : 0u)) : ~0u);
            if constexpr (LOCAL) {
                // (flexible-fill pairs: H itself, + gap + B)
                const uint32_t fx = (S[0].fx ? 0xFFFFu : 0u) | (S[1].fx ? 0xFFFF0000u : 0u);
                auto dec = [&](uint32_t v, uint32_t c) { return vsel(fx, pk_add(v, GB2), pk_lshr4(pk_add(v, c))); };
                gl0 = vsel(mL0, dec(l0, cl), GB2);
                gl1 = vsel(mL1, dec(l1, pk_add(cl, ONE)), GB2);
                // the decode constant moves by -z per column
                const uint32_t dx = ((uint32_t)(-8 * S[0].z) & 0xFFFFu) | ((uint32_t)(-8 * S[1].z) << 16);
                uint32_t ctq = ct;
#pragma unroll
                for (int q = 0; q < 5; ++q) {
                    // (columns past W: H = 0, see ck_gain_table)
                    const int x = lg + 8 * q;
                    const uint32_t mw = (x <= W[0] ? 0xFFFFu : 0u) | (x <= W[1] ? 0xFFFF0000u : 0u);
                    const uint32_t s = vt[0][q] | (vt[1][q] << 16);
                    G.top[x] = vsel((q == 0 ? m0 : mT) & mw, dec(s, ctq), GB2);
                    ctq = pk_add(ctq, dx);
                }
            } else {
                // the stored S values as they are; the boundaries computed: column 0 S(i, 0) =
                // C0 i, row 0 S(0, j) = R0 j (stripe 0's top row).  Flexible-fill pairs store H,
                // whose S can pass int16 on long pairs: the window holds S - Sb instead, Sb the
                // bias part of S at its corner (16 g, c0) (-ma c0 + gap (c0 - 16 g)), i.e. H
                // - gap (i - 16 g) down the left column and H + (gap - ma) x along the top row
                auto pack = [](int a0, int a1) { return ((uint32_t)a0 & 0xFFFFu) | ((uint32_t)a1 << 16); };
                int sb[2], al[2], at[2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    sb[h] = S[h].fx ? -ma * c0[h] + gap * (c0[h] - 16 * g[h]) : 0;
                    al[h] = S[h].fx ? -gap * (2 * lg + 1) : 0;  // the lane's first row
                    at[h] = S[h].fx ? (gap - ma) * lg : 0;       // column x = lg
                }
                const uint32_t SB = pack(sb[0], sb[1]), AL = pack(al[0], al[1]), AT = pack(at[0], at[1]);
                const uint32_t AG = pack(S[0].fx ? -gap : 0, S[1].fx ? -gap : 0);
                const uint32_t AX = pack(S[0].fx ? 8 * (gap - ma) : 0, S[1].fx ? 8 * (gap - ma) : 0);
                const int ir0 = 16 * g[0] + 2 * lg + 1, ir1 = 16 * g[1] + 2 * lg + 1;
                const uint32_t cb = pk_sub(pack(C0 * ir0, C0 * ir1), SB);
                const uint32_t mE = (live[0] && c0[0] > 0 ? 0xFFFFu : 0u) | (live[1] && c0[1] > 0 ? 0xFFFF0000u : 0u);
                gl0 = vsel(mE, pk_add(l0, AL), cb);
                gl1 = vsel(mE, pk_add(l1, pk_add(AL, AG)), pk_add(cb, rep16(C0)));
                const uint32_t rowb = pk_sub(pack(R0 * (c0[0] + lg), R0 * (c0[1] + lg)), SB);
                const uint32_t colb = pk_sub(pack(C0 * 16 * g[0], C0 * 16 * g[1]), SB);
                uint32_t rq = rowb, aq = AT;
#pragma unroll
                for (int q = 0; q < 5; ++q) {
                    const uint32_t s = pk_add(vt[0][q] | (vt[1][q] << 16), aq);
                    const uint32_t alt = q == 0 ? vsel(mT, colb, rq) : rq;  // (q > 0: column > 0)
                    G.top[lg + 8 * q] = vsel(q == 0 ? m0 : mT, s, alt);
                    rq = pk_add(rq, rep16(8 * R0));
                    aq = pk_add(aq, AX);
                }
            }
        }
        if constexpr (LOCAL) {
#pragma unroll
            for (int h = 0; h < 2; ++h) *reinterpret_cast<uint16_t*>(&G.qb[h][2 * lg]) = (uint16_t)(vq[h][0] | (vq[h][1] << 8));
        }
        // the window's sweep kind (wave-uniform): TAB when every query row is A, C, G, T
        const bool tab = tab_ok && !ballot(!acgt);
        if (tab) {
#pragma unroll
            for (int q = 0; q < 4; ++q) G.tb[9 + lg + 8 * q] = make_uint2(gtab[vb[0][q]], gtab[vb[1][q]]);
            q0 = row_selector(vq[0][0], vq[1][0]);
            q1 = row_selector(vq[0][1], vq[1][1]);
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) G.tb[9 + lg + 8 * q] = make_uint2(vb[0][q] | (vb[1][q] << 16), 0u);
            q0 = vq[0][0] | (vq[1][0] << 16);
            q1 = vq[0][1] | (vq[1][1] << 16);
        }
        ck_wave_sync();

        // ---- the sweep: step k, lane lg computes column x = k - lg + 1 of its two rows of both pairs
        const int need = max(W[0], W[1]) + kCkLanes - 1;  // steps this lane's pairs need
        uint32_t upp = G.top[0];  // the previous step's up candidate of row 2 lg (lane 0: H(16g, c0) + gap + B)
        const uint2* tbl = &G.tb[9 - lg];
        auto block = [&](auto kb_tag, auto tab_tag) {
            constexpr int kb = decltype(kb_tag)::value;
            constexpr bool TAB = decltype(tab_tag)::value;
            uint32_t tv[8];
            uint2 bv[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                tv[s] = G.top[kb + s + 1];
                if constexpr (TAB) bv[s] = tbl[kb + s];
                else bv[s].x = tbl[kb + s].x;
            }
            uint32_t a0 = acc[0][kb / 8], a1 = acc[1][kb / 8];
            if constexpr (!LOCAL) {
                // global / semi: S values, no clamp; D and I signs of saturating differences
                // (S and its candidates are int16 -- fits_int16 -- their differences need not be)
#pragma unroll
                for (int s = 0; s < 8; ++s) {
                    const uint32_t dpp = (uint32_t)__builtin_amdgcn_mov_dpp((int)gl1, 0x111, 0xF, 0xF, true);
                    const uint32_t up0 = first ? tv[s] : dpp;
                    const uint32_t e0 = TAB ? mismatch_flags(bv[s].x, bv[s].y, q0) : pk_min_u16(q0 ^ bv[s].x, ONE);
                    const uint32_t e1 = TAB ? mismatch_flags(bv[s].x, bv[s].y, q1) : pk_min_u16(q1 ^ bv[s].x, ONE);
                    const uint32_t dg0 = pk_mad_i16(e0, KE2, upp), lf0 = pk_add(gl0, GL2);
                    const uint32_t m10 = pk_max(dg0, lf0), hn0 = pk_max(m10, up0);
                    const uint32_t dg1 = pk_mad_i16(e1, KE2, gl0), lf1 = pk_add(gl1, GL2);
                    const uint32_t m11 = pk_max(dg1, lf1), hn1 = pk_max(m11, hn0);
                    const uint32_t mk = 0x01010101u << (7 - s);
                    a0 = bfi(mk, sign_bytes(pk_sub_sat(m10, up0), pk_sub_sat(dg0, lf0)), a0);  // [I0A, I0B, D0A, D0B]
                    a1 = bfi(mk, sign_bytes(pk_sub_sat(m11, hn0), pk_sub_sat(dg1, lf1)), a1);  // [I1A, I1B, D1A, D1B]
                    if (kb >= 8 || kb + s >= lg) {
                        gl0 = hn0;
                        gl1 = hn1;
                    }
                    upp = up0;
                }
                acc[0][kb / 8] = a0;
                acc[1][kb / 8] = a1;
                return;
            }
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                // the first row: up from the lane above's second row (row_shr:1; a
                // group's first lane: the top row), diagonal = the previous step's up
                const uint32_t dpp = (uint32_t)__builtin_amdgcn_mov_dpp((int)gl1, 0x111, 0xF, 0xF, true);
                const uint32_t up0 = first ? tv[s] : dpp;
                uint32_t dg0, dg1;
                if constexpr (TAB) dg0 = upp + mismatch_flags(bv[s].x, bv[s].y, q0) + KN;  // (v_add3_u32)
                else dg0 = pk_mad_i16(pk_min_u16(q0 ^ bv[s].x, ONE), KD2, pk_add(upp, SA2));
                const uint32_t m10 = pk_max(dg0, gl0);
                const uint32_t hn0 = pk_max3_pos(m10, up0, B2);  // H + B (clamp at H = 0)
                const uint32_t gn0 = pk_add(hn0, GAP2);
                // the second row: up = the first row's new value, diagonal = its previous one
                if constexpr (TAB) dg1 = gl0 + mismatch_flags(bv[s].x, bv[s].y, q1) + KN;
                else dg1 = pk_mad_i16(pk_min_u16(q1 ^ bv[s].x, ONE), KD2, pk_add(gl0, SA2));
                const uint32_t m11 = pk_max(dg1, gl1);
                const uint32_t hn1 = pk_max3_pos(m11, gn0, B2);
                const uint32_t gn1 = pk_add(hn1, GAP2);
                // signs: D (up beats both), I (left beats the diagonal)
                const uint32_t mk = 0x01010101u << (7 - s);
                a0 = bfi(mk, sign_bytes(pk_sub(m10, up0), pk_sub(dg0, gl0)), a0);   // [I0A, I0B, D0A, D0B]
                a1 = bfi(mk, sign_bytes(pk_sub(m11, gn0), pk_sub(dg1, gl1)), a1);   // [I1A, I1B, D1A, D1B]
                if (kb >= 8 || kb + s >= lg) {  // (ramp: columns <= 0 keep the checkpoint)
                    gl0 = gn0;
                    gl1 = gn1;
                }
                upp = up0;
            }
            acc[0][kb / 8] = a0;
            acc[1][kb / 8] = a1;
        };
        auto sweep = [&](auto tab_tag) {
            block(std::integral_constant<int, 0>{}, tab_tag);
            block(std::integral_constant<int, 8>{}, tab_tag);
            if (ballot(need > 16)) {
                block(std::integral_constant<int, 16>{}, tab_tag);
                if (ballot(need > 24)) {
                    block(std::integral_constant<int, 24>{}, tab_tag);
                    if (ballot(need > 32)) block(std::integral_constant<int, 32>{}, tab_tag);
                }
            }
        };
        if (tab) sweep(std::true_type{});
        else sweep(std::false_type{});
        // Per pair and row: step k at bit 39 - k of a 40-bit row (block b's byte at bits
        // 8 (4 - b)); column x = k - lg + 1 at bit W - x of the window word: bits
        // [8 - lg, 40 - lg) of the row, shifted down by 32 - W.  (Steps past the blocks
        // that ran hold stale bits; they are columns past W and fall off.)
        auto word = [&](const uint32_t (&ac)[kCkBlocks], uint32_t bi, int Wh) -> uint32_t {
            const uint32_t lo = __builtin_amdgcn_perm(ac[1], ac[2], ((4u + bi) << 24) | (bi << 16) | 0x0C0Cu) |
                                __builtin_amdgcn_perm(ac[3], ac[4], 0x0C0C0000u | ((4u + bi) << 8) | bi);
            const uint32_t w32 = __builtin_amdgcn_alignbit(ac[0] >> (8u * bi), lo, (uint32_t)(8 - lg));
            return w32 >> ((uint32_t)(32 - Wh) & 31u);
        };
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t i0 = word(acc[0], (uint32_t)h, W[h]), d0 = word(acc[0], 2u + h, W[h]);
            const uint32_t i1 = word(acc[1], (uint32_t)h, W[h]), d1 = word(acc[1], 2u + h, W[h]);
            G.row[h][2 * lg] = make_uint2(~i0 | d0, d0);
            G.row[h][2 * lg + 1] = make_uint2(~i1 | d1, d1);
        }
        ck_wave_sync();

        // ---- the walk across the window, one row per step (lanes 0-3: pair A, 4-7: pair B):
        // the I run from the current column (up to the first NI bit, at most to column 0),
        // then the D or M move out of the row -- or, when the run reaches column c0, on in
        // the next window.  Flags as 0 / 1 integers; the loop keeps only what the next step
        // depends on and lists each step's record; the events come from the records.  A local
        // walk also stops on the first cell with H = 0 (its cost, :20-28): found after the
        // loop from the records, whose moves fix the cost of every cell on the path.
        const int mr = hh ? r[1] : r[0], mW = hh ? W[1] : W[0], mg = hh ? g[1] : g[0], mc0 = hh ? c0[1] : c0[0];
        const bool mlive = hh ? live[1] : live[0];
        // (<= 2 events per row step, + an I-run split; the boundary runs check their own room)
        const bool room = nev + 2u * (uint32_t)(mr + 1) + 1u <= cap;
        uint32_t wl = (mlive && room) ? 1u : 0u, nrec = 0, pos = 0;
        int rr = mr;
        const uint2* rp = &G.row[hh][rr - 1];  // the row a move up reaches (a walk only moves up)
        uint32_t* recs = G.rec[hh];
        uint32_t* recp = recs;                  // step k's record at recs[k] (the steps of a live walk are its records)
        auto row_step = [&](const uint2& w2, uint32_t* rec) {
            // (NI's bit W is set when W < 32; a run to the edge of a 32-column window finds no
            // NI bit, hence the 33rd bit and the bound)
            const uint32_t run = min((uint32_t)__builtin_ctzll((uint64_t)(w2.x >> pos) | (1ull << 32)), (uint32_t)mW - pos);
            const uint32_t p1 = pos + run;
            const uint32_t edge = p1 >= (uint32_t)mW ? 1u : 0u;
            const uint32_t dmove = (w2.y >> (p1 & 31u)) & 1u;
            const uint32_t mv = wl & (edge ^ 1u);
            *rec = run | (dmove << 8) | (edge << 9) | (p1 << 10);  // (p1: the move's column, bit W - x)
            nrec += wl;
            pos += (wl ? run : 0u) + (mv & (dmove ^ 1u));  // (a select: v_mul_lo_u32 is quarter rate)
            rr -= (int)mv;
            wl = mv & ((uint32_t)~rr >> 31) & (pos < (uint32_t)mW ? 1u : 0u);
        };
        // Two steps per loop iteration with the row words read one step ahead
        // into alternating registers (a single one became a copy at the loop's
        // end, which waited for the read).
        uint2 wa = rp[1], wb;
        while (ballot(wl != 0u)) {
            wb = rp[0];
            __builtin_amdgcn_sched_barrier(0);  // (issued here, not sunk to its use)
            row_step(wa, recp);
            if (!ballot(wl != 0u)) break;
            wa = rp[-1];
            __builtin_amdgcn_sched_barrier(0);
            row_step(wb, recp + 1);
            rp -= 2;
            recp += 2;
        }
        ck_wave_sync();
        // events of the records: an I run (with the run carried from the previous window
        // on the first record) and the D or M move; a record that ran to the window's edge
        // carries its run to the next window.  Consecutive M moves with no I run between
        // them are one event, written at the run's last record (the formatter's work
        // goes with the events: ~1,000 a config-2 pair, about half of them M moves that
        // continue an M run).  Records 4 lw .. 4 lw + 3 per lane; the pair's M-move and
        // no-I-run masks over its 16 records are OR-ed over the pair's 4 lanes.
        bool zstop = false;
        if constexpr (LOCAL) {
            // the cost before record k: H(k + 1) = H(k) - gap (run + a D move) - s (an M move,
            // s of the cell it leaves: query row mr - k, column x = W - p1); the walk ends on
            // the first record k in 1 .. nrec with H(k) = 0 (a gap move never lowers H, so only
            // after an M move).  Records 4 lw .. 4 lw + 3 per lane, prefix over the quad.
            int dk[4], sum = 0;
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const uint32_t k = 4u * (uint32_t)lw + (uint32_t)h;
                const uint32_t rc = k < nrec ? recs[k] : 0x200u;
                const bool ed = rc & 0x200u, dm = rc & 0x100u;
                const uint32_t x = (uint32_t)mW - ((rc >> 10) & 63u);  // (p1 <= W: x in 0 .. 32)
                const uint2 tv = G.tb[8u + x];
                const uint32_t q = G.qb[hh][(uint32_t)(mr - (int)k) & 15u];
                int sc;
                if (tab) sc = (int)(((hh ? tv.y : tv.x) >> (8u * ((q >> 1) & 3u))) & 0xFFu) - 128 + gap;  // ck_gain_table
                else sc = ((tv.x >> (16 * hh)) & 0xFFu) == q ? ma : mi;
                dk[h] = -gap * (int)((rc & 63u) + (!ed && dm ? 1u : 0u)) - (!ed && !dm ? sc : 0);
                sum += dk[h];
            }
            int inc = sum;
            const int s1 = (int)quad<0x90>((uint32_t)inc);
            inc += lw >= 1 ? s1 : 0;
            const int s2 = (int)quad<0x40>((uint32_t)inc);
            inc += lw >= 2 ? s2 : 0;
            const int tot = (int)quad<0xFF>((uint32_t)inc);
            int hk = mcost + inc - sum;  // H before record 4 lw
            uint32_t zf = 0;
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const uint32_t k = 4u * (uint32_t)lw + (uint32_t)h;
                zf |= (k >= 1u && k <= nrec && hk == 0) ? 1u << k : 0u;
                hk += dk[h];
            }
            zf |= (lw == 3 && nrec >= 16u && hk == 0) ? 1u << 16 : 0u;  // after the 16th record
            const uint32_t z1 = quad<0xB1>(zf);
            zf |= z1;
            const uint32_t z2 = quad<0x4E>(zf);
            zf |= z2;
            const uint32_t kz = (uint32_t)__builtin_ctz(zf | (1u << 17));
            zstop = kz <= nrec;
            nrec = min(nrec, kz);
            mcost += tot;  // (stopped: no longer read)
        }
        {
            uint32_t rcs[4], mm = 0, zm = 0;
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const uint32_t k = 4u * (uint32_t)lw + (uint32_t)h;
                rcs[h] = k < nrec ? recs[k] : 0x200u;  // (past the list: no event)
                const uint32_t runI = (rcs[h] & 63u) + (k == 0 ? kI : 0u);
                mm |= ((rcs[h] & 0x300u) == 0 ? 1u : 0u) << k;  // an M move
                zm |= (runI == 0 ? 1u : 0u) << k;
            }
            const uint32_t o1 = quad<0xB1>(mm), z1 = quad<0xB1>(zm);  // quad_perm [1, 0, 3, 2]
            mm |= o1;
            zm |= z1;
            const uint32_t o2 = quad<0x4E>(mm), z2 = quad<0x4E>(zm);  // quad_perm [2, 3, 0, 1]
            mm |= o2;
            zm |= z2;
            const uint32_t cont = mm & zm & (mm << 1);  // record k continues record k - 1's M run
            uint32_t ev[8], ne = 0;
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const uint32_t k = 4u * (uint32_t)lw + (uint32_t)h, rc = rcs[h];
                const uint32_t runI = (rc & 63u) + (k == 0 ? kI : 0u);
                const bool ed = rc & 0x200u, iev = !ed && runI > 0;
                // an M run ending here: its first record is the last one at or below k that
                // does not continue a run (bit 0 never does)
                const uint32_t below = ~cont & ((2u << k) - 1u);
                const uint32_t mcount = k + 1u - (31u - (uint32_t)__builtin_clz(below));
                const bool mend = ((mm >> k) & 1u) && !((cont >> (k + 1u)) & 1u);
                ev[2 * h] = (runI << 2) | 1u;
                ev[2 * h + 1] = (rc & 0x100u) ? ((1u << 16) | 3u) : (mcount << 2);  // D: a D run of 1, no move; M run
                ne |= (iev ? 1u : 0u) << (2 * h);
                ne |= (!ed && ((rc & 0x100u) || mend) ? 1u : 0u) << (2 * h + 1);
            }
            // exclusive prefix of the lane's event counts over the pair's 4 lanes
            const uint32_t cnt = (uint32_t)__builtin_popcount(ne);
            // (each cross-lane move outside the select: inside `?:` it became a branch that
            // masked its source lanes off, and a masked-off DPP source reads as the old value)
            uint32_t inc = cnt;
            const uint32_t s1 = quad<0x90>(inc);  // quad_perm [0, 0, 1, 2]
            inc += lw >= 1 ? s1 : 0u;
            const uint32_t s2 = quad<0x40>(inc);  // quad_perm [0, 0, 0, 1]
            inc += lw >= 2 ? s2 : 0u;
            const uint32_t tot = quad<0xFF>(inc);  // quad_perm [3, 3, 3, 3]
            uint32_t at = nev + inc - cnt;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                if ((ne >> e) & 1u) rout[at] = ev[e];
                at += (ne >> e) & 1u;
            }
            // the carried I run: the last record's when it ran to the edge
            const uint32_t last = nrec ? recs[nrec - 1] : 0u;
            if (mlive) {
                kI = nrec ? ((last & 0x200u) ? (last & 63u) + (nrec == 1 ? kI : 0u) : 0u) : kI;
                nev += tot;
            }
        }
        // the window's end: the walker's pair, then both pairs' cell in every lane
        int mi_ = hh ? ci[1] : ci[0], mj = hh ? cj[1] : cj[0];
        bool ml = mlive;
        if (mlive) {
            mi_ = 16 * mg + rr + 1;
            mj = mc0 + mW - (int)pos;
            if (kI >= 8192u) {  // (an I run's count field is 14 bits; runs of one op merge in the text)
                if (lw == 0) rout[nev] = (kI << 2) | 1u;
                ++nev;
                kI = 0;
            }
            ++windows;
            const bool done = zstop || mi_ < 1 || mj < 1;  // row 0 / column 0: H = 0
            if (!LOCAL && done) {
                // the boundary: INSERTs along row 0, DELETEs down column 0 (:81-92) -- after an
                // I run that reached column 0 in this window
                emit(true, kI);
                kI = 0;
                if (mi_ < 1) emit(true, (uint32_t)mj);
                else emit(false, (uint32_t)mi_);
            }
            mdone = done;
            ml = !done && room && windows <= mnm + 16u;
        }
        // (row_half_mirror: lane l <- lane 7 - l of its 8-lane group, the other pair's walker)
        auto other = [](int v) { return __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false); };
        const int oi = other(mi_), oj = other(mj), ol = other(ml ? 1 : 0);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const bool mine = h == hh;
            ci[h] = mine ? mi_ : oi;
            cj[h] = mine ? mj : oj;
            live[h] = mine ? ml : (ol != 0);
        }
        ck_wave_sync();
    }
    if (mhas && lw == 0) {
        // (a walk stopped by the event cap or the window bound before a cell with
        // H = 0 -- never a correct one, its events <= n + m -- would hand over a
        // truncated CIGAR: the plan's error word says so)
        if (!mdone || capped) atomicOr(a.err, kErrWalkCap);
        a.cigar_len[mp] = nev;  // the event count, for format_runs_kernel
    }
    ck_fallback_walks<MODE>(a, lane);
}

}  // namespace

hipError_t launch_walk_ck(int mode, const TraceArgs& a, hipStream_t s) {
    const dim3 g((a.count + kWavesPerBlock * kCkGroups * 2 - 1) / (kWavesPerBlock * kCkGroups * 2)), b(kBlock);
    switch (mode) {
        case kLocal: hipLaunchKernelGGL(traceback_ck_kernel<kLocal>, g, b, 0, s, a); break;
        case kGlobal: hipLaunchKernelGGL(traceback_ck_kernel<kGlobal>, g, b, 0, s, a); break;
        case kSemi: hipLaunchKernelGGL(traceback_ck_kernel<kSemi>, g, b, 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace ta
