// bioinfo1_amd/csrc/ta_device.h -- device helpers shared by the int32 kernels
// (ta_kernels.hip) and the packed dual-pair kernels (ta_dual.hip): wave
// primitives, target/boundary chunk loads, and the run-jumping traceback.
#pragma once

#include <climits>
#include <type_traits>

#include "ta_internal.h"

namespace ta {
namespace {


__device__ __forceinline__ int wadd(int a, int b) { return (int)((uint32_t)a + (uint32_t)b); }
__device__ __forceinline__ int wmul(uint32_t a, int b) { return (int)(a * (uint32_t)b); }

// DPP wave_shr:1 -- lane l gets v of lane l-1, lane 0 gets `lane0`.
// Must run with all 64 lanes enabled.
__device__ __forceinline__ int wave_shr1(int lane0, int v) {
    return __builtin_amdgcn_update_dpp(lane0, v, 0x138, 0xF, 0xF, false);
}

__device__ __forceinline__ int rdlane(int v, uint32_t l) { return __builtin_amdgcn_readlane(v, (int)l); }

// Global wave index.  readfirstlane tells the compiler it is wave-uniform
// (threadIdx.x >> 6 is not provably so), which keeps the pair's lengths, the
// loop counters and all per-pair control flow in SGPRs / scalar branches.
__device__ __forceinline__ uint32_t wave_id() {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)));
}

__device__ __forceinline__ uint64_t ballot(bool c) { return __builtin_amdgcn_ballot_w64(c); }

// acc*2 + (this lane's bit of `mask`) in one v_addc_co_u32 (the lane mask is
// the carry-in).  hipcc does not form this from C++ (it emits a cndmask +
// shift + or), so it is spelled out.
__device__ __forceinline__ uint32_t shl1_add_lanebit(uint32_t acc, uint64_t mask) {
    uint32_t r;
    uint64_t carry_out;
    asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=s"(carry_out) : "v"(acc), "s"(mask));
    return r;
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ int first_lane(bool c) {
    const unsigned long long b = __ballot(c);
    return b ? __ffsll((long long)b) - 1 : -1;
}

// 256 target characters per chunk, 4 per lane; out-of-range bytes are 0.
__device__ __forceinline__ uint32_t load_tchunk(const uint8_t* T, uint32_t m, uint32_t k, int lane) {
    const uint32_t base = k * 256u + 4u * (uint32_t)lane;
    uint32_t w = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const uint32_t idx = base + b;
        const uint32_t c = idx < m ? (uint32_t)T[idx] : 0u;
        w |= c << (8 * b);
    }
    return w;
}

// 64 boundary-row values per chunk: column 64k+lane+1.
__device__ __forceinline__ int load_bchunk(const int32_t* B, uint32_t m, uint32_t k, int lane) {
    const uint32_t j = k * 64u + (uint32_t)lane + 1u;
    return j <= m ? B[j] : 0;
}

// ---------------------------------------------------------------------------
// Traceback.  One wave per pair; the walk state (i, j) is wave-uniform and
// lives in SGPRs.  The wave keeps a tile of the pointer matrix in 4 VGPRs:
// wave-lane k holds the dwords of stripes L0..L0+3 at step tt0+k (64 steps x
// 64 rows).  Each iteration resolves a whole run of one op instead of one
// cell (SURVEY §7 "traceback latency"):
//   D (vertical)   -- the rows above in the same dword: the D plane shifted
//                     so that row r is bit 0, counted on the SALU (trailing ones);
//   I (horizontal) -- every wave-lane extracts row r of its step; the run is
//                     the streak of I codes in the ballot going down from
//                     the current step;
//   M (diagonal)   -- every wave-lane extracts the diagonal cell of its step
//                     (row r - (t - step)); same ballot streak.
// The iteration computes the D run and the one ballot unconditionally and
// picks with selects (no divergent control flow on the SALU).  Runs are
// clipped to the current stripe and tile; the next iteration picks the walk
// up from there.
//
// Runs are not formatted as they are found: RunWriter parks each finished
// run (op, count) in lane nb of two VGPRs, and every 64 runs the wave formats
// them at once -- each lane its own run's decimal digits, offsets from a
// wave prefix sum -- right to left into the slot (the walk goes backwards).
struct RunWriter {
    char* end;       // one past the slot's last byte; text grows towards the front
    uint32_t used;   // bytes written so far
    uint32_t op, cnt;  // the open run (op 0: nothing pushed yet)
    uint32_t nb;     // runs parked in rc / ro
    uint32_t rc, ro; // VGPRs: lane k = count / op char of parked run k
    int lane;
    __device__ __forceinline__ void flush_parked() {
        const bool act = (uint32_t)lane < nb;
        uint32_t c = rc;
        const uint32_t digits = 1u + (c >= 10u) + (c >= 100u) + (c >= 1000u) + (c >= 10000u) + (c >= 100000u) +
                                (c >= 1000000u) + (c >= 10000000u) + (c >= 100000000u) + (c >= 1000000000u);
        const uint32_t L = act ? digits + 1u : 0u;
        uint32_t incl = L;  // inclusive prefix sum over lanes
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = (uint32_t)__shfl_up((int)incl, o, 64);
            if (lane >= o) incl += v;
        }
        // run k's text ends where runs 0..k-1 (found earlier, written further right) begin
        char* p = end - used - (incl - L) - 1;
        if (act) *p = (char)ro;
#pragma unroll
        for (uint32_t d = 0; d < 10u; ++d) {  // fixed trip count: no divergent loop
            if (d < digits && act) p[-1 - (int)d] = (char)('0' + c % 10u);
            c /= 10u;
        }
        used += (uint32_t)rdlane((int)incl, 63);
        nb = 0;
    }
    __device__ __forceinline__ void park() {
        const bool here = (uint32_t)lane == nb;
        rc = here ? cnt : rc;
        ro = here ? op : ro;
        if (++nb == 64u) flush_parked();
    }
    // k >= 1 always (every caller moves the walk)
    __device__ __forceinline__ void push(uint32_t o, uint32_t k) {
        if (o == op) {
            cnt += k;
            return;
        }
        if (op) park();
        op = o;
        cnt = k;
    }
    __device__ __forceinline__ void finish() {
        if (!op) {  // RLE of an empty op string: "1" + '\0' (:145-160)
            used = 2;
            *(end - 2) = '1';
            *(end - 1) = '\0';
            return;
        }
        park();
        if (nb) flush_parked();
    }
};

// length of the streak of set bits in b going down from bit `from` (bit `from` is set)
__device__ __forceinline__ uint32_t streak_down(uint64_t b, uint32_t from) {
    return (uint32_t)__clzll((long long)~(b << (63u - from)));  // shifted-in zeros stop the streak
}

// What the local walk needs besides the codes: the reference's loop runs
// while the current cell's cost is > 0 (team_alignment.cpp:202).  The walk
// tracks that cost exactly -- a cell with cost > 0 is unclamped, so its
// parent's cost is its own minus the step's score (match_func / indel,
// :20-28) -- instead of reading a STOP code, so the packed local fill need
// not encode one.  Unused in global / semi-global walks.
struct WalkSeq {
    const uint8_t* Q;
    const uint8_t* T;
    int h;  // the goal cell's cost (the pair's score)
    int ma, mi, gap;
};

// Lane L: bytes S[base-1-L] (bits 7:0) and S[base-65-L] (bits 15:8), zero below S[0].
__device__ __forceinline__ uint32_t seq_window(const uint8_t* S, uint32_t base, int lane) {
    const uint32_t L = (uint32_t)lane;
    uint32_t v = 0;
    if (L < base) v = S[base - 1 - L];
    if (L + 64u < base) v |= (uint32_t)S[base - 65 - L] << 8;
    return v;
}

template <int MODE>
__device__ __forceinline__ void traceback_pair(const uint32_t* P, uint32_t n, uint32_t m, uint32_t gi, uint32_t gj,
                                               char* slot, uint64_t cap, int lane, uint64_t* start_in_slot,
                                               uint32_t* len, const WalkSeq& seq, bool blk = false) {
    RunWriter w{slot + cap, 0u, 0u, 0u, 0u, 0u, 0u, lane};
    int H = seq.h;  // local: cost of the walk's current cell
    uint32_t qbase = 0, tbase = 0, qw = 0, tw = 0;  // local: byte windows (seq_window)
    // local: gap runs need no bytes when their sequence has no '-' and gap <= 0
    bool gfastD = false, gfastI = false;
    const int posM = max(0, max(seq.ma, seq.mi));
    if (MODE == kLocal) {
        bool a = false, b = false;
        const uint32_t nm = max(n, m);
        for (uint32_t k0 = (uint32_t)lane; k0 < nm; k0 += 256) {  // 8 loads in flight per wait
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u) {
                const uint32_t k = k0 + 64u * u;
                a |= k < n && seq.Q[k] == '-';
                b |= k < m && seq.T[k] == '-';
            }
        }
        gfastD = ballot(a) == 0 && seq.gap <= 0;
        gfastI = ballot(b) == 0 && seq.gap <= 0;
        qbase = gi;  // the walk only moves up / left: windows end at the goal cell
        tbase = gj;
        qw = seq_window(seq.Q, gi, lane);
        tw = seq_window(seq.T, gj, lane);
    }
    if (MODE == kSemi && (gj != m || gi != n)) {  // :306-315
        if (gi == n) {
            if (m - gj) w.push('I', m - gj);
        } else if (gj == m && n - gi) {
            w.push('D', n - gi);
        }
    }
    const uint32_t Tmax = pass_steps(m);
    uint32_t i = gi, j = gj;
    // tile = steps [tt0, tt0+64) x stripes [tL0, tL0+4) of pass tP.  The walk
    // never moves to a larger step or stripe within a pass, so only the lower
    // bounds (and the pass) need checking.  `cur` is the tile column of
    // stripe cur_ln (re-selected only when the walk changes stripe).
    uint32_t tP = 0xFFFFFFFFu, tt0 = 0, tL0 = 0, cur_ln = 0xFFFFFFFFu;
    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, cur = 0;
    while (true) {
        if (MODE == kLocal) {
            if (H <= 0 || min(i, j) == 0) break;  // cost 0 ends the walk (:202); row/col 0 cost 0
        } else {
            if (i == 0) {  // row 0: INSERT parents (:89-92)
                if (j) w.push('I', j);
                break;
            }
            if (j == 0) {  // column 0: DELETE parents (:83-86)
                w.push('D', i);
                break;
            }
        }
        const uint32_t row = i - 1;
        const uint32_t ln = (row >> 4) & 63u, r = row & 15u;
        const uint32_t t = (j - 1) + ln;
        if ((int)((t - tt0) | (ln - tL0)) < 0 || (row >> 10) != tP) {
            // (readfirstlane: keeps the tile origin in SGPRs; hipcc computes
            // the clamped subtractions on the VALU)
            tP = row >> 10;  // kPassRows = 1024
            tL0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(max(ln, 3u) - 3u));
            tt0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(max(t, 63u) - 63u));
            const uint32_t ts = tt0 + (uint32_t)lane;
            c0 = c1 = c2 = c3 = 0;
            if (ts < Tmax && blk) {  // blocked layout: 4 stripes of one step, 64 bytes apart
                const uint32_t* q = P + blk_index(tP, ts, tL0, blk_count(m));
                c0 = q[0];
                c1 = q[kBlkSteps];
                c2 = q[2 * kBlkSteps];
                c3 = q[3 * kBlkSteps];
            } else if (ts < Tmax) {
                const uint32_t* q = P + ((uint64_t)tP * Tmax + ts) * kWave + tL0;
                c0 = q[0];
                c1 = q[1];
                c2 = q[2];
                c3 = q[3];
            }
            cur_ln = 0xFFFFFFFFu;
        }
        if (ln != cur_ln) {
            const uint32_t sel = ln - tL0;
            cur = sel == 0 ? c0 : sel == 1 ? c1 : sel == 2 ? c2 : c3;
            cur_ln = ln;
        }
        const uint32_t kk = t - tt0;
        // bit planes (ta_internal.h Code): row r's D bit at 31 - r, I bit at
        // 15 - r.  x = dw >> (15 - r): bit 16 + k / bit k = D / I of row r - k.
        const uint32_t sh = 15u - r;
        const uint32_t x = (uint32_t)rdlane((int)cur, kk) >> sh;
        // Branch-free: the D run (SALU) and the one ballot (I: row r at every
        // step; M: step tt0+lane holds row r - (kk - lane), i.e. shift
        // sh + (kk - lane)) are both computed and picked with selects; hipcc
        // turns uniform if/else chains here into costly flag-register flow.
        // D wins over I (the packed local fill stores raw compares; the int32
        // fill's STOP code (D and I) only marks cost-0 cells, never reached here)
        const uint32_t dflag = (x >> 16) & 1u, iflag = x & 1u;
        // D cells of rows r, r-1, ..: trailing ones
        const uint32_t dp = x >> 16;
        const uint32_t drun = (uint32_t)__builtin_ctz(~dp);  // <= r + 1
        const uint32_t lsh = sh + (kk - (uint32_t)lane) * (iflag ^ 1u);
        const uint32_t v = (cur >> (lsh & 31u)) & 0x10001u;
        const uint32_t streak = streak_down(ballot(v == iflag), kk);
        const uint32_t hrun = min(streak, iflag ? j : min(j, r + 1u));
        const uint32_t run = dflag ? drun : hrun;
        const uint32_t op = dflag ? 'D' : ('M' - 4u * iflag);
        if (MODE == kLocal) {
            // cost along the run: move k leaves cell c_k (lane k: row i-1-k / column j-1-k
            // bytes); the walk stops at the first c_k (k >= 1) whose cost is 0.  A run can
            // reach 0 only if H <= run * (largest positive step score); otherwise the cost
            // just moves by the run's total.
            uint32_t emit = run;
            bool stop = false;
            const bool gfast = op != 'M' && (op == 'D' ? gfastD : gfastI);
            // the bytes of the run's cells (lane k: q[i-1-k], t[j-1-k]) from 128-byte
            // windows refilled only after 64 rows / columns of progress, one ds_bpermute each
            uint32_t qb = 0, tb = 0;
            if (!gfast) {
                if (qbase - i > 64u) {
                    qbase = i;
                    qw = seq_window(seq.Q, i, lane);
                }
                if (tbase - j > 64u) {
                    tbase = j;
                    tw = seq_window(seq.T, j, lane);
                }
                const uint32_t oq = qbase - i + (uint32_t)lane, ot = tbase - j + (uint32_t)lane;  // < 128
                const uint32_t qv = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((oq & 63u) << 2), (int)qw);
                const uint32_t tv = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((ot & 63u) << 2), (int)tw);
                qb = (qv >> ((oq >> 6) << 3)) & 0xFFu;
                tb = (tv >> ((ot >> 6) << 3)) & 0xFFu;
            }
            const uint64_t inrun = run >= 64u ? ~0ull : ((1ull << run) - 1ull);
            if (gfast) {
                H -= (int)run * seq.gap;  // uniform gap steps (gap <= 0) never lower the cost
            } else if (op == 'M' && H > (int)run * posM) {
                const int c = __builtin_popcountll(ballot(qb == tb) & inrun);  // matches
                H -= c * seq.ma + ((int)run - c) * seq.mi;
            } else {
                const bool in = (uint32_t)lane < run;
                int d;
                if (op == 'M') d = (qb == tb) ? seq.ma : seq.mi;
                else d = (((op == 'D') ? qb : tb) == '-') ? 0 : seq.gap;
                int incl = in ? d : 0;  // inclusive prefix over the run's cells
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int v = __shfl_up(incl, o, 64);
                    if (lane >= o) incl += v;
                }
                const uint64_t z = ballot(in && H - incl <= 0);
                if (z) {
                    emit = (uint32_t)__builtin_ctzll(z) + 1u;
                    stop = true;
                } else {
                    H -= rdlane(incl, run - 1u);
                }
            }
            w.push(op, emit);
            i -= (op == 'I') ? 0u : emit;
            j -= dflag ? 0u : emit;
            if (stop) break;
            continue;
        }
        w.push(op, run);
        i -= (op == 'I') ? 0u : run;
        j -= dflag ? 0u : run;
    }
    w.finish();
    *start_in_slot = cap - w.used;
    *len = w.used;
}

// Select v[idx] for a wave-uniform runtime idx without dynamic register
// indexing (which the compiler would lower through LDS or scratch).
template <int R>
__device__ __forceinline__ int select_row(const int (&v)[R], uint32_t idx) {
    int x = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) x |= v[k] & -(int)(idx == (uint32_t)k);
    return x;
}

// Compile-time loop: f(std::integral_constant<int, I>) for I in [B, E).
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

template <int C>
__device__ __forceinline__ int max3_imm(int a, int b) {
    // max(a, b, C) with C an inline constant.  Kept opaque so that hipcc does
    // not split it back into two v_max when a later compare reads the result
    // (it rewrites h == C into max(a,b) <= C).
    int r;
    asm("v_max3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "i"(C));
    return r;
}

// What one pass reports to the running goal.
struct PassOut {
    int h;           // local: best score of the pass; semi: best of column m
    uint32_t i, j;   // its cell (1-based rows), i == 0 when no candidate
    int row_h;       // semi, last pass: best of row n
    uint32_t row_j;
    int corner;      // global, last pass: H[n][m]
};

}  // namespace
}  // namespace ta
