// bioinfo1_amd/csrc/ta_planner.cpp -- host planning of linear-gap and affine
// batches (ta_planner.h).  No HIP: the device drivers (ta_api.hip,
// ta_affine.hip) upload what this computes.
#include "ta_planner.h"

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <functional>
#include <numeric>

namespace ta {

// The flexible fill keeps V = S - O within a wave's span: 1,024 rows + 2 x 64
// columns of cells whose neighbours differ by at most |score| + |gap| <= 2*mag
// (plus the 64-step drift between rebases).  Global / semi keep S = H - ma*j +
// gap*(j - i): a vertical step of S lies in [0, hs - 2*gap] (H moves by
// [gap, hs - gap] down a column) and a horizontal one within 4*mag, so the span
// is at most (3*1024 + 8*64 + 8)*mag -- inside the same bound for mag <= 6.
// Local mode also ranks a column's 16 rows by 16 * (V_r - V_0) + 15 - r,
// within 16 * 15 * 2 * mag.
bool flex_fits(int mode, int ma, int mi, int gap) {
    (void)mode;
    const long long mag = std::max({1LL, std::llabs(ma), std::llabs(mi), std::llabs(gap)});
    return (kPassRows + 3LL * kWave) * 2 * mag * 2 <= 30000;
}

// Local mode: the values a wave holds lie in [0, 0x7BFF] (ta_flex.hip: the
// three-input max on f16 bit patterns) -- the frame of ta_layout.h
// flex_local_c0: above the lane-uniform clamp base zu (kept within 64 steps of
// drift of c0) by at most 15 rows of |gap| plus H <= hmax, candidates one step
// (mag) below or above.
bool flex_local_fits(uint32_t n, uint32_t m, int ma, int mi, int gap) {
    const long long mag = std::max({1LL, std::llabs(ma), std::llabs(mi), std::llabs(gap)});
    const long long hmax = (long long)std::min(n, m) * std::max({0LL, (long long)ma, (long long)mi}) +
                           ((long long)n + m) * std::max(0LL, (long long)gap);
    const long long c0 = flex_local_c0(ma, mi, gap);
    const long long hi = c0 + 64LL * std::max(0, gap - ma) + 15LL * std::max(0, -gap) + hmax + 16 * mag;
    return mag <= 64 && hi <= 0x7BFF && hmax + 3LL * kWave * std::llabs(ma) + 8 * mag <= 30000;
}

// Checkpoints of the flexible fill hold H itself as int16 (ta_flex.hip CK), and the
// recomputing walk keeps a window of a global / semi pair as S minus its corner's bias
// part, H plus at most (|gap| + |gap - ma|) x 48 (ta_walk_ck.hip): H must lie within
// +-30,000 for rows to n + 15 (semi H >= gap min(i, j), global (i + j) min(0, gap);
// H <= hs min(i, j) + (i + j) max(0, gap)); local values also meet flex_local_fits.
bool flex_ck_fits(int mode, uint32_t n, uint32_t m, int ma, int mi, int gap) {
    const long long N = (long long)n + 16, M = m, g = gap, K = std::min(N, M);
    const long long mag = std::max({1LL, std::llabs(ma), std::llabs(mi), std::llabs(gap)});
    const long long hi = K * std::max({0LL, (long long)ma, (long long)mi}) + (N + M) * std::max(0LL, g);
    const long long lo = mode == kLocal ? 0 : mode == kSemi ? K * std::min(0LL, g) : (N + M) * std::min(0LL, g);
    return lo - 100 * mag >= -30000 && hi + 100 * mag <= 30000 &&
           (mode != kLocal || flex_local_fits(n, m, ma, mi, gap));
}

// Bounds of the biased 16-bit values of ta_dual.hip (S and every candidate),
// with a margin; pairs that do not fit run in the int32 kernel.
bool fits_int16(int mode, uint32_t n, uint32_t m, int ma, int mi, int gap) {
    if (n == 0 || m == 0) return false;
    const long long N = n, M = m;
    const long long mag = std::max({1LL, std::llabs(ma), std::llabs(mi), std::llabs(gap)});
    const long long hmax = std::min(N, M) * std::max({0LL, (long long)ma, (long long)mi}) + (N + M) * std::max(0LL, (long long)gap);
    long long lo, hi;
    if (mode == kLocal) {
        const long long z = 1 - 16LL * ma;  // S = 16H + z*j - i
        hi = 16 * hmax + std::max(0LL, z) * M + 32 * mag;
        lo = std::min(0LL, z) * M - N - 32 * mag;
        if (16 * hmax + 15 > 32767) return false;  // the argmax key 16H + 15 - r
    } else {
        // S = H - ma*j + gap*(j - i) over the rows 0..n+15 (the last lane's padding
        // rows) and columns 0..m.  H >= gap*min(i, j) (semi: gap steps from a 0
        // boundary) or (i + j)*min(0, gap) (global), H <= hs*min(i, j) + (i + j)*gp.
        // Both bounds and the bias are linear on either side of i = j, so their
        // extremes lie on the vertices of the two triangles; the row-n values
        // H - gap*n that the semi-global kernel also keeps packed are covered too.
        const long long N1 = N + 16, g = gap, K = std::min(N1, M);
        const long long hs = std::max({0LL, (long long)ma, (long long)mi}), gp = std::max(0LL, g);
        const long long pts[5][2] = {{0, 0}, {N1, 0}, {0, M}, {N1, M}, {K, K}};
        lo = LLONG_MAX;
        hi = LLONG_MIN;
        for (const auto& pt : pts) {
            const long long i = pt[0], j = pt[1], mn = std::min(i, j);
            const long long hl = (mode == kGlobal) ? (i + j) * std::min(0LL, g) : std::min(0LL, g) * mn;
            const long long hh = hs * mn + (i + j) * gp;
            const long long b = -(long long)ma * j + g * (j - i);
            lo = std::min({lo, hl + b, hl - g * N1, hl - g * N});
            hi = std::max({hi, hh + b, hh - g * N1, hh - g * N});
        }
        lo -= 8 * mag;
        hi += 8 * mag;
    }
    return hi <= 32000 && lo >= -32000;
}

// Every packed value of aff_dual_pass within int16, with margins.  The kernel
// keeps S = V - ma*j + X*(j - i) for V = H, E, F.  Per cell (i, j), rows up to
// n + 15 (the last lane's padding rows):
//   H >= min(0, O + X*min(i, j))            semi (a gap run from a 0 boundary;
//        (O + X*max(i, j) when X > 0)         0 on the boundary itself)
//   H >= 2*min(0, O) + (i + j)*min(0, X)    global (down the column, then right)
//   H <= hs*min(i, j) + (i + j)*(max(0, O) + max(0, X))
// E and F lie within one gap step (|O| + |X|) of an H, the -inf stand-ins are
// H - K, candidates one more step.  The lower bounds are concave and the upper
// one linear on either side of i = j, so their extremes over the grid lie on
// the vertices of the two triangles; the semi row-n values H - X*n are
// covered too.
bool affine_fits_int16(int mode, uint32_t n, uint32_t m, int ma, int mi, int open, int ext) {
    if (mode == kLocal || n == 0 || m == 0) return false;
    const long long N = n, N1 = N + 16, M = m, O = open, X = ext;
    const long long hs = std::max({0LL, (long long)ma, (long long)mi});
    const long long gp = std::max(0LL, O) + std::max(0LL, X);
    const long long k = std::llabs(O) + std::llabs(X) + 2;
    const long long marg = 2 * k + 2 * std::llabs(ma) + std::llabs(mi) + 8;
    const long long K = std::min(N1, M);
    const long long pts[5][2] = {{0, 0}, {N1, 0}, {0, M}, {N1, M}, {K, K}};
    long long lo = LLONG_MAX, hi = LLONG_MIN;
    for (const auto& pt : pts) {
        const long long i = pt[0], j = pt[1], mn = std::min(i, j), mx = std::max(i, j);
        const long long hl = (mode == kGlobal) ? 2 * std::min(0LL, O) + (i + j) * std::min(0LL, X)
                                               : std::min(0LL, O + X * (X <= 0 ? mn : mx));
        const long long hh = hs * mn + (i + j) * gp;
        const long long b = -(long long)ma * j + X * (j - i);
        lo = std::min({lo, hl + b, hl - X * N});
        hi = std::max({hi, hh + b, hh - X * N});
    }
    return lo - marg >= -32000 && hi + marg <= 32000;
}

namespace {

// Pairs by descending cells (fewer stragglers: the big ones start first),
// equal shapes adjacent so they can be coupled for the two-pair kernels.
std::vector<uint32_t> by_cells(uint32_t n_pairs, const uint32_t* qlen, const uint32_t* tlen) {
    std::vector<uint32_t> o(n_pairs);
    std::iota(o.begin(), o.end(), 0u);
    bool uniform = true;
    for (uint32_t p = 1; p < n_pairs && uniform; ++p) uniform = qlen[p] == qlen[0] && tlen[p] == tlen[0];
    if (uniform) return o;  // already in order (stable)
    std::stable_sort(o.begin(), o.end(), [&](uint32_t a, uint32_t b) {
        const uint64_t ca = (uint64_t)qlen[a] * tlen[a], cb = (uint64_t)qlen[b] * tlen[b];
        if (ca != cb) return ca > cb;
        return qlen[a] != qlen[b] ? qlen[a] > qlen[b] : tlen[a] > tlen[b];
    });
    return o;
}

std::vector<uint64_t> slot_offsets(uint32_t n_pairs, const uint32_t* qlen, const uint32_t* tlen, uint64_t* total) {
    std::vector<uint64_t> off(n_pairs);
    uint64_t so = 0;
    for (uint32_t p = 0; p < n_pairs; ++p) {
        off[p] = so;
        so += cigar_slot_bytes(qlen[p], tlen[p]);
    }
    *total = so;
    return off;
}

// Chunk boundaries over units in launch order: a chunk closes when the next
// unit's codes would exceed the budget.  A chunk closed by the budget is then
// trimmed to a whole number of "rounds" -- multiples of wave_quantum waves (one
// wave per SIMD) -- when it holds at least one: the fill is VALU-bound, so a
// chunk takes as long as its busiest SIMD, and 2,500 waves on 1,024 SIMDs
// (3 on some, 2 on others) run at 2.44 / 3 of the rate of 2,048 (config 5
// affine: 100k pairs in 20 chunks of 5,000 vs 25 of 4,096).
std::vector<size_t> chunk_starts(size_t n_units, uint64_t budget, uint32_t wave_quantum,
                                 const std::function<uint64_t(size_t)>& codes,
                                 const std::function<uint64_t(size_t)>& waves) {
    std::vector<size_t> starts;
    size_t k = 0;
    while (k < n_units) {
        const size_t start = k;
        uint64_t used = 0, w = 0;
        while (k < n_units) {
            const uint64_t c = codes(k);
            if (k > start && used + c > budget) break;
            used += c;
            w += waves(k);
            ++k;
        }
        if (k < n_units && wave_quantum && w >= wave_quantum) {
            const uint64_t target = w / wave_quantum * wave_quantum;
            while (w > target && k > start + 1) {
                --k;
                w -= waves(k);
            }
        }
        starts.push_back(start);
    }
    return starts;
}

// Ticket order of one chunk's pass tasks (units first .. first+count-1, unit
// w with off[w+1] - off[w] passes).  A task's predecessor (the same unit's
// pass - 1) must hold an earlier ticket: its wave is then running, so every
// poll ends.  Pass-major (start-aligned): every unit's pass 0, then every
// pass 1, ...; the longest units' last passes get the last tickets and run
// alone at the end of the launch.  End-aligned (default): level L = pass -
// passes, ascending, so every unit's last pass is in the last level and the
// long chains start first.  Within a level: plan order (most cells first).
template <class Emit>
void order_pass_tasks(const std::vector<uint32_t>& off, uint32_t first, uint32_t count, bool end_aligned, Emit emit) {
    uint32_t maxp = 0;
    for (uint32_t w = first; w < first + count; ++w) maxp = std::max(maxp, off[w + 1] - off[w]);
    for (uint32_t lv = 0; lv < maxp; ++lv)
        for (uint32_t w = first; w < first + count; ++w) {
            const uint32_t P = off[w + 1] - off[w];
            if (end_aligned) {
                if (lv + P >= maxp) emit(w, lv + P - maxp);
            } else if (lv < P) {
                emit(w, lv);
            }
        }
}

}  // namespace

void build_plan(Plan& pl, uint32_t n_pairs, const uint32_t* qlen, const uint32_t* tlen, int type, int match,
                int mismatch, int gap, bool want_cigar, uint64_t budget, uint32_t flags, uint32_t wave_quantum) {
    pl = Plan{};
    pl.n_pairs = n_pairs;
    pl.type = type;
    pl.match = match;
    pl.mismatch = mismatch;
    pl.gap = gap;
    pl.want_cigar = want_cigar;
    pl.qlen.assign(qlen, qlen + n_pairs);
    pl.tlen.assign(tlen, tlen + n_pairs);
    // Local mode keeps V = 32*score + row tag in int32; take the unscaled
    // ("wide") kernel when any local value could reach 2^25 in magnitude.
    uint64_t maxlen = 0;
    for (uint32_t p = 0; p < n_pairs; ++p) maxlen = std::max<uint64_t>(maxlen, (uint64_t)qlen[p] + tlen[p]);
    const uint64_t mag = std::max<uint64_t>({1ull, (uint64_t)std::llabs(match), (uint64_t)std::llabs(mismatch),
                                             (uint64_t)std::llabs(gap)});
    pl.wide = (type == kLocal) && (maxlen * mag >= (1ull << 25));
    const bool dual = !(flags & kPlanInt32Only);
    const std::vector<uint32_t> order = by_cells(n_pairs, qlen, tlen);
    pl.slot_off = slot_offsets(n_pairs, qlen, tlen, &pl.slots_bytes);
    const uint64_t budget_dw = std::max<uint64_t>(budget / 4, 1);
    pl.ptr_off.assign(n_pairs, 0);
    pl.bnd_off.assign(n_pairs, 0);
    // Work units: one pair (int32 fill), an equal-shape couple (dual fill) or
    // a couple of different shapes (flexible dual fill), then longest first.
    struct Unit {
        int kind;  // 0 single, 1 dual, 2 flex
        uint32_t a, b;
        uint64_t cost;  // cells one wave sweeps
    };
    std::vector<Unit> units;
    units.reserve(n_pairs);
    // Checkpoints save the fill ~0.3 of its time but the recomputing walk is a
    // longer chain per pair than the band walk (one window per 16 rows): they pay
    // once the cells per unit of the longest path pass ~2.5e6 (1 kb pairs: from
    // ~5,000 pairs on; 8 to 4,096 measured slower, profiles/bench/r05_ck_batches.txt).
    uint64_t cells = 0, longest = 1;
    for (uint32_t p = 0; p < n_pairs; ++p) {
        cells += (uint64_t)qlen[p] * tlen[p];
        longest = std::max<uint64_t>(longest, (uint64_t)qlen[p] + tlen[p]);
    }
    const bool ck_size = (flags & kPlanCk) || cells >= 2500000ull * longest;
    // a plan that may take checkpoints couples its leftover ragged pairs with themselves in
    // the flexible fill (not the int32 fill, which only stores codes)
    const bool ck_want = want_cigar && ck_size && mag < (1ull << 22) && (type != kLocal || gap <= 0) &&
                         !(flags & (kPlanNoCk | kPlanNoBlk | kPlanWalk1 | kPlanWalk2));
    std::vector<uint32_t> rest;
    const bool flex_ok = dual && !(flags & kPlanNoFlex) && flex_fits(type, match, mismatch, gap);
    // A pair left without a partner (an odd pair of equal shapes, a ragged pair no
    // neighbour couples with) runs coupled with itself in the dual kernel, like a
    // lone pair, rather than in the int32 fill: a drop-in batch of 3 x 1 kb went
    // 1.12 -> 0.78 ms with the packed fill and walk for all of its pairs
    // (profiles/bench/r05_batch_latency.txt).
    // (tiny pairs keep the int32 fill: alone, its one fused launch is the shortest --
    // unless checkpoints are forced, kPlanCk: the tests' way into the checkpoint walks)
    auto lone_dual = [&](uint32_t p) {
        return dual && ((uint64_t)qlen[p] * tlen[p] >= 4096 || (flags & kPlanCk)) && n_passes(qlen[p]) < 64 &&
               fits_int16(type, qlen[p], tlen[p], match, mismatch, gap);
    };
    for (uint32_t k = 0; k < n_pairs;) {
        const uint32_t p = order[k];
        const uint32_t n = qlen[p], m = tlen[p];
        // (equal shapes within int16 stay on the dual fill even when multi-pass: measured faster
        // than the pipelined flexible fill on config 5, 4,056 vs 3,765 GCUPS)
        // (< 64 passes: the hand-off tags epoch * 64 + pass + 1 never wrap to 0, ta_dual.hip)
        const bool couple = dual && k + 1 < n_pairs && qlen[order[k + 1]] == n && tlen[order[k + 1]] == m &&
                            n_passes(n) < 64 && fits_int16(type, n, m, match, mismatch, gap);
        // A lone pair (one-pair batches: the drop-in call) runs coupled with
        // itself in the packed kernel -- both halves compute it, its codes are
        // written once -- whose wave and lane walk finish sooner than one int32
        // wave walking inside the fill, except for tiny pairs where the one
        // fused launch wins.
        const bool self = dual && n_pairs == 1 && (uint64_t)n * m >= 4096 && n_passes(n) < 64 &&
                          fits_int16(type, n, m, match, mismatch, gap);
        if (couple) {
            units.push_back({1, p, order[k + 1], (uint64_t)n * m});
            k += 2;
        } else if (self) {
            units.push_back({1, p, p, (uint64_t)n * m});
            ++k;
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
            if (qlen[p] && tlen[p] && (type != kLocal || flex_local_fits(qlen[p], tlen[p], match, mismatch, gap)) &&
                (!ck_want || flex_ck_fits(type, qlen[p], tlen[p], match, mismatch, gap)))
                cand.push_back(p);
            else
                units.push_back({0, p, p, (uint64_t)qlen[p] * tlen[p]});
        }
        auto key = [&](uint32_t p) { return ((uint64_t)n_passes(qlen[p]) << 4) | (qlen[p] & 15u); };
        std::stable_sort(cand.begin(), cand.end(), [&](uint32_t a, uint32_t b) {
            if (key(a) != key(b)) return key(a) < key(b);
            if (qlen[a] != qlen[b]) return qlen[a] > qlen[b];
            return tlen[a] > tlen[b];
        });
        for (size_t i = 0; i < cand.size();) {
            const uint32_t A = cand[i];
            if (i + 1 < cand.size() && key(cand[i + 1]) == key(A) && n_passes(qlen[A]) < 64) {
                const uint32_t B = cand[i + 1];
                const uint64_t M = std::max(tlen[A], tlen[B]);
                const uint64_t wave = (uint64_t)qlen[A] * M;
                const uint64_t useful = (uint64_t)qlen[A] * tlen[A] + (uint64_t)qlen[B] * tlen[B];
                if (4 * useful >= 3 * 2 * wave) {  // waste <= 25 %
                    units.push_back({2, A, B, wave});
                    i += 2;
                    continue;
                }
            }
            // a long pair without a partner is coupled with itself: one wave per pass;
            // a shorter one in the dual kernel when it fits int16 (lone_dual)
            const uint32_t ps = n_passes(qlen[A]);
            if ((ps >= 4 || (ck_want && !lone_dual(A))) && ps < 64)
                units.push_back({2, A, A, (uint64_t)qlen[A] * tlen[A]});
            else
                units.push_back({lone_dual(A) ? 1 : 0, A, A, (uint64_t)qlen[A] * tlen[A]});
            ++i;
        }
    } else {
        for (uint32_t p : rest) units.push_back({lone_dual(p) ? 1 : 0, p, p, (uint64_t)qlen[p] * tlen[p]});
    }
    std::stable_sort(units.begin(), units.end(), [](const Unit& x, const Unit& y) { return x.cost > y.cost; });
    // Local walks of short pairs in plans of equal-shape couples only run as band
    // walks (one lane per pair, ta_walk_band.h) over the blocked code layout:
    // the dual fill stages each stripe's 16 steps and writes them as 64
    // contiguous bytes, the unit a walk following its stripe reads.
    uint64_t len_sum = 0;
    for (uint32_t p = 0; p < n_pairs; ++p) len_sum += (uint64_t)qlen[p] + tlen[p];
    const bool short_pairs = len_sum <= 6000ull * std::max<uint32_t>(n_pairs, 1);
    // Local plans take the blocked layout only with checkpoints (ck_size, gap <= 0) or
    // under TA_PLAN_NO_CK (blocked codes and band walks): below the checkpoint size the
    // [step][lane] codes (whose fill reads its per-step operands from the LDS list) and
    // the lane walks finish sooner at every batch size measured, 8-4096 pairs of
    // 200-1000 bases (3-6 %, scripts/exp/batch_latency.py, profiles/bench/r06s_batch_latency.txt).
    // (Batches of fewer than 8 pairs keep the lane walks with any flag.)
    bool all_dual = !units.empty(), all_packed = !units.empty(), any_flex = false;
    for (const Unit& u : units) {
        all_dual = all_dual && u.kind == 1;
        all_packed = all_packed && u.kind >= 1;
        any_flex = any_flex || u.kind == 2;
    }
    // Global / semi-global plans of equal-shape couples (config 5) take checkpoints
    // and recomputing walks by the same rule, whatever their lengths: their walks end
    // on row 0 / column 0 (ta_walk_ck.hip) and need no cost, so no gap-sign condition.
    const bool edge_ck = want_cigar && type != kLocal && all_dual && mag < (1ull << 22) && ck_size &&
                         !(flags & (kPlanNoCk | kPlanNoBlk | kPlanWalk1 | kPlanWalk2));
    // Plans with flexible couples (config 3: ragged reads) in any mode, when every unit
    // is packed and every flexible pair's H fits the checkpoints (flex_ck_fits; local
    // walks need gap <= 0, ck_want)
    bool flex_fit = true;
    for (const Unit& u : units)
        if (u.kind == 2)
            flex_fit = flex_fit && flex_ck_fits(type, qlen[u.a], tlen[u.a], match, mismatch, gap) &&
                       flex_ck_fits(type, qlen[u.b], tlen[u.b], match, mismatch, gap);
    const bool flex_ck = ck_want && any_flex && all_packed && flex_fit && !(flags & kPlanNoFlexCk);
    pl.blk = (want_cigar && type == kLocal && all_dual && short_pairs && n_pairs >= 8 && mag < (1ull << 22) &&
              ((flags & kPlanNoCk) || (ck_size && gap <= 0)) && !(flags & (kPlanNoBlk | kPlanWalk1 | kPlanWalk2))) ||
             edge_ck || flex_ck;
    // Multi-pass int32 pairs run one wave per (pair, pass) like the packed
    // fills (their passes overlap instead of following each other on one
    // wave); the walk then runs in the traceback kernel.
    const bool pipe_singles = !(flags & kPlanSerialPasses);
    auto unit_codes = [&](size_t k) -> uint64_t {
        const Unit& u = units[k];
        if (!want_cigar) return 0;
        return ptr_dwords_any(qlen[u.a], tlen[u.a], pl.blk) +
               (u.kind && u.a != u.b ? ptr_dwords_any(qlen[u.b], tlen[u.b], pl.blk) : 0);
    };
    auto unit_waves = [&](size_t k) -> uint64_t {
        const Unit& u = units[k];
        // packed fills and pipelined int32 pairs: one wave per (pair or couple, pass)
        return (u.kind || pipe_singles) && qlen[u.a] && tlen[u.a] ? n_passes(qlen[u.a]) : 1;
    };
    const std::vector<size_t> starts = chunk_starts(units.size(), budget_dw, wave_quantum, unit_codes, unit_waves);
    size_t next_cut = 1;
    pl.order.reserve(n_pairs);
    Plan::Chunk cur{};
    uint32_t couples_before = 0;
    auto open_chunk = [&]() {
        cur = Plan::Chunk{(uint32_t)pl.order.size(), 0, (uint32_t)pl.singles.size(), 0,
                          (uint32_t)(pl.duals.size() / 2), 0, (uint32_t)(pl.flexes.size() / 2), 0,
                          couples_before, 0, 0, 0, 0};
    };
    open_chunk();
    for (size_t k = 0; k < units.size(); ++k) {
        const Unit& u = units[k];
        const uint32_t na = qlen[u.a], ma = tlen[u.a], mb = tlen[u.b];
        const bool two = u.kind && u.a != u.b;
        if (next_cut < starts.size() && k == starts[next_cut]) {
            pl.chunks.push_back(cur);
            open_chunk();
            ++next_cut;
        }
        const uint32_t q[2] = {u.a, u.b};
        for (int h = 0; h < (two ? 2 : 1); ++h) {
            const uint32_t x = q[h];
            pl.ptr_off[x] = cur.ptr_dwords;
            pl.bnd_off[x] = cur.bnd_words;
            const uint64_t xd = want_cigar ? ptr_dwords_any(qlen[x], tlen[x], pl.blk) : 0;
            // flex: pair A holds both pairs' absolute int32 boundary rows, interleaved;
            // each pair keeps a region of its own for the int32 fallback ('-' in a query)
            uint64_t bw = bnd_words(qlen[x], tlen[x]);
            if (u.kind == 2 && h == 0 && n_passes(na) > 1)
                bw = std::max<uint64_t>(bw, 8ull * ((uint64_t)std::max(ma, mb) + 1));
            // dual: pair A holds the couple's packed hand-off records, 2 buffers x 8 bytes per column
            if (u.kind == 1 && h == 0 && n_passes(na) > 1) bw = std::max<uint64_t>(bw, 4ull * ((uint64_t)ma + 1));
            // pipelined int32 fill: the pair's hand-off records, 2 buffers x 8 bytes per column
            if (u.kind == 0 && pipe_singles && n_passes(na) > 1) bw = std::max<uint64_t>(bw, 4ull * ((uint64_t)ma + 1));
            bw += bw & 1;  // keep every region 8-byte aligned (64-bit hand-off records)
            cur.ptr_dwords += xd;
            cur.bnd_words += bw;
            pl.order.push_back(x);
        }
        if (u.kind == 1) {
            pl.duals.push_back(u.a);
            pl.duals.push_back(u.b);
            ++cur.dcount;
            cur.dpasses = std::max(cur.dpasses, n_passes(na));
        } else if (u.kind == 2) {
            pl.flexes.push_back(u.a);
            pl.flexes.push_back(u.b);
            ++cur.fcount;
        } else {
            pl.singles.push_back(u.a);
            ++cur.scount;
            if (pipe_singles && na && ma) cur.spasses = std::max(cur.spasses, n_passes(na));
        }
        if (u.kind) {
            pl.n_dual_pairs += 2;
            ++couples_before;
        }
        cur.count += two ? 2 : 1;
    }
    if (cur.count) pl.chunks.push_back(cur);
    // A fill kernel that walks its own pair only pays when nothing else of the
    // chunk runs in the separate traceback kernel anyway.
    bool piped = false;
    for (const auto& c : pl.chunks) piped |= c.spasses > 1;
    pl.fused = want_cigar && pl.n_dual_pairs == 0 && !(flags & kPlanUnfused) && !piped;
    // Local walks of short pairs: lane walks (one lane per pair steps cell by cell
    // through LDS tiles, ta_walk_lane.h; indel costs kept as int8).  Two pairs per
    // wave (32 lanes each, ta_walk2.h): 0.65 vs 0.77 ms for one pair per wave on
    // config 2; their runs are clipped to 32 cells, so batches of long pairs (long
    // M runs) keep the one-pair walk (config 3 local: 4.1 vs 6.3 ms).  24-bit
    // multiplies of the scores in the run walks.
    // (local: a positive gap lowers the cost in gap runs -- the one-pair walk)
    if (pl.blk) pl.walk_group = (gap <= 0 || type != kLocal) ? 64 : 0;
    else if ((flags & kPlanWalk1) || mag >= (1ull << 22) || !short_pairs) pl.walk_group = 0;
    else if ((flags & kPlanWalk2) || gap < -128 || gap > 127) pl.walk_group = 32;
    else pl.walk_group = 16;
    pl.ck = pl.blk && pl.walk_group == 64 && !(flags & kPlanNoCk) && ck_size;
    // (Each dual wave walking its own two pairs right after its fill measured
    // slower: config 2 3.10 ms vs 2.19 + 0.65; the walk inherits the fill's
    // register allocation and all waves finish their fills together anyway.)
    pl.flex_task_off.assign(1, 0);
    for (size_t w = 0; w < pl.flexes.size() / 2; ++w)
        pl.flex_task_off.push_back(pl.flex_task_off.back() + n_passes(qlen[pl.flexes[2 * w]]));
    pl.flex_tasks.assign(pl.flex_task_off.back(), 0u);
    const bool end_aligned = !(flags & kPlanPassMajor);
    pl.end_aligned = end_aligned;
    for (const auto& ch : pl.chunks) {
        uint32_t at = pl.flex_task_off[ch.fbegin];
        order_pass_tasks(pl.flex_task_off, ch.fbegin, ch.fcount, end_aligned,
                         [&](uint32_t w, uint32_t ps) { pl.flex_tasks[at++] = w * 64u + ps; });
    }
    if (piped) {
        pl.single_task_off.assign(1, 0);
        for (uint32_t p : pl.singles)
            pl.single_task_off.push_back(pl.single_task_off.back() + (qlen[p] && tlen[p] ? n_passes(qlen[p]) : 0));
        pl.single_tasks.assign(pl.single_task_off.back(), 0ull);
        for (const auto& ch : pl.chunks) {
            if (ch.spasses < 2) continue;  // single-pass singles: the one-wave-per-pair fill
            uint32_t at = pl.single_task_off[ch.sbegin];
            order_pass_tasks(pl.single_task_off, ch.sbegin, ch.scount, end_aligned,
                             [&](uint32_t w, uint32_t ps) { pl.single_tasks[at++] = ((uint64_t)w << 32) | ps; });
        }
    }
    for (const auto& c : pl.chunks) {
        pl.ws_ptr_dwords = std::max(pl.ws_ptr_dwords, c.ptr_dwords);
        pl.ws_bnd_words = std::max(pl.ws_bnd_words, c.bnd_words);
    }
}

void build_affine_plan(AffinePlan& pl, uint32_t n_pairs, const uint32_t* qlen, const uint32_t* tlen, int type,
                       int match, int mismatch, int gap_open, int gap_extend, bool want_cigar, uint64_t budget,
                       uint32_t flags, uint32_t wave_quantum) {
    pl = AffinePlan{};
    pl.n_pairs = n_pairs;
    pl.type = type;
    pl.match = match;
    pl.mismatch = mismatch;
    pl.open = gap_open;
    pl.extend = gap_extend;
    pl.want_cigar = want_cigar;
    pl.end_aligned = !(flags & kPlanPassMajor);
    pl.qlen.assign(qlen, qlen + n_pairs);
    pl.tlen.assign(tlen, tlen + n_pairs);
    const std::vector<uint32_t> byc = by_cells(n_pairs, qlen, tlen);
    // units: couples of equal shape for the packed fill (global / semi, values
    // within int16), else single pairs
    const bool dual_ok = !(flags & kPlanInt32Only);
    std::vector<std::pair<uint32_t, uint32_t>> units;  // (a, b); b == UINT32_MAX: single
    units.reserve(n_pairs);
    for (uint32_t k = 0; k < n_pairs;) {
        const uint32_t x = byc[k];
        if (dual_ok && k + 1 < n_pairs && qlen[byc[k + 1]] == qlen[x] && tlen[byc[k + 1]] == tlen[x] &&
            n_passes(qlen[x]) < 64 &&  // hand-off tags epoch * 64 + pass + 1 never wrap (ta_affine.hip)
            affine_fits_int16(type, qlen[x], tlen[x], match, mismatch, gap_open, gap_extend)) {
            units.push_back({x, byc[k + 1]});
            k += 2;
        } else {
            units.push_back({x, UINT32_MAX});
            ++k;
        }
    }
    pl.slot_off = slot_offsets(n_pairs, qlen, tlen, &pl.slots_bytes);
    const uint64_t budget_entries = std::max<uint64_t>(budget / 8, 1);
    pl.ptr_off.assign(n_pairs, 0);
    pl.bnd_off.assign(n_pairs, 0);
    AffinePlan::Chunk c{0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    auto unit_codes = [&](size_t k) -> uint64_t {
        const auto& u = units[k];
        if (!want_cigar) return 0;
        return ptr_dwords(qlen[u.first], tlen[u.first]) +
               (u.second == UINT32_MAX ? 0 : ptr_dwords(qlen[u.second], tlen[u.second]));
    };
    // the packed fill runs one wave per (couple, pass); the int32 fill one per
    // pair, or one per (pair, pass) when pipelined
    const bool pipe_singles = !(flags & kPlanSerialPasses);
    auto unit_waves = [&](size_t k) -> uint64_t {
        const auto& u = units[k];
        if (u.second == UINT32_MAX && !(pipe_singles && qlen[u.first] && tlen[u.first])) return 1;
        return n_passes(qlen[u.first]);
    };
    const std::vector<size_t> starts = chunk_starts(units.size(), budget_entries, wave_quantum, unit_codes, unit_waves);
    size_t next_cut = 1;
    for (size_t k = 0; k < units.size(); ++k) {
        const auto& u = units[k];
        const uint32_t ids[2] = {u.first, u.second};
        const int cnt = u.second == UINT32_MAX ? 1 : 2;
        if (next_cut < starts.size() && k == starts[next_cut]) {
            pl.chunks.push_back(c);
            c = {(uint32_t)pl.order.size(), 0, (uint32_t)pl.singles.size(), 0, (uint32_t)(pl.duals.size() / 2), 0, 0, 0, 0, 0};
            ++next_cut;
        }
        for (int h = 0; h < cnt; ++h) {
            const uint32_t p = ids[h];
            pl.ptr_off[p] = c.ptr_entries;
            pl.bnd_off[p] = c.bnd_entries;
            c.ptr_entries += want_cigar ? ptr_dwords(qlen[p], tlen[p]) : 0;
            // a multi-pass couple's pair A holds the pass hand-off records: 2 buffers x
            // (H, F) x 8 bytes per column = 4 int2 entries; pair B keeps its own
            // boundary row for the int32 fallback ('-' in a query)
            uint64_t bw = bnd_words(qlen[p], tlen[p]);
            if (cnt == 2 && h == 0 && n_passes(qlen[p]) > 1) bw = std::max<uint64_t>(bw, 4ull * ((uint64_t)tlen[p] + 1));
            // a pipelined single: its own records, the same 4 entries per column
            if (cnt == 1 && pipe_singles && n_passes(qlen[p]) > 1) bw = std::max<uint64_t>(bw, 4ull * ((uint64_t)tlen[p] + 1));
            c.bnd_entries += bw;
            pl.order.push_back(p);
            ++c.count;
        }
        if (cnt == 2) {
            pl.duals.push_back(u.first);
            pl.duals.push_back(u.second);
            ++c.dcount;
            c.dpasses = std::max(c.dpasses, n_passes(qlen[u.first]));
        } else {
            pl.singles.push_back(u.first);
            ++c.scount;
            if (pipe_singles && qlen[u.first] && tlen[u.first]) c.spasses = std::max(c.spasses, n_passes(qlen[u.first]));
        }
    }
    if (c.count) pl.chunks.push_back(c);
    bool piped = false;
    for (const auto& ch : pl.chunks) piped |= ch.spasses > 1;
    if (piped) {
        pl.single_task_off.assign(1, 0);
        for (uint32_t p : pl.singles)
            pl.single_task_off.push_back(pl.single_task_off.back() + (qlen[p] && tlen[p] ? n_passes(qlen[p]) : 0));
        pl.single_tasks.assign(pl.single_task_off.back(), 0ull);
        for (const auto& ch : pl.chunks) {
            if (ch.spasses < 2) continue;
            uint32_t at = pl.single_task_off[ch.sbegin];
            order_pass_tasks(pl.single_task_off, ch.sbegin, ch.scount, !(flags & kPlanPassMajor),
                             [&](uint32_t w, uint32_t ps) { pl.single_tasks[at++] = ((uint64_t)w << 32) | ps; });
        }
    }
    for (const auto& ch : pl.chunks) {
        pl.ws_ptr_entries = std::max(pl.ws_ptr_entries, ch.ptr_entries);
        pl.ws_bnd_entries = std::max(pl.ws_bnd_entries, ch.bnd_entries);
    }
}

uint64_t host_batch_code_bytes(uint32_t n_pairs, const uint32_t* qlen, const uint32_t* tlen, uint64_t bytes_per_entry) {
    uint64_t need = 0;
    for (uint32_t p = 0; p < n_pairs; ++p) need += ptr_dwords_blk(qlen[p], tlen[p]) * bytes_per_entry;
    return need;
}

}  // namespace ta
