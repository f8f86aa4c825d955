// tests/cpp/range_proofs.cpp -- brute-force check of the range bounds the
// packed local fills rely on for their three-input max on f16 bit patterns
// (every value must stay in [0, 0x7BFF]):
//   * local_max3_offset (ta_layout.h, ta_dual.hip): S = 16H + z*j - i in both frames
//     (z = 1 - 16 ma, and the equal-gain z = -1 of the fills without codes) plus the
//     offset and the lane frame (z + 16) * lane, for every cell of every row up to n + 15
//     (the last lane's padding rows) and every candidate (diag / left / up before the max);
//   * flex_local_fits (ta_planner.cpp, ta_flex.hip): H itself is bounded by the
//     planner's hmax for every cell, and every cell and candidate of the local
//     flexible fill's frame (ta_layout.h flex_local_c0: zu - gap*r + H with the
//     row-0 clamp base zu anywhere in its 65-step drift from c0) lies in
//     [0, 0x7BFF].
// The DP is the reference's local recurrence (team_alignment.cpp:171-194) on
// random bytes ('-' in targets, whose gap steps are free).  Prints "ok" or the
// first violation; exit status 0 / 1.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "ta_layout.h"
#include "ta_planner.h"

static int match_s(char a, char b, int ma, int mi) { return a == b ? ma : mi; }
static int indel_s(char c, int gap) { return c == '-' ? 0 : gap; }

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 3000;
    std::mt19937 rng(0x3A11);
    // queries never hold '-' in the packed fills (those couples go to the int32 fill)
    const char qalpha[] = "ACGTNa", talpha[] = "ACGT-N";
    long checked = 0, dual_cases = 0, flex_cases = 0;
    for (int it = 0; it < iters; ++it) {
        const uint32_t big = (it % 10 == 0) ? 2000 : 90;  // every tenth near the bounds' limits
        const uint32_t n = 1 + rng() % big, m = 1 + rng() % big;
        const int ma = (int)(rng() % 9) - 2, mi = (int)(rng() % 9) - 6, gap = (int)(rng() % 7) - 4;
        const int na = 2 + rng() % 5;  // alphabet size: more matches when small
        std::string q(n + 16, 'A'), t(m, 'A');
        for (auto& c : q) c = qalpha[rng() % na];
        for (auto& c : t) c = talpha[rng() % na];
        const int offs[2] = {ta::local_max3_offset(n, m, ma, mi, gap, false),
                             ta::local_max3_offset(n, m, ma, mi, gap, true)};
        const bool flex = ta::flex_local_fits(n, m, ma, mi, gap);
        if (offs[0] < 0 && offs[1] < 0 && !flex) continue;
        dual_cases += (offs[0] >= 0) + (offs[1] >= 0);
        flex_cases += flex;
        // rows up to n + 15: the padding rows compute on whatever bytes sit there
        const uint32_t N = n + 15;
        std::vector<long> H((N + 1) * (m + 1), 0);
        auto at = [&](uint32_t i, uint32_t j) -> long& { return H[(size_t)i * (m + 1) + j]; };
        long hmax_pl = (long)std::min(n, m) * std::max({0, ma, mi}) + ((long)n + m) * std::max(0, gap);
        for (uint32_t i = 1; i <= N; ++i)
            for (uint32_t j = 1; j <= m; ++j) {
                const long d = at(i - 1, j - 1) + match_s(q[i - 1], t[j - 1], ma, mi);
                const long l = at(i, j - 1) + indel_s(t[j - 1], gap);
                const long u = at(i - 1, j) + indel_s(q[i - 1], gap);
                long h = d;
                if (l > h) h = l;
                if (u > h) h = u;
                if (h < 0) h = 0;
                at(i, j) = h;
                for (int eq = 0; eq < 2; ++eq) {
                    const int off = offs[eq];
                    if (off < 0) continue;
                    // S of the cell and of each candidate (same row/column offset), in
                    // the frame of the lane that holds row i: + (z + 16) * lane
                    const long z = ta::local_max3_z(ma, eq != 0);
                    const long lane = (long)(((i - 1) % 1024) / 16);
                    // (eq: the left and up candidates enter as one max plus the shared gain --
                    // the same values)
                    for (long cand : {d, l, u, h}) {
                        const long s = 16 * cand + z * (long)j - (long)i + off + (z + 16) * lane;
                        ++checked;
                        if (s < 0 || s > 0x7BFF) {
                            std::printf("max3 offset violated: eq=%d n=%u m=%u sc=%d,%d,%d i=%u j=%u cand=%ld S'=%ld off=%d\n",
                                        eq, n, m, ma, mi, gap, i, j, cand, s, off);
                            return 1;
                        }
                    }
                }
                if (flex && i <= n && h > hmax_pl) {
                    std::printf("flex hmax violated: n=%u m=%u sc=%d,%d,%d H=%ld hmax=%ld\n", n, m, ma, mi, gap, h,
                                hmax_pl);
                    return 1;
                }
                if (flex && i <= n) {
                    const long c0 = ta::flex_local_c0(ma, mi, gap), r = (long)((i - 1) % 16);
                    const long zlo = c0 - 65L * std::max(0, ma - gap), zhi = c0 + 65L * std::max(0, gap - ma);
                    for (long cand : {d, l, u, h}) {
                        ++checked;
                        const long lo = zlo - (long)gap * r + cand, hi = zhi - (long)gap * r + cand;
                        if (lo < 0 || hi > 0x7BFF) {
                            std::printf("flex local frame violated: n=%u m=%u sc=%d,%d,%d i=%u j=%u cand=%ld [%ld, %ld]\n",
                                        n, m, ma, mi, gap, i, j, cand, lo, hi);
                            return 1;
                        }
                    }
                }
            }
    }
    // fits_int16 (ta_planner.cpp) for the global / semi-global dual fill (ta_dual.hip):
    // S = H - ma*j + gap*(j - i), every cell and candidate of rows up to n + 15, the
    // semi row-n values H(n, j) - gap*n, all within int16 whenever it admits the shape
    // (no '-' in either sequence: such couples go to the int32 fill)
    long lin_cases = 0;
    for (int it = 0; it < iters + 4; ++it) {
        const uint32_t big = (it % 10 == 0) ? 3000 : 90;
        uint32_t n = 1 + rng() % big, m = 1 + rng() % big;
        int ma = (int)(rng() % 9) - 2, mi = (int)(rng() % 9) - 6, gap = (int)(rng() % 7) - 4;
        int mode = (it & 1) ? ta::kGlobal : ta::kSemi;
        if (it >= iters) {  // config 5's shape and scoring, and the largest shapes the bound admits
            const uint32_t shapes[4][2] = {{10000, 10000}, {10000, 10000}, {15000, 9000}, {9000, 15000}};
            n = shapes[it - iters][0];
            m = shapes[it - iters][1];
            ma = 1, mi = -1, gap = -1;
            mode = (it - iters) == 1 ? ta::kGlobal : ta::kSemi;
        }
        if (!ta::fits_int16(mode, n, m, ma, mi, gap)) continue;
        ++lin_cases;
        const int na = 2 + rng() % 4;
        const char alpha[] = "ACGTN";
        std::string q(n + 16, 'A'), t(m, 'A');
        for (auto& c : q) c = alpha[rng() % na];
        for (auto& c : t) c = alpha[rng() % na];
        const uint32_t N = n + 15;
        const long init = mode == ta::kGlobal ? gap : 0;
        std::vector<long> H((N + 1) * (m + 1), 0);
        auto at = [&](uint32_t i, uint32_t j) -> long& { return H[(size_t)i * (m + 1) + j]; };
        for (uint32_t i = 0; i <= N; ++i) at(i, 0) = init * (long)i;
        for (uint32_t j = 0; j <= m; ++j) at(0, j) = init * (long)j;
        auto bad = [&](long v, const char* what, uint32_t i, uint32_t j) {
            ++checked;
            if (v >= -32768 && v <= 32767) return false;
            std::printf("fits_int16 violated (%s): mode=%d n=%u m=%u sc=%d,%d,%d i=%u j=%u v=%ld\n", what, mode, n, m, ma,
                        mi, gap, i, j, v);
            return true;
        };
        for (uint32_t i = 1; i <= N; ++i)
            for (uint32_t j = 1; j <= m; ++j) {
                const long d = at(i - 1, j - 1) + (q[i - 1] == t[j - 1] ? ma : mi);
                const long l = at(i, j - 1) + gap, u = at(i - 1, j) + gap;
                const long h = std::max({d, l, u});
                at(i, j) = h;
                const long b = -(long)ma * j + (long)gap * ((long)j - (long)i);
                for (long cand : {d, l, u, h})
                    if (bad(cand + b, "cell", i, j)) return 1;
                if (mode == ta::kSemi && i == n && bad(h - (long)gap * n, "row n", i, j)) return 1;
            }
    }
    // affine_fits_int16 (ta_planner.cpp) for the packed affine fill (ta_affine.hip):
    // S = V - ma*j + X*(j - i) for V = H, E, F and every candidate (diag, E open /
    // extend, F open / extend), the -inf stand-ins H - K, rows up to n + 15, the semi
    // row-n values H - X*n; rolling rows (config 5's 10k x 10k shape included)
    long aff_cases = 0;
    for (int it = 0; it < iters / 2 + 2; ++it) {
        const uint32_t big = (it % 10 == 0) ? 3000 : 90;
        uint32_t n = 1 + rng() % big, m = 1 + rng() % big;
        int ma = (int)(rng() % 9) - 2, mi = (int)(rng() % 9) - 6, O = (int)(rng() % 9) - 5, X = (int)(rng() % 5) - 3;
        int mode = (it & 1) ? ta::kGlobal : ta::kSemi;
        if (it >= iters / 2) {
            n = m = 10000;
            ma = 1, mi = -1, O = -2, X = -1;
            mode = (it - iters / 2) ? ta::kGlobal : ta::kSemi;
        }
        if (!ta::affine_fits_int16(mode, n, m, ma, mi, O, X)) continue;
        ++aff_cases;
        const int na = 2 + rng() % 4;
        const char alpha[] = "ACGTN";
        std::string q(n + 16, 'A'), t(m, 'A');
        for (auto& c : q) c = alpha[rng() % na];
        for (auto& c : t) c = alpha[rng() % na];
        const uint32_t N = n + 15;
        const long K = std::labs(O) + std::labs(X) + 2;
        std::vector<long> Hp(m + 1), Fp(m + 1), Hc(m + 1), Fc(m + 1);
        auto h0 = [&](long i) { return mode == ta::kGlobal && i ? O + i * X : 0L; };
        for (uint32_t j = 0; j <= m; ++j) {
            Hp[j] = h0(j);  // row 0 (global: O + j*X)
            Fp[j] = Hp[j] - K;
        }
        auto bad = [&](long v, const char* what, long i, long j) {
            ++checked;
            if (v >= -32768 && v <= 32767) return false;
            std::printf("affine_fits_int16 violated (%s): mode=%d n=%u m=%u sc=%d,%d,%d,%d i=%ld j=%ld v=%ld\n", what,
                        mode, n, m, ma, mi, O, X, i, j, v);
            return true;
        };
        for (uint32_t i = 1; i <= N; ++i) {
            Hc[0] = h0(i);
            long E = Hc[0] - K;
            Fc[0] = Hc[0] - K;
            if (bad(Hc[0] - (long)X * i, "column 0", i, 0) || bad(E - (long)X * i, "column 0 E", i, 0)) return 1;
            for (uint32_t j = 1; j <= m; ++j) {
                const long b = -(long)ma * j + (long)X * ((long)j - (long)i);
                const long d = Hp[j - 1] + (q[i - 1] == t[j - 1] ? ma : mi);
                const long eo = Hc[j - 1] + O + X, ee = E + X;
                const long fo = Hp[j] + O + X, fe = Fp[j] + X;
                E = std::max(eo, ee);
                const long F = std::max(fo, fe);
                const long h = std::max({d, E, F});
                Hc[j] = h;
                Fc[j] = F;
                for (long v : {d, eo, ee, fo, fe, E, F, h, h - K})
                    if (bad(v + b, "cell", i, j)) return 1;
                if (mode == ta::kSemi && i == n && bad(h - (long)X * n, "row n", i, j)) return 1;
            }
            std::swap(Hp, Hc);
            std::swap(Fp, Fc);
        }
    }
    std::printf("ok: %ld values (%ld max3-offset cases, %ld flex-local cases, %ld global/semi dual cases, %ld affine "
                "cases)\n", checked, dual_cases, flex_cases, lin_cases, aff_cases);
    return 0;
}
