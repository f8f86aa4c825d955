/*
 * oracle/affine_oracle.c -- CPU statement of the affine-gap EXTENSION of
 * team::Align (BASELINE config 5, "affine gaps + full CIGAR traceback").
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (bioinfo1_amd/,
 * libteam_alignment.so) links, loads or calls this file.  Only tests/ and
 * bench.py's cpu_baseline leg use it, as the checker / the timed CPU baseline.
 *
 * The reference has no affine-gap alignment: team_alignment.cpp is linear-gap
 * only (the "Gotoh" in team_alignment.hpp:11 is a label).  So this file is a
 * DEFINITION, not a restatement, and parity for gap_open != 0 is UNPINNED
 * against the reference.  The definition is chosen so that it is pinned where
 * the two meet: with gap_open == 0 it reduces exactly -- score, target_begin
 * and CIGAR bytes -- to team::Align(..., gap = gap_extend), for every mode,
 * every scoring and '-' bytes included.  tests/test_affine.py checks that
 * against the reference-built goldens in tests/golden/.
 *
 * Definition (Gotoh, three int32 matrices).  A gap of length L costs
 * gap_open + L * gap_extend; like indel() (team_alignment.cpp:25-28) a '-'
 * byte makes its gap step free: open and extend are both 0 for that step.
 *   go_t = t[j-1]=='-' ? 0 : open+extend,  ge_t = t[j-1]=='-' ? 0 : extend
 *   go_q, ge_q likewise from q[i-1]
 *   E(i,j) = max(H(i,j-1) + go_t, E(i,j-1) + ge_t)   E-ext = (2nd > 1st), ties open
 *   F(i,j) = max(H(i-1,j) + go_q, F(i-1,j) + ge_q)   F-ext likewise
 *   H(i,j) = MATCH diag = H(i-1,j-1) + s(q,t); INSERT if E > H; DELETE if F > H
 *            (strict, MATCH > INSERT > DELETE on ties: :108-113); local clamps
 *            at 0 keeping the source (:185)
 *   boundaries (the reference's :83-92 with a gap of length i / j):
 *            H(i,0) = global ? open + i*extend : 0 (i >= 1), H(0,j) likewise,
 *            H(0,0) = 0;  E(i,0) = F(0,j) = -inf.  '-' is ignored there, as in
 *            the reference's boundary loops.
 *   goal, score and target_begin exactly as the reference (:117-121,
 *   :186-199, :265-285), over H.
 *   traceback from the goal in state H: H-state follows the source (local:
 *   stops at H <= 0, :202); INSERT/DELETE move to E/F-state, which emits one
 *   I/D, moves, and stays in E/F if that cell's E-ext/F-ext is set, else
 *   returns to H-state.  Row 0 / column 0 are INSERT / DELETE runs
 *   (global/semi) as in the reference; then reverse, the semi-global trailing
 *   I/D (:306-315) and the decimal RLE incl. "1\0" (:145-160).
 * With open == 0: H >= E everywhere, so E-ext is never set and E = H(i,j-1) +
 * indel(t[j-1]) = the reference's opt1; likewise F; the walk is the
 * reference's walk.
 *
 * Range: every |value| must stay below 2^26 (the GPU kernel keys the local
 * argmax as 16*H + row): (n + m + 2) * max(|match|, |mismatch|, |open| +
 * |extend|) < 2^26, else OR_ERR_RANGE.  Inside that range nothing wraps.
 */
#include <limits.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { AF_OK = 0, AF_ERR_BAD_TYPE = 1, AF_ERR_NOMEM = 3, AF_ERR_CAP = 4, AF_ERR_RANGE = 5 };
#define AF_NEG (-(1 << 29))

/* defined in align_oracle.c (the reference's RLE, :145-160) */
int or_rle_public(const char* ops, size_t len, char* out, size_t cap, size_t* out_len);

static int iabs_(int x) { return x < 0 ? -x : x; }

int oracle_affine_in_range(unsigned n, unsigned m, int match, int mismatch, int open, int extend) {
    long long pm = iabs_(match);
    if (iabs_(mismatch) > pm) pm = iabs_(mismatch);
    if ((long long)iabs_(open) + iabs_(extend) > pm) pm = (long long)iabs_(open) + iabs_(extend);
    return ((long long)n + m + 2) * pm < (1ll << 26);
}

/* bit layout of the per-cell code: 0..1 source (0 M, 1 I, 2 D), 2 E-ext, 3 F-ext */
int oracle_align_affine(const char* q, unsigned n, const char* t, unsigned m, int type, int match, int mismatch,
                        int open, int extend, int want_cigar, int* score_out, unsigned* target_begin_out,
                        char* cigar_out, size_t cigar_cap, size_t* cigar_len) {
    if (type < 0 || type > 2) return AF_ERR_BAD_TYPE;
    if (!oracle_affine_in_range(n, m, match, mismatch, open, extend)) return AF_ERR_RANGE;
    const int global = type == 0, local = type == 1, semi = type == 2;
    const size_t W = (size_t)m + 1;
    int* Hm = (int*)malloc(((size_t)n + 1) * W * sizeof(int));
    unsigned char* code = (unsigned char*)calloc(((size_t)n + 1) * W, 1);
    int* E = (int*)malloc(W * sizeof(int)); /* E of the current row, by column */
    int* F = (int*)malloc(W * sizeof(int)); /* F of the previous / current row, by column */
    if (!Hm || !code || !E || !F) {
        free(Hm), free(code), free(E), free(F);
        return AF_ERR_NOMEM;
    }
#define H(i, j) Hm[(size_t)(i) * W + (size_t)(j)]
#define CODE(i, j) code[(size_t)(i) * W + (size_t)(j)]
    H(0, 0) = 0;
    for (unsigned j = 1; j <= m; ++j) {
        H(0, j) = global ? open + (int)j * extend : 0;
        F[j] = AF_NEG;
    }
    int max_cost = INT_MIN;
    unsigned gi = 0, gj = 0;
    for (unsigned i = 1; i <= n; ++i) {
        const char qc = q[i - 1];
        const int goq = qc == '-' ? 0 : open + extend, geq = qc == '-' ? 0 : extend;
        H(i, 0) = global ? open + (int)i * extend : 0;
        int e = AF_NEG; /* E(i,0) */
        for (unsigned j = 1; j <= m; ++j) {
            const char tc = t[j - 1];
            const int got = tc == '-' ? 0 : open + extend, get = tc == '-' ? 0 : extend;
            const int eo = H(i, j - 1) + got, ee = e + get;
            const int eext = ee > eo;
            e = eext ? ee : eo;
            const int fo = H(i - 1, j) + goq, fe = F[j] + geq;
            const int fext = fe > fo;
            F[j] = fext ? fe : fo;
            int h = H(i - 1, j - 1) + (qc == tc ? match : mismatch), src = 0;
            if (e > h) { h = e; src = 1; }
            if (F[j] > h) { h = F[j]; src = 2; }
            if (local) {
                if (h < 0) h = 0;
                if (h > max_cost) { max_cost = h; gi = i; gj = j; }
            }
            H(i, j) = h;
            CODE(i, j) = (unsigned char)(src | (eext << 2) | (fext << 3));
        }
    }
    unsigned tb = 0;
    if (global) {
        gi = n;
        gj = m;
    } else if (local) {
        tb = gj + 1;
    } else {
        for (unsigned i = 0; i <= n; ++i)
            if (H(i, m) > max_cost) { max_cost = H(i, m); gi = i; gj = m; }
        for (unsigned j = 0; j <= m; ++j)
            if (H(n, j) > max_cost) { max_cost = H(n, j); gi = n; gj = j; }
    }
    const int score = H(gi, gj);
    int status = AF_OK;
    if (want_cigar) {
        char* ops = (char*)malloc(2 * ((size_t)n + m) + 1);
        if (!ops) status = AF_ERR_NOMEM;
        size_t nops = 0;
        unsigned i = gi, j = gj;
        int state = 0; /* 0 H, 1 E, 2 F */
        while (status == AF_OK) {
            if (state == 0) {
                if (local && (i == 0 || j == 0 || H(i, j) <= 0)) break; /* :202 */
                if (!local && i == 0) { while (j) { ops[nops++] = 'I'; --j; } break; }
                if (!local && j == 0) { while (i) { ops[nops++] = 'D'; --i; } break; }
                const int src = CODE(i, j) & 3;
                if (src == 0) { ops[nops++] = 'M'; --i; --j; }
                else state = src;
            } else if (state == 1) {
                const int ext = (CODE(i, j) >> 2) & 1;
                ops[nops++] = 'I';
                --j;
                state = ext ? 1 : 0;
            } else {
                const int ext = (CODE(i, j) >> 3) & 1;
                ops[nops++] = 'D';
                --i;
                state = ext ? 2 : 0;
            }
        }
        if (status == AF_OK) {
            for (size_t a = 0, b = nops ? nops - 1 : 0; a < b; ++a, --b) {
                char x = ops[a];
                ops[a] = ops[b];
                ops[b] = x;
            }
            if (semi && (gj != m || gi != n)) { /* :306-315 */
                if (gi == n) for (unsigned k = gj; k < m; ++k) ops[nops++] = 'I';
                else if (gj == m) for (unsigned k = gi; k < n; ++k) ops[nops++] = 'D';
            }
            int r = or_rle_public(ops, nops, cigar_out, cigar_cap, cigar_len);
            if (r) status = AF_ERR_CAP;
        }
        free(ops);
    }
#undef H
#undef CODE
    free(Hm), free(code), free(E), free(F);
    if (status != AF_OK) return status;
    if (score_out) *score_out = score;
    if (target_begin_out) *target_begin_out = tb;
    return AF_OK;
}

/* Batch driver (tests, bench.py cpu_baseline): as oracle_align_batch. */
int oracle_align_affine_batch(unsigned n_pairs, const char* qbytes, const uint64_t* qoff, const uint32_t* qlen,
                              const char* tbytes, const uint64_t* toff, const uint32_t* tlen, int type, int match,
                              int mismatch, int open, int extend, int want_cigar, int n_threads, int32_t* scores,
                              uint32_t* target_begins, char* cigar_arena, const uint64_t* cigar_slot_off,
                              uint32_t* cigar_lens, int32_t* status) {
    int bad = 0;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic) reduction(+ : bad)
#endif
    for (long p = 0; p < (long)n_pairs; ++p) {
        int sc = 0;
        unsigned tb = 0;
        size_t cl = 0;
        char* slot = want_cigar ? cigar_arena + cigar_slot_off[p] : NULL;
        const size_t cap = 2 * ((size_t)qlen[p] + tlen[p]) + 2;
        int r = oracle_align_affine(qbytes + qoff[p], qlen[p], tbytes + toff[p], tlen[p], type, match, mismatch,
                                    open, extend, want_cigar, &sc, &tb, slot, cap, &cl);
        status[p] = r;
        scores[p] = sc;
        target_begins[p] = tb;
        cigar_lens[p] = (uint32_t)cl;
        if (r) ++bad;
    }
    return bad;
}

/*
 * Size-independent property (TEST INFRASTRUCTURE): the affine cost of the path
 * a CIGAR spells equals `score`.  Global/semi paths run (0,0)->(n,m) (semi:
 * boundary runs and the appended trailing run are free, and a trailing run
 * may be partly genuine); local paths end at column target_begin-1 at some
 * row.  Runs on row 0 / column 0 are charged as the boundary (global: open +
 * L*extend for the whole boundary run).  Returns 0 when consistent.
 */
int oracle_affine_cigar_check(const char* q, unsigned n, const char* t, unsigned m, int type, int match,
                              int mismatch, int open, int extend, const char* cig, size_t clen, int score,
                              unsigned target_begin) {
    if (clen == 2 && cig[0] == '1' && cig[1] == '\0')
        return (type == 1 ? score == 0 : (n == 0 && m == 0 && score == 0)) ? 0 : 1;
    size_t k = 0;
    unsigned long nm = 0, ni = 0, nd = 0;
    while (k < clen) {
        unsigned long c = 0;
        if (cig[k] < '0' || cig[k] > '9') return 2;
        while (k < clen && cig[k] >= '0' && cig[k] <= '9') c = c * 10 + (unsigned long)(cig[k++] - '0');
        if (k >= clen || c == 0) return 3;
        const char op = cig[k++];
        if (op == 'M') nm += c;
        else if (op == 'I') ni += c;
        else if (op == 'D') nd += c;
        else return 4;
    }
    unsigned long tj0;
    if (type == 1) {
        if (nm + nd > n || nm + ni > m || target_begin < 1 + nm + ni) return 5;
        tj0 = target_begin - 1 - (nm + ni);
    } else {
        if (nm + nd != n || nm + ni != m) return 5;
        tj0 = 0;
    }
    const unsigned long rows_hi = type == 1 ? n - (nm + nd) : 0;
    for (unsigned long r0 = 0; r0 <= rows_hi; ++r0) {
        unsigned long i = r0, j = tj0;
        long long s = 0;
        int ok = 0;
        char prev = 0; /* op of the previous cell (gap opens when the op changes) */
        size_t kk = 0;
        while (kk < clen) {
            unsigned long c = 0;
            while (cig[kk] >= '0' && cig[kk] <= '9') c = c * 10 + (unsigned long)(cig[kk++] - '0');
            const char op = cig[kk++];
            const int last = kk >= clen;
            const int tail = type == 2 && last && op != 'M';
            if (tail && s == score) ok = 1;
            for (unsigned long x = 0; x < c; ++x) {
                long long d;
                if (op == 'M') {
                    d = q[i] == t[j] ? match : mismatch;
                    ++i, ++j;
                } else if (op == 'I') {
                    if (i == 0) d = type == 0 ? (j == 0 ? open + extend : extend) : 0; /* boundary row */
                    else d = t[j] == '-' ? 0 : (prev == 'I' ? extend : open + extend);
                    ++j;
                } else {
                    if (j == 0) d = type == 0 ? (i == 0 ? open + extend : extend) : 0;
                    else d = q[i] == '-' ? 0 : (prev == 'D' ? extend : open + extend);
                    ++i;
                }
                prev = op;
                s += d;
                if (tail && s == score) ok = 1;
            }
        }
        if (s == score) ok = 1;
        if (ok) return 0;
        if (type != 1) return type == 0 ? 6 : 7;
    }
    return 8;
}

int oracle_affine_cigar_check_batch(unsigned n_pairs, const char* qbytes, const uint64_t* qoff, const uint32_t* qlen,
                                    const char* tbytes, const uint64_t* toff, const uint32_t* tlen, int type,
                                    int match, int mismatch, int open, int extend, const int32_t* score,
                                    const uint32_t* target_begin, const char* arena, const uint64_t* cig_off,
                                    const uint32_t* cig_len, int32_t* status) {
    long bad = 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : bad)
    for (long p = 0; p < (long)n_pairs; ++p) {
        status[p] = oracle_affine_cigar_check(qbytes + qoff[p], qlen[p], tbytes + toff[p], tlen[p], type, match,
                                              mismatch, open, extend, arena + cig_off[p], cig_len[p], score[p],
                                              target_begin[p]);
        bad += status[p] != 0;
    }
    return (int)bad;
}
