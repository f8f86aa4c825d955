/*
 * oracle/align_oracle.c -- CPU restatement of the reference team::Align()
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (bioinfo1_amd/,
 * libteam_alignment.so) may link, load or call this file.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only
 * as the checker / the timed CPU baseline.
 *
 * Parity is pinned: tests/test_oracle.py checks this restatement against the
 * golden vectors in tests/golden/ which were produced by the reference's own
 * team_alignment.cpp compiled unmodified from /root/reference (see
 * oracle/Makefile and tests/golden/make_golden.py).
 *
 * It keeps the reference's algorithmic shape: a freshly
 * allocated, zero-filled (n+1)x(m+1) matrix of 8-byte {cost, parent} cells,
 * row-major fill, parent-pointer traceback, reverse, decimal run-length
 * encoding.  Every step cites the reference line it restates
 * (paths relative to /root/reference/team_alignment/).
 *
 * Arithmetic note: the reference adds plain `int`s.  Signed overflow is UB in
 * C/C++, but the compiled reference wraps (two's complement).  We add in
 * uint32 and reinterpret, which is what the compiled reference does and what
 * the GPU's v_add_u32 does.
 */
#include <limits.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_MATCH 0  /* team_alignment.cpp:8  */
#define OR_INSERT 1 /* team_alignment.cpp:9  (consumes target only) */
#define OR_DELETE 2 /* team_alignment.cpp:10 (consumes query only)  */

enum { OR_OK = 0, OR_ERR_BAD_TYPE = 1, OR_ERR_CIGAR = 2, OR_ERR_NOMEM = 3, OR_ERR_CAP = 4 };

typedef struct {
    int cost;   /* team_alignment.cpp:16 */
    int parent; /* team_alignment.cpp:17 */
} or_cell;

static inline int wadd(int a, int b) { return (int)((uint32_t)a + (uint32_t)b); }

/* match_func, team_alignment.cpp:20-23: raw byte equality, case-sensitive. */
static inline int or_match(char a, char b, int match, int mismatch) { return a == b ? match : mismatch; }

/* indel, team_alignment.cpp:25-28: a '-' character makes the gap free. */
static inline int or_indel(char c, int gap) { return c == '-' ? 0 : gap; }

/* Run-length compress ops[0..len) (already in forward order) into out.
 * team_alignment.cpp:145-160 / 222-237 / 319-334.  When len == 0 the
 * reference reads result[0] of an empty std::string (== '\0') and emits
 * "1" followed by that NUL: the 2-byte string "1\0". */
static int or_rle(const char* ops, size_t len, char* out, size_t cap, size_t* out_len) {
    size_t w = 0;
    char prev = len ? ops[0] : '\0';
    unsigned long count = 1;
    char digits[24];
    for (size_t k = 1; k <= len; ++k) {
        if (k < len && ops[k] == prev) {
            ++count;
            continue;
        }
        /* flush run (to_string(count) + prev) */
        int nd = 0;
        unsigned long c = count;
        do {
            digits[nd++] = (char)('0' + c % 10);
            c /= 10;
        } while (c);
        if (w + (size_t)nd + 1 > cap) return OR_ERR_CAP;
        while (nd) out[w++] = digits[--nd];
        out[w++] = prev;
        if (k < len) {
            prev = ops[k];
            count = 1;
        }
    }
    if (len == 0) { /* "1\0" */
        if (cap < 2) return OR_ERR_CAP;
        out[0] = '1';
        out[1] = '\0';
        w = 2;
    }
    *out_len = w;
    return OR_OK;
}

/* The same RLE for affine_oracle.c (the extension shares the reference's CIGAR format). */
int or_rle_public(const char* ops, size_t len, char* out, size_t cap, size_t* out_len) {
    return or_rle(ops, len, out, cap, out_len);
}

/*
 * oracle_align -- restates team::Align (team_alignment.cpp:49-350).
 *   type: 0 global, 1 local, 2 semiGlobal (team_alignment.hpp:8-12).
 *   want_cigar != 0 mirrors passing a non-null std::string* cigar.
 *   cigar bytes are written to cigar_out[0..*cigar_len) (not NUL-terminated;
 *   the "1\0" case contains an embedded NUL).
 * Returns OR_OK, OR_ERR_BAD_TYPE (reference throws "Unknown AlignmentType
 * provided.", :73/:347) or OR_ERR_CIGAR ("Unknown error in determining cigar
 * string.", :135/:214/:299).
 */
int oracle_align(const char* q, unsigned n, const char* t, unsigned m, int type, int match, int mismatch,
                 int gap, int want_cigar, int* score_out, unsigned* target_begin_out, char* cigar_out,
                 size_t cigar_cap, size_t* cigar_len) {
    int init;
    switch (type) { /* team_alignment.cpp:58-74 */
        case 0: init = gap; break;
        case 1: init = 0; break;
        case 2: init = 0; break;
        default: return OR_ERR_BAD_TYPE;
    }
    const size_t W = (size_t)m + 1;
    /* team_alignment.cpp:77: value-initialised (zeroed) matrix */
    or_cell* M = (or_cell*)calloc(((size_t)n + 1) * W, sizeof(or_cell));
    if (!M) return OR_ERR_NOMEM;
#define C(i, j) M[(size_t)(i) * W + (size_t)(j)]
    /* team_alignment.cpp:83-86: first column (unsigned * int) */
    for (unsigned i = 0; i <= n; ++i) {
        C(i, 0).cost = (int)(i * (unsigned)init);
        C(i, 0).parent = OR_DELETE;
    }
    /* team_alignment.cpp:89-92: first row, row wins at (0,0) */
    for (unsigned j = 0; j <= m; ++j) {
        C(0, j).cost = (int)(j * (unsigned)init);
        C(0, j).parent = OR_INSERT;
    }
    /* fill: global 102-116, local 171-194, semi 249-264 (identical body,
     * local adds the clamp + first-strict argmax) */
    int max_cost = INT_MIN;
    unsigned gi = 0, gj = 0;
    for (unsigned i = 1; i <= n; ++i) {
        const char qc = q[i - 1];
        const int gq = or_indel(qc, gap);
        or_cell* row = &C(i, 0);
        const or_cell* up = &C(i - 1, 0);
        for (unsigned j = 1; j <= m; ++j) {
            const char tc = t[j - 1];
            const int o0 = wadd(up[j - 1].cost, or_match(qc, tc, match, mismatch));
            const int o1 = wadd(row[j - 1].cost, or_indel(tc, gap));
            const int o2 = wadd(up[j].cost, gq);
            int c = o0, p = OR_MATCH;
            if (o1 > c) { c = o1; p = OR_INSERT; } /* strict >, :108-113 */
            if (o2 > c) { c = o2; p = OR_DELETE; }
            if (type == 1) {
                if (c < 0) c = 0;         /* :185, parent kept */
                if (c > max_cost) {       /* :186-192 first strict max */
                    max_cost = c;
                    gi = i;
                    gj = j;
                }
            }
            row[j].cost = c;
            row[j].parent = p;
        }
    }
    unsigned tb = 0;
    if (type == 0) { /* :117-121 */
        gi = n;
        gj = m;
        tb = 0;
    } else if (type == 1) { /* :197-199 end column + 1 */
        tb = gj + 1;
    } else { /* :265-278 last column (i ascending) then last row (strict) */
        for (unsigned i = 0; i <= n; ++i)
            if (C(i, m).cost > max_cost) {
                max_cost = C(i, m).cost;
                gi = i;
                gj = m;
            }
        for (unsigned j = 0; j <= m; ++j)
            if (C(n, j).cost > max_cost) {
                max_cost = C(n, j).cost;
                gi = n;
                gj = j;
            }
        tb = 0; /* :283-285 */
    }
    const int score = C(gi, gj).cost; /* :169/245/342 */
    int status = OR_OK;
    if (want_cigar) {
        /* worst case: n+m ops + semi tail (bounded by n+m) */
        char* ops = (char*)malloc((size_t)n + (size_t)m + 1);
        size_t nops = 0;
        if (!ops) {
            free(M);
            return OR_ERR_NOMEM;
        }
        unsigned i = gi, j = gj;
        if (type == 1) { /* :201-217 while cost > 0 */
            while (C(i, j).cost > 0) {
                const int d = C(i, j).parent;
                if (d == OR_MATCH) { ops[nops++] = 'M'; --i; --j; }
                else if (d == OR_INSERT) { ops[nops++] = 'I'; --j; }
                else if (d == OR_DELETE) { ops[nops++] = 'D'; --i; }
                else { status = OR_ERR_CIGAR; break; }
            }
        } else { /* global :123-138, semi :286-302 */
            /* semi tests the stale loop variable j (== m+1 > 0) instead of
             * global_j > 0 in the INSERT branch (:292).  Only row 0 holds
             * INSERT parents at j == 0 and (0,0) ends the walk, so the two
             * readings coincide; we restate the stale form literally. */
            const int semi_stale_j_pos = 1; /* j after the row scan = m+1 > 0 */
            while (i > 0 || j > 0) {
                const int d = C(i, j).parent;
                if (i > 0 && j > 0 && d == OR_MATCH) { ops[nops++] = 'M'; --i; --j; }
                else if ((type == 2 ? semi_stale_j_pos : j > 0) && d == OR_INSERT) { ops[nops++] = 'I'; --j; }
                else if (i > 0 && d == OR_DELETE) { ops[nops++] = 'D'; --i; }
                else { status = OR_ERR_CIGAR; break; }
            }
        }
        if (status == OR_OK) {
            /* reverse (:141, :218, :303) */
            for (size_t a = 0, b = nops ? nops - 1 : 0; a < b; ++a, --b) {
                char x = ops[a];
                ops[a] = ops[b];
                ops[b] = x;
            }
            char* full = ops;
            size_t nfull = nops;
            char* grown = NULL;
            if (type == 2 && (gj != m || gi != n)) { /* :306-315 trailing I / D */
                size_t extra = (gi == n) ? (size_t)(m - gj) : (gj == m ? (size_t)(n - gi) : 0);
                char c = (gi == n) ? 'I' : 'D';
                grown = (char*)malloc(nops + extra + 1);
                if (!grown) { free(ops); free(M); return OR_ERR_NOMEM; }
                memcpy(grown, ops, nops);
                memset(grown + nops, c, extra);
                full = grown;
                nfull = nops + extra;
            }
            int r = or_rle(full, nfull, cigar_out, cigar_cap, cigar_len);
            if (r) status = r;
            free(grown);
        }
        free(ops);
    }
#undef C
    free(M);
    if (status != OR_OK) return status;
    if (score_out) *score_out = score;
    if (target_begin_out) *target_begin_out = tb;
    return OR_OK;
}

/* Upper bound on CIGAR bytes for an n x m pair: every run costs
 * digits(count)+1 <= 2*count bytes, and there are at most n+m ops;
 * the empty case costs 2 ("1\0"). */
size_t oracle_cigar_bound(unsigned n, unsigned m) { return 2 * ((size_t)n + (size_t)m) + 2; }

/*
 * Batch driver used by the tests and by bench.py's cpu_baseline.  SoA inputs
 * (concatenated bytes + offsets + lengths), CIGAR into per-pair fixed slots of
 * oracle_cigar_bound() bytes at cigar_slot_off[p].  OpenMP over pairs with
 * schedule(dynamic), as the reference mapper intended (team_mapper.cpp:596).
 * Returns the number of pairs with a non-OK status (status[] per pair).
 */
int oracle_align_batch(unsigned n_pairs, const char* qbytes, const uint64_t* qoff, const uint32_t* qlen,
                       const char* tbytes, const uint64_t* toff, const uint32_t* tlen, int type, int match,
                       int mismatch, int gap, int want_cigar, int n_threads, int32_t* scores,
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
        int r = oracle_align(qbytes + qoff[p], qlen[p], tbytes + toff[p], tlen[p], type, match, mismatch, gap,
                             want_cigar, &sc, &tb, slot, oracle_cigar_bound(qlen[p], tlen[p]), &cl);
        status[p] = r;
        scores[p] = sc;
        target_begins[p] = tb;
        cigar_lens[p] = (uint32_t)cl;
        if (r) ++bad;
    }
    return bad;
}

int oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/*
 * Size-independent property check (TEST INFRASTRUCTURE): walks a CIGAR the
 * way team_alignment.cpp builds it and recomputes the score of that path, for
 * batches too large to re-align on the CPU.  Returns 0 when the CIGAR
 * consumes exactly what the mode requires and the path's score equals
 * `score`; otherwise a nonzero code naming the first violated property.
 *   global (cpp:123-160): path (0,0)->(n,m); every op is charged.
 *   local  (cpp:201-237): path ends at the goal (gj = target_begin-1) and is
 *                         charged in full; consumption <= n, m.
 *   semi   (cpp:286-334): path (0,0)->(n,m); boundary runs (I on row 0, D on
 *                         column 0) and the appended trailing run (I on row n,
 *                         D on column m) are free.
 */
int oracle_cigar_check(const char* q, unsigned n, const char* t, unsigned m, int type, int match, int mismatch,
                       int gap, const char* cig, size_t clen, int score, unsigned target_begin) {
    /* parse runs */
    size_t k = 0;
    unsigned long nm = 0, ni = 0, nd = 0;
    if (clen == 2 && cig[0] == '1' && cig[1] == '\0') /* empty op string (cpp:145-160) */
        return (type == 1 ? score == 0 : (n == 0 && m == 0 && score == 0)) ? 0 : 1;
    /* first pass: totals */
    while (k < clen) {
        unsigned long c = 0;
        if (cig[k] < '0' || cig[k] > '9') return 2;
        while (k < clen && cig[k] >= '0' && cig[k] <= '9') c = c * 10 + (unsigned long)(cig[k++] - '0');
        if (k >= clen || c == 0) return 3;
        char op = cig[k++];
        if (op == 'M') nm += c;
        else if (op == 'I') ni += c;
        else if (op == 'D') nd += c;
        else return 4;
    }
    unsigned long qi, tj;
    if (type == 1) {
        if (nm + nd > n || nm + ni > m || target_begin < 1 + nm + ni) return 5;
        tj = target_begin - 1 - (nm + ni); /* path starts at column gj - (M+I), gj = target_begin - 1 */
        qi = 0;                                /* row unknown: try every start row */
    } else {
        if (nm + nd != n || nm + ni != m) return 5;
        qi = 0;
        tj = 0;
    }
    unsigned long rows_hi = (type == 1) ? n - (nm + nd) : 0;
    for (unsigned long r0 = 0; r0 <= rows_hi; ++r0) {
        unsigned long i = (type == 1) ? r0 : qi, j = tj;
        int s = 0, ok = 0;
        size_t kk = 0;
        while (kk < clen) {
            unsigned long c = 0;
            while (cig[kk] >= '0' && cig[kk] <= '9') c = c * 10 + (unsigned long)(cig[kk++] - '0');
            const char op = cig[kk++];
            const int last = kk >= clen;
            /* semi: a trailing I run (row n) / D run (column m) may end in the
             * appended free part (cpp:319-334), merged into the same RLE run:
             * accept if the score matches after any genuine prefix of it */
            const int tail = type == 2 && last && op != 'M';
            if (tail && s == score) ok = 1;
            for (unsigned long x = 0; x < c; ++x) {
                int d;
                if (op == 'M') {
                    d = or_match(q[i], t[j], match, mismatch);
                    ++i, ++j;
                } else if (op == 'I') { /* row 0 = boundary: init per cell (cpp:83-92), never '-' */
                    d = (i == 0) ? (type == 0 ? gap : 0) : or_indel(t[j], gap);
                    ++j;
                } else {
                    d = (j == 0) ? (type == 0 ? gap : 0) : or_indel(q[i], gap);
                    ++i;
                }
                s = wadd(s, d);
                if (tail && s == score) ok = 1;
            }
        }
        if (s == score) ok = 1;
        if (ok) return 0;
        if (type != 1) return type == 0 ? 6 : 7;
    }
    return 8;
}

int oracle_cigar_check_batch(unsigned n_pairs, const char* qbytes, const uint64_t* qoff, const uint32_t* qlen,
                             const char* tbytes, const uint64_t* toff, const uint32_t* tlen, int type, int match,
                             int mismatch, int gap, const int32_t* score, const uint32_t* target_begin,
                             const char* arena, const uint64_t* cig_off, const uint32_t* cig_len, int32_t* status) {
    long bad = 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : bad)
    for (long p = 0; p < (long)n_pairs; ++p) {
        status[p] = oracle_cigar_check(qbytes + qoff[p], qlen[p], tbytes + toff[p], tlen[p], type, match, mismatch,
                                       gap, arena + cig_off[p], cig_len[p], score[p], target_begin[p]);
        bad += status[p] != 0;
    }
    return (int)bad;
}
