// bioinfo1_amd/csrc/ta_walk2.h -- the local-mode traceback with two pairs
// per wave: each group of G = 32 lanes walks one pair.  Same walk as
// traceback_pair<kLocal> (ta_device.h: one run per iteration from a tile of
// the code matrix, the cost tracked exactly so that the walk stops where the
// reference's does, team_alignment.cpp:201-217; RLE written right to left),
// but every piece of walk state is a VGPR holding its group's value instead
// of an SGPR: the SALU work of the one-pair walk becomes VALU work shared by
// two pairs, and config 2's 10,000 walks fit the chip in one round of waves
// instead of 8,192 walks + a latency-bound tail.  (G = 16, four pairs per
// wave, measured slower: 2,500 waves cannot hide the walk's latency.)
//
// Per group: the tile is G steps x 4 stripes (lane li holds step tt0 + li);
// runs are clipped to G cells; the byte windows hold 2G bytes per sequence
// (lane li: S[base-1-li], S[base-1-G-li]); parked runs are flushed every G.
// Cross-lane reads stay inside the group (ds_bpermute to h*G + idx, G-wide
// shuffles); a ballot's group part is its G bits.
#pragma once

#include "ta_device.h"

namespace ta {
namespace {

// G lanes per group (a pair's walk); group h of the wave holds lanes [h*G, h*G + G)
template <int G>
__device__ __forceinline__ uint32_t group_bits(uint64_t b, uint32_t h) {
    if constexpr (G == 32) return h ? (uint32_t)(b >> 32) : (uint32_t)b;
    else return (uint32_t)(b >> (h * G)) & ((1u << G) - 1u);
}
template <int G>
__device__ __forceinline__ uint32_t gread(uint32_t v, uint32_t h, uint32_t idx) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((h * G + (idx & (G - 1u))) << 2), (int)v);
}
// inclusive prefix sum over the G lanes of the group
template <int G>
__device__ __forceinline__ int group_prefix(int v, uint32_t li) {
#pragma unroll
    for (int o = 1; o < G; o <<= 1) {
        const int u = __shfl_up(v, o, G);
        if (li >= (uint32_t)o) v += u;
    }
    return v;
}
// Lane li: S[base-1-li] (bits 7:0) and S[base-1-G-li] (bits 15:8), zero below S[0].
template <int G>
__device__ __forceinline__ uint32_t seq_window_g(const uint8_t* S, uint32_t base, uint32_t li) {
    uint32_t v = 0;
    if (li < base) v = S[base - 1 - li];
    if (li + G < base) v |= (uint32_t)S[base - 1 - G - li] << 8;
    return v;
}

// The run writer of one group (RunWriter, ta_device.h, with G parked runs).
template <int G>
struct GroupWriter {
    char* end;
    uint32_t used, op, cnt, nb, rc, ro;
    uint32_t h, li;
    __device__ __forceinline__ void flush() {
        const bool act = li < nb;
        uint32_t c = rc;
        const uint32_t digits = 1u + (c >= 10u) + (c >= 100u) + (c >= 1000u) + (c >= 10000u) + (c >= 100000u) +
                                (c >= 1000000u) + (c >= 10000000u) + (c >= 100000000u) + (c >= 1000000000u);
        const uint32_t L = act ? digits + 1u : 0u;
        const uint32_t incl = (uint32_t)group_prefix<G>((int)L, li);
        char* p = end - used - (incl - L) - 1;
        if (act) *p = (char)ro;
#pragma unroll
        for (uint32_t d = 0; d < 10u; ++d) {
            if (d < digits && act) p[-1 - (int)d] = (char)('0' + c % 10u);
            c /= 10u;
        }
        used += gread<G>(incl, h, G - 1);
        nb = 0;
    }
    __device__ __forceinline__ void park() {
        const bool here = li == nb;
        rc = here ? cnt : rc;
        ro = here ? op : ro;
        if (++nb == (uint32_t)G) flush();
    }
    __device__ __forceinline__ void push(uint32_t o, uint32_t k) {
        if (o == op) {
            cnt += k;
            return;
        }
        if (op) park();
        op = o;
        cnt = k;
    }
};

// One group's pair (has = false: the group idles through the walk).
struct GroupPair {
    bool has;
    uint32_t n, m, gi, gj;
    int score;
    const uint32_t* P;  // the pair's codes
    const uint8_t* Q;
    const uint8_t* T;
    char* slot;  // the pair's CIGAR slot (cigar_slot_bytes(n, m))
};

// The local walk of group lane / G's pair; returns the CIGAR's start in the
// slot and its length (the same in every lane of the group).
template <int G>
__device__ __forceinline__ void walk_group_local(const GroupPair& gp, int ma, int mi, int gap, int lane,
                                                 uint64_t* start_in_slot, uint32_t* len) {
    const uint32_t h = (uint32_t)lane / G, li = (uint32_t)lane % G;
    const bool has = gp.has;
    const uint32_t n = gp.n, m = gp.m;
    const uint32_t* P = gp.P;
    const uint8_t* Q = gp.Q;
    const uint8_t* T = gp.T;
    const uint64_t cap = cigar_slot_bytes(n, m);
    const int posM = max(0, max(ma, mi));
    GroupWriter<G> w{gp.slot + cap, 0u, 0u, 0u, 0u, 0u, 0u, h, li};
    uint32_t i = gp.gi, j = gp.gj;
    int H = gp.score;
    // gap runs need no bytes when their sequence has no '-' and gap <= 0
    bool qd = false, td = false;
    for (uint32_t x = li; x < max(n, m); x += G) {
        qd |= x < n && Q[x] == '-';
        td |= x < m && T[x] == '-';
    }
    const bool gfastD = group_bits<G>(ballot(qd), h) == 0 && gap <= 0;
    const bool gfastI = group_bits<G>(ballot(td), h) == 0 && gap <= 0;
    uint32_t qbase = i, tbase = j;
    uint32_t qw = seq_window_g<G>(Q, i, li), tw = seq_window_g<G>(T, j, li);
    const uint32_t Tmax = pass_steps(m);
    uint32_t tP = 0xFFFFFFFFu, tt0 = 0, tL0 = 0;
    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    bool live = has && H > 0 && min(i, j) > 0;  // cost 0 ends the walk (:202); row/col 0 cost 0
    // The iteration runs branch-free for both halves: a finished half computes
    // on frozen coordinates and applies nothing (run 0, its writer's own op).
    // Only rare work branches: tile / window reloads, the prefix-sum stop
    // search and the writer's flush.
    while (ballot(live)) {
        const uint32_t row = (live ? i : 1u) - 1;
        const uint32_t ln = (row >> 4) & 63u, r = row & 15u;
        const uint32_t t = ((live ? j : 1u) - 1) + ln;
        if (live && ((int)((t - tt0) | (ln - tL0)) < 0 || (row >> 10) != tP)) {
            tP = row >> 10;  // kPassRows = 1024
            tL0 = max(ln, 3u) - 3u;
            tt0 = max(t, G - 1u) - (G - 1u);
            const uint32_t ts = tt0 + li;
            c0 = c1 = c2 = c3 = 0;
            if (ts < Tmax) {
                const uint32_t* q = P + ((uint64_t)tP * Tmax + ts) * kWave + tL0;
                c0 = q[0];
                c1 = q[1];
                c2 = q[2];
                c3 = q[3];
            }
        }
        const uint32_t sel = ln - tL0;
        const uint32_t cur = sel == 0 ? c0 : sel == 1 ? c1 : sel == 2 ? c2 : c3;
        const uint32_t kk = (t - tt0) & (G - 1u);
        // bit planes (ta_internal.h Code): row r's D bit at 31 - r, I bit at 15 - r
        const uint32_t sh = 15u - r;
        const uint32_t x = gread<G>(cur, h, kk) >> sh;
        const uint32_t dflag = (x >> 16) & 1u, iflag = x & 1u;
        const uint32_t drun = (uint32_t)__builtin_ctz(~(x >> 16));  // D cells of rows r, r-1, ..
        const uint32_t lsh = iflag ? sh : sh + kk - li;
        const uint32_t v = (cur >> (lsh & 31u)) & 0x10001u;
        const uint32_t mb = group_bits<G>(ballot(v == iflag), h);
        const uint32_t streak = (uint32_t)__clz((int)~(mb << (31u - kk)));  // 32 when all set
        const uint32_t hrun = min(streak, iflag ? j : min(j, r + 1u));
        const uint32_t run = live ? (dflag ? drun : hrun) : 0u;
        const uint32_t op = live ? (dflag ? 'D' : ('M' - 4u * iflag)) : w.op;
        // cost along the run (traceback_pair: move k leaves cell c_k; the walk stops
        // at the first c_k whose cost is 0)
        const bool gfast = op != 'M' && (op == 'D' ? gfastD : gfastI);
        const uint32_t inrun = run >= 32u ? ~0u : ((1u << run) - 1u);
        uint32_t qb = 0, tb = 0;
        int c = 0;
        if (ballot(live && !gfast)) {
            // the bytes of the run's cells (lane li: q[i-1-li], t[j-1-li]) from 2G-byte
            // windows refilled after G rows / columns of progress
            if (live && qbase - i > (uint32_t)G) {
                qbase = i;
                qw = seq_window_g<G>(Q, i, li);
            }
            if (live && tbase - j > (uint32_t)G) {
                tbase = j;
                tw = seq_window_g<G>(T, j, li);
            }
            const uint32_t oq = qbase - i + li, ot = tbase - j + li;  // < 2G
            qb = (gread<G>(qw, h, oq) >> ((oq / G) << 3)) & 0xFFu;
            tb = (gread<G>(tw, h, ot) >> ((ot / G) << 3)) & 0xFFu;
            c = __builtin_popcount(group_bits<G>(ballot(qb == tb), h) & inrun);  // matches of an M run
        }
        const bool whole = gfast || (op == 'M' && H > __mul24((int)run, posM));  // the run cannot reach cost 0
        int Hn = gfast ? H - __mul24((int)run, gap) : H - (__mul24((int)run, mi) + __mul24(c, ma - mi));
        uint32_t emit = run;
        bool stop = false;
        if (ballot(live && !whole)) {  // some half may stop inside its run: prefix sums
            const bool in = li < run;
            int d;
            if (op == 'M') d = (qb == tb) ? ma : mi;
            else d = (((op == 'D') ? qb : tb) == '-') ? 0 : gap;
            const int incl = group_prefix<G>(in ? d : 0, li);
            const uint32_t z = group_bits<G>(ballot(in && H - incl <= 0), h);
            if (live && !whole) {
                if (z) {
                    emit = (uint32_t)__builtin_ctz(z) + 1u;
                    stop = true;
                } else {
                    Hn = H - (int)gread<G>((uint32_t)incl, h, run - 1u);
                }
            }
        }
        H = live ? Hn : H;
        // the writer (RunWriter::push): same op extends the open run, else park it
        const bool same = op == w.op;
        const bool park = !same && w.op != 0u;
        w.rc = (park && li == w.nb) ? w.cnt : w.rc;
        w.ro = (park && li == w.nb) ? w.op : w.ro;
        w.nb += park ? 1u : 0u;
        w.cnt = same ? w.cnt + emit : emit;
        w.op = op;
        if (w.nb == (uint32_t)G) w.flush();
        i -= (op == 'I') ? 0u : emit;
        j -= dflag ? 0u : emit;
        live = live && !stop && H > 0 && min(i, j) > 0;
    }
    // finish (RunWriter::finish): "1" + '\0' for an empty op string (:145-160)
    if (has && !w.op) {
        w.used = 2;
        if (li == 0) {
            *(w.end - 2) = '1';
            *(w.end - 1) = '\0';
        }
    }
    const bool more = has && w.op;
    if (more) w.park();
    if (more && w.nb) w.flush();
    *start_in_slot = cap - w.used;
    *len = w.used;
}

// Local walks of pairs k = (64/G)*widx + h of a traceback launch (a.order).
template <int G>
__device__ __forceinline__ void traceback_group_local(const TraceArgs& a, uint32_t widx, int lane) {
    const uint32_t h = (uint32_t)lane / G, li = (uint32_t)lane % G;
    const uint32_t k = (64u / G) * widx + h;
    GroupPair gp{};
    gp.has = k < a.count;
    const uint32_t p = gp.has ? (a.order ? a.order[a.begin + k] : a.begin + k) : 0u;
    if (gp.has) {
        gp.n = a.qlen[p];
        gp.m = a.tlen[p];
        gp.gi = a.goal_i[p];
        gp.gj = a.goal_j[p];
        gp.score = a.score[p];
        gp.P = a.ptrs + a.ptr_off[p];
        gp.Q = a.qbytes + a.qoff[p];
        gp.T = a.tbytes + a.toff[p];
        gp.slot = a.slots + a.slot_off[p];
    } else {
        gp.P = a.ptrs;
        gp.Q = a.qbytes;
        gp.T = a.tbytes;
        gp.slot = a.slots;
    }
    uint64_t st;
    uint32_t len;
    walk_group_local<G>(gp, a.match, a.mismatch, a.gap, lane, &st, &len);
    if (gp.has && li == 0) {
        a.cigar_start[p] = a.slot_off[p] + st;
        a.cigar_len[p] = len;
    }
}

}  // namespace
}  // namespace ta
