// bioinfo1_amd/csrc/ta_flex.hip -- the packed two-pair fill for pairs of
// DIFFERENT shapes and any length (all three modes), so ragged long-read
// batches (config 3: 1-20 kb windows; `-a local` mapping) get the v_pk_*
// throughput of ta_dual.hip.  Same results and the same 2-bit pointer codes as
// the int32 fill; the traceback kernel is shared.
//
// What differs from dual_pass (ta_dual.hip):
//  * Wave-uniform rebasing.  The stored value is V = S - O with S = H - ma*j
//    (global / semi: S = H - ma*j + gap*(j - i), so that the up candidate is
//    the value above itself, as ta_dual.hip) and O a per-pair wave-uniform
//    int32 offset.  Every 64 steps all lanes
//    subtract the same packed value from all their cells (O absorbs it), so
//    values exchanged between lanes need no conversion.  In a linear-gap DP
//    adjacent cells differ by at most max|score| + |gap|, so
//    the ~1,024 x 64 cells a wave holds, plus 64 steps of drift, span a few
//    thousand: V fits int16 for any n and m, where absolute S does not
//    (S reaches -(n+m) on a 20 kb pair).  Everything absolute -- the pass
//    boundary row, the best of row n, the column-m candidates, the corner --
//    is kept in int32 as V + O.
//  * Two shapes.  The couple shares the query pass count and n mod 16 (so the
//    last lane of the last pass holds the same NV rows for both), pair A has
//    the larger n, and the wave runs max(mA, mB) columns.  Pair B's cells
//    past its own n or m never feed its valid cells (the recurrence only
//    looks up and left), so they are computed and ignored: its pointer codes
//    are stored only for its own steps, its column-m candidates and corner
//    are captured when the lanes reach column mB, its row-n best only counts
//    columns <= mB and is read from its own last lane.
//  * Local mode (team_alignment.cpp:171-194).  S = H - ma*j + gap*(j - i) as
//    in global / semi (the up candidate is the value above itself), held in
//    the lane frame V + (17*gap - ma)*lane (ta_layout.h flex_local_c0), in
//    which the clamp H >= 0 of row r of every lane is V >= zu - gap*r with zu
//    uniform over the wave: the 16 bases of a step are 8 SGPRs (two rows per
//    register, picked by op_sel, as ta_dual.hip) and a rebase is one scalar.
//    The reference's argmax is the first strict maximum in
//    row-major order.  Per step each lane ranks its 16 rows by the key
//    16*(V_r - V_0) + 15 - r (rows of one column differ by at most
//    |score| + |gap| each, so it fits int16: larger H first, then the smaller
//    row), one packed max tree; then per pair an int32 key 16*H + 15 - r
//    against the lane's running best (strict '>': an equal key keeps the
//    earlier column) -- exactly the order of ta_dual.hip's local key, without
//    its 16*H bound on the scores.  Pair B counts only its own rows and
//    columns.
#include "ta_device.h"
#include "ta_packed.h"

namespace ta {
namespace {

#ifdef TA_FLEX_MODE

// the gains as 32-bit adds on the non-negative values (flex_pass SW); 0: v_pk_add_u16
#ifndef TA_SWAR
#define TA_SWAR 1
#endif
// CK (with TA_FLEX_CIGAR, a translation unit of its own): checkpoints instead of codes,
// in the dual fill's layout (ta_layout.h ck_row_index / ck_col_index, each pair with its
// own block count) and as H itself -- the frame of V (rebased every 64 steps, a lane
// frame in local mode) taken out at the store -- for the recomputing walk
// (ta_walk_ck.hip), which tells these pairs by their flag (2)
#ifndef TA_FLEX_CK
#define TA_FLEX_CK 0
#endif
constexpr bool kFlexCk = TA_FLEX_CK != 0;

__device__ __forceinline__ int sext_lo(uint32_t x) { return (int)(int16_t)(x & 0xFFFFu); }
__device__ __forceinline__ int sext_hi(uint32_t x) { return (int)(int16_t)(x >> 16); }

// global-address-space view for the hand-off records (agent-scope atomics on
// global pointers: sc1 loads / stores, never flat)
typedef __attribute__((address_space(1))) unsigned long long gu64;

struct FlexIo {
    const uint8_t* Q[2];
    const uint8_t* T[2];
    uint32_t* ptrs[2];
    uint32_t n[2], m[2];
    // Pass hand-off (each pass of a couple runs on its own wave): the bottom
    // row of pass p goes to 8-byte records rec_w[2*j + h] = tag << 32 |
    // absolute S (the data is its own flag: MI355X guide, Guideline 16 R2),
    // written with relaxed agent-scope (sc1) stores; pass p+1 polls a chunk
    // of 64 columns with sc1 loads until every record carries the tag it
    // expects.  Two buffers alternate by pass parity: pass p+2 overwrites
    // column j only after pass p+1 has written its own column j, i.e. long
    // after pass p+1 read column j of pass p.
    uint64_t* rec_w;        // this pass's bottom row (null on the last pass)
    const uint64_t* rec_r;  // the previous pass's (null on pass 0)
    uint32_t tag_w, tag_r;
    uint32_t* err;
    uint32_t* cbuf;  // CK: this wave's LDS staging of 16 steps' bottom rows, [step][lane]
    // this wave's per-step operands of the current 64 steps, entry k for step 64c + k: both
    // pairs' mismatch tables of the new target byte, the row above, the bytes (flex_pass)
    uint4* lst;
};

struct FlexOut {
    PassOut o[2];
};

// 64 columns per chunk of the previous pass's bottom row (absolute S, both
// pairs); polls (bounded) until the producing wave has written all of them
__device__ __forceinline__ void load_rec_chunk(const FlexIo& io, uint32_t M, uint32_t k, int lane, int (&v)[2]) {
    const uint32_t j = k * 64u + (uint32_t)lane + 1u;
    const gu64* r = (const gu64*)(io.rec_r + 2ull * j);
    for (uint32_t spins = 0;; ++spins) {
        bool ok = true;
        v[0] = v[1] = 0;
        if (j <= M) {
            const uint64_t x = __hip_atomic_load(r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t y = __hip_atomic_load(r + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = (uint32_t)(x >> 32) == io.tag_r && (uint32_t)(y >> 32) == io.tag_r;
            v[0] = (int)(uint32_t)x;
            v[1] = (int)(uint32_t)y;
        }
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
        if (spins > (1u << 22)) {  // bounded: the kernel always ends
            if (lane == 0) atomicOr(io.err, 1u);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// CLS: both queries hold only A, C, G, T -- mismatch flags by table lookup
// (ta_packed.h mismatch_table / row_selector), one v_perm per row.
template <int MODE, bool CIGAR, int NV, bool CLS>
__device__ __forceinline__ FlexOut flex_pass(const FillArgs& a, const FlexIo& io, uint32_t pass, bool last_pass,
                                             bool tdash, int lane) {
    constexpr int R = kRows;
    const int ma = a.match, mi = a.mismatch, gap = a.gap;
    const int init = (MODE == kGlobal) ? gap : 0;
    const int rowb = gap;  // the -gap*i term of S (the up gain is 0)
    const uint32_t KD = rep16(mi - ma);
    const int glg = gap - ma + rowb;  // left gain, target byte != '-'
    const int gld = -ma + rowb;       // left gain, target byte == '-'
    uint32_t ONE = 0x00010001u;
    asm volatile("" : "+s"(ONE));  // opaque: keeps v_pk_min_u16
    const uint32_t M = max(io.m[0], io.m[1]);
    const uint32_t n = io.n[0];  // pair A has the larger n
    const uint32_t row_base = pass * kPassRows;
    const uint32_t nrows = min((uint32_t)kPassRows, n - row_base);
    const uint32_t nl = (nrows + R - 1) / R;
    const uint32_t nlh[2] = {nl, (min((uint32_t)kPassRows, io.n[1] - row_base) + R - 1) / R};
    const bool has_next = !last_pass;
    constexpr bool CK = kFlexCk && CIGAR;
    constexpr bool CODES = CIGAR && !CK;

    constexpr bool LOCAL = MODE == kLocal;
    // local: every value is kept in [0, 0x7BFF] (flex_local_fits) so the clamp
    // folds into a three-input max (pk_max3_pos_bc): every rebase puts the
    // wave-uniform row-0 clamp base zu at C0 (ta_layout.h flex_local_c0) -- a
    // margin for 64 steps of drift and one step of candidates below it.
    // global / semi: every rebase puts lane 0's (or the last lane's) first row
    // at C0 = 0x4000, the middle of the non-negative int16 range, which the
    // wave's values leave by at most 15,000 (flex_fits).  So in every mode the
    // values and candidates are non-negative int16 and the gains can be added
    // by one 32-bit add per row (SW, ta_packed.h swar_add).
    const int C0 = LOCAL ? flex_local_c0(ma, mi, gap) : 0x4000;
    constexpr bool SW = TA_SWAR != 0;
    // local: the lane frame (+ dl * lane; the hand-off adds dl) and the row-0 clamp
    // base zu of the current step, the same in every lane (t = -1 here)
    const int dl = LOCAL ? 17 * gap - ma : 0;
    const uint32_t D2 = rep16(dl);
    int zu = C0 - gap;
    // offsets: S(i, 0) = i * init, so start from the pass's first row
    int O[2] = {wmul(row_base, init - rowb) - C0, wmul(row_base, init - rowb) - C0};
    uint32_t q2[R], H2[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i0 = row_base + (uint32_t)lane * R + r;
        const uint32_t qa = i0 < io.n[0] ? (uint32_t)io.Q[0][i0] : 0u, qb = i0 < io.n[1] ? (uint32_t)io.Q[1][i0] : 0u;
        q2[r] = CLS ? row_selector(qa, qb) : (qa | (qb << 16));
        H2[r] = rep16(wmul((uint32_t)lane * R + r + 1, init - rowb) + C0 + dl * lane);  // S(i, 0) - O (+ frame)
    }
    uint32_t recv = rep16(wmul((uint32_t)lane * R, init - rowb) + C0 + dl * lane);
    uint32_t tc2 = 0, tA = 0x01010101u, tB = 0x01010101u;
    // local: the running best key 16*H + 15 - r and its column per pair
    int bestk[2] = {INT_MIN, INT_MIN};
    uint32_t bestj[2] = {0, 0};
    // captures (absolute int32): column m_h candidates (semi) / corner (global), row-n best (semi)
    int capv[2] = {INT_MIN, INT_MIN}, capr[2] = {0, 0};
    int rb[2] = {INT_MIN, INT_MIN};
    uint32_t rbj[2] = {0, 0};

    // A step's wave-uniform operands -- both pairs' mismatch tables of the new target byte,
    // the row above, the raw bytes -- come from one LDS read of a 64-entry list each lane
    // fills for its column every 64 steps (after the rebase: the row above is stored
    // relative to the chunk's O), instead of v_readlane and SALU table arithmetic per step
    // (as ta_dual.hip LST); the DPP hand-offs take the read registers as their lane-0 value
    uint32_t tnext[2];
    auto tbyte = [&](int h, uint32_t c) -> uint32_t {  // target byte of step 64c + lane
        const uint32_t k = c * 64u + (uint32_t)lane;
        return k < io.m[h] ? (uint32_t)io.T[h][k] : 0u;
    };
#pragma unroll
    for (int h = 0; h < 2; ++h) tnext[h] = tbyte(h, 0);
    // the previous pass's bottom row, polled one 64-column chunk at a time just
    // before it is needed (no prefetch of the next chunk: that would make every
    // pass trail its predecessor by one more chunk)
    int bcur[2] = {0, 0};
    if (pass > 0) load_rec_chunk(io, M, 0, lane, bcur);
    // the list of chunk c (its bytes in tnext; the row above: pass 0 S(0, j), later passes
    // the polled records, less dl -- added back by the hand-off -- and O)
    auto lst_fill = [&](uint32_t c) {
        const int j = (int)(c * 64u) + lane + 1;
        int ta, tb;
        if (pass == 0) {
            const int s0 = (init - ma + rowb) * j - dl;
            ta = s0 - O[0];
            tb = s0 - O[1];
        } else {
            ta = bcur[0] - dl - O[0];
            tb = bcur[1] - dl - O[1];
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // (after the last chunk's reads)
        io.lst[lane] = make_uint4(mismatch_table(tnext[0]), mismatch_table(tnext[1]),
                                  ((uint32_t)ta & 0xFFFFu) | ((uint32_t)tb << 16), tnext[0] | (tnext[1] << 16));
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
        for (int h = 0; h < 2; ++h) tnext[h] = tbyte(h, c + 1);
    };
    lst_fill(0);
    const uint32_t steps = M + nl - 1;
    const uint32_t Tmax0 = pass_steps(io.m[0]), Tmax1 = pass_steps(io.m[1]);
    // CK: each pair's blocks of this pass (ta_layout.h ck_row_index: nb_h * 1024 dwords a pass)
    const uint32_t nbh[2] = {blk_count(io.m[0]), blk_count(io.m[1])};
    uint32_t* prow0 = CIGAR ? io.ptrs[0] + (uint64_t)pass * (CK ? nbh[0] * (kBlkSteps * kWave) : Tmax0 * kWave) : nullptr;
    uint32_t* prow1 = CIGAR ? io.ptrs[1] + (uint64_t)pass * (CK ? nbh[1] * (kBlkSteps * kWave) : Tmax1 * kWave) : nullptr;
    // CK, global / semi: H = V + O + (ma - gap) j + gap i for the cell of row i, column j,
    // j = t - l + 1 at step t: the lane's part for its bottom row (i = 16 (l + 1) in the
    // pass); the step's part, O + (ma - gap) (t + 1), is per pair and wave-uniform (ck_step)
    const uint32_t KLB = rep16(-(ma - rowb) * lane + rowb * (int)(row_base + (uint32_t)(lane + 1) * R));
    auto ck_step = [&](uint32_t t, int c) -> uint32_t {  // (+ c in each half)
        const int u = (ma - rowb) * (int)(t + 1) + c;
        return ((uint32_t)(O[0] + u) & 0xFFFFu) | ((uint32_t)(O[1] + u) << 16);
    };
    // CK: H of row r from its value (local: above the row's clamp base zu - gap r, the
    // lane frame and O cancel, ta_flex.hip header)
    auto ck_h = [&](uint32_t v, int r, uint32_t t) -> uint32_t {
        if constexpr (LOCAL) return pk_sub(v, rep16(zu - gap * r));
        else return pk_add(pk_add(v, KLB), ck_step(t, -rowb * (R - 1 - r)));
    };
    // every 16 steps (and at the pass's end): the staged bottom rows of the steps up to t,
    // and at a block's end (full) the 16 rows, both split by pair (v_perm); pair B only
    // within its own blocks
    auto ck_flush = [&](uint32_t t, bool full) {
        const uint32_t b = t >> 4;
        uint32_t x[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) x[q] = io.cbuf[q * kWave + lane];
        uint32_t hr[R];
        if (full) {
#pragma unroll
            for (int r = 0; r < R; ++r) hr[r] = ck_h(H2[r], r, t);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (b >= nbh[h]) continue;
            const uint32_t sel = h ? 0x07060302u : 0x05040100u;
            uint32_t* dr = (h ? prow1 : prow0) + ((uint64_t)b * kWave + (uint32_t)lane) * 8u;
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 2; ++q)
                *reinterpret_cast<uint4*>(dr + 4 * q) =
                    make_uint4(__builtin_amdgcn_perm(x[8 * q + 1], x[8 * q], sel), __builtin_amdgcn_perm(x[8 * q + 3], x[8 * q + 2], sel),
                               __builtin_amdgcn_perm(x[8 * q + 5], x[8 * q + 4], sel), __builtin_amdgcn_perm(x[8 * q + 7], x[8 * q + 6], sel));
            if (full) {
                uint32_t* dc = dr + (uint64_t)nbh[h] * kWave * 8u;
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    *reinterpret_cast<uint4*>(dc + 4 * q) =
                        make_uint4(__builtin_amdgcn_perm(hr[8 * q + 1], hr[8 * q], sel), __builtin_amdgcn_perm(hr[8 * q + 3], hr[8 * q + 2], sel),
                                   __builtin_amdgcn_perm(hr[8 * q + 5], hr[8 * q + 4], sel), __builtin_amdgcn_perm(hr[8 * q + 7], hr[8 * q + 6], sel));
            }
        }
    };

    auto reload = [&](uint32_t t) {
        if (pass > 0) {
            load_rec_chunk(io, M, t >> 6, lane, bcur);
        }
        // rebase (every 64 steps, all lanes alike): a lane that holds current cells
        // to C0; local: the row-0 clamp base zu back to C0 (both pairs alike)
        const uint32_t d = LOCAL ? rep16(zu - C0) : pk_sub((uint32_t)rdlane((int)H2[0], t < M ? 0u : nl - 1), rep16(C0));
#pragma unroll
        for (int r = 0; r < R; ++r) H2[r] = pk_sub(H2[r], d);
        recv = pk_sub(recv, d);
        if (LOCAL) zu = C0;
        O[0] += sext_lo(d);
        O[1] += sext_hi(d);
        lst_fill(t >> 6);
    };
    auto capture = [&](int h, int j, bool active) {
        // lanes at column m_h: this pass's column-m candidates (semi) or the corner (global)
        if (!active || j != (int)io.m[h]) return;
        const int oh = O[h];
        if (MODE == kSemi) {
            const uint32_t nv = (uint32_t)lane < nlh[h] - 1 ? R : ((uint32_t)lane == nlh[h] - 1 ? NV : 0);
            int cv = INT_MIN, cr = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                // H - (ma - gap)*m_h: S plus the row term gap*i
                const int v = (h ? sext_hi(H2[r]) : sext_lo(H2[r])) + oh + rowb * (int)(row_base + (uint32_t)lane * R + r + 1);
                if ((uint32_t)r < nv && v > cv) {
                    cv = v;
                    cr = r;
                }
            }
            capv[h] = cv;
            capr[h] = cr;
        } else {
            capv[h] = (h ? sext_hi(H2[NV - 1]) : sext_lo(H2[NV - 1])) + oh + rowb * (int)io.n[h];  // row n_h
        }
    };
    auto step = [&](uint32_t t, auto masked_tag) {
        constexpr bool MASKED = decltype(masked_tag)::value;
        const uint4 e = io.lst[t & 63u];  // (one address for the wave: a broadcast)
        const uint32_t prev = recv;
        recv = (uint32_t)wave_shr1((int)e.z, (int)H2[R - 1]);
        if constexpr (LOCAL) recv = pk_add(recv, D2);  // into this lane's frame
        if constexpr (CLS) {
            tA = (uint32_t)wave_shr1((int)e.x, (int)tA);
            tB = (uint32_t)wave_shr1((int)e.y, (int)tB);
            if (tdash) tc2 = (uint32_t)wave_shr1((int)e.w, (int)tc2);
        } else {
            tc2 = (uint32_t)wave_shr1((int)e.w, (int)tc2);
        }
        if (LOCAL) zu += gap - ma;

        const int j = (int)t - lane + 1;
        const bool active = !MASKED || (((uint32_t)lane < nl) & (j >= 1) & (j <= (int)M));
        uint32_t acc0 = 0, acc1 = 0;
        if (active) {
            uint32_t GL = rep16(glg), GLk = swar_k(glg);
            if (tdash) {
                const int ga = ((tc2 & 0xFFFFu) == '-') ? gld : glg;
                const int gb = ((tc2 >> 16) == '-') ? gld : glg;
                GL = ((uint32_t)ga & 0xFFFFu) | ((uint32_t)gb << 16);
                GLk = (uint32_t)(ga + gb * 65536);  // (per half: swar_add's constant)
            }
            auto e_of = [&](int r) {  // 0 on a match, 1 otherwise
                if constexpr (CLS) return mismatch_flags(tA, tB, q2[r]);
                else return pk_min_u16(q2[r] ^ tc2, ONE);
            };
            uint32_t dnext = pk_mad_i16(e_of(0), KD, prev);
            uint32_t upv = recv;
            // local: the clamp bases of rows 2k, 2k + 1 in the halves of W[k] (op_sel
            // picks one for both pairs), wave-uniform (SALU); all >= 0, no borrows
            uint32_t W[R / 2];
            if constexpr (LOCAL) {
                W[0] = ((uint32_t)zu & 0xFFFFu) | ((uint32_t)(zu - gap) << 16);
#pragma unroll
                for (int k = 1; k < R / 2; ++k) W[k] = W[0] - (uint32_t)(2 * k * gap) * 0x10001u;
            }
            static_for<0, R>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                const uint32_t old = H2[r];
                const uint32_t diag = dnext;
                const uint32_t left = SW ? swar_add(old, GLk) : pk_add(old, GL);
                if constexpr (r + 1 < R) dnext = pk_mad_i16(e_of(r + 1), KD, old);
                const uint32_t up = upv;  // the value above itself (S's -gap*i term)
                const uint32_t m1 = pk_max(diag, left);
                uint32_t hv;
                if constexpr (LOCAL) hv = pk_max3_pos_bc<r & 1>(m1, up, W[r / 2]);  // clamp folded in, :185
                else hv = pk_max(m1, up);
                if (CODES) {
                    // raw compares (D wins over I in the walk; local walks track the cost)
                    const uint32_t wd = pk_sub_sat(m1, up);
                    const uint32_t wi = pk_sub_sat(diag, left);
                    uint32_t& acc = (r < 8) ? acc0 : acc1;
                    acc = bfi(0x01010101u << (7 - (r & 7)), sign_bytes(wd, wi), acc);
                }
                H2[r] = hv;
                upv = hv;
            });
            if (LOCAL) {
                // the lane's best row of this column per pair: key 16*(V_r - V_0) + 15 - r,
                // + kKeyOff so that the keys are non-negative for the three-input max tree.
                // H_r - H_0 = V_r - V_0 + gap*r (row r's clamp base is gap*r below row 0's);
                // |16*(H_r - H_0)| <= 16*15*2*mag < 4096 (flex_fits)
                constexpr int kKeyOff = 4096;
                uint32_t K[R];
                K[0] = rep16(kKeyOff + 15);
#pragma unroll
                for (int r = 1; r < R; ++r)
                    K[r] = pk_mad_i16(pk_sub(H2[r], H2[0]), 0x00100010u, rep16(kKeyOff + 15 - r + 16 * gap * r));
                const uint32_t lo = max3_reduce<NV>(K);
                uint32_t kA = lo, kB = lo;
                if constexpr (NV != R) {  // the pair's last lane holds NV valid rows
                    const uint32_t full = pk_max(lo, max3_reduce<R - NV>(K + NV));
                    kA = ((uint32_t)lane == nlh[0] - 1) ? lo : full;
                    kB = ((uint32_t)lane == nlh[1] - 1) ? lo : full;
                }
                const int kk[2] = {sext_lo(kA) - kKeyOff, sext_hi(kB) - kKeyOff};
                const int v0[2] = {sext_lo(H2[0]), sext_hi(H2[0])};
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    // 16*H + 15 - r = 16*H_0 + key (cells of this pair only), where H_0 = V_0 - zu:
                    // row 0's value above its clamp base (the lane frame and O cancel)
                    const int key = ((v0[h] - zu) << 4) + kk[h];
                    const bool better = (uint32_t)lane < nlh[h] && j <= (int)io.m[h] && key > bestk[h];
                    bestk[h] = better ? key : bestk[h];
                    bestj[h] = better ? (uint32_t)j : bestj[h];
                }
            }
            if (MODE == kSemi && last_pass) {  // row n of each pair: H = S + ma*j, columns <= m_h, strict '>'
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int v = (h ? sext_hi(H2[NV - 1]) : sext_lo(H2[NV - 1])) + O[h] + (ma - rowb) * j + rowb * (int)io.n[h];
                    const bool better = j <= (int)io.m[h] && v > rb[h];
                    rb[h] = better ? v : rb[h];
                    rbj[h] = better ? (uint32_t)j : rbj[h];
                }
            }
            if (has_next && (uint32_t)lane == nl - 1) {
                const uint64_t tg = (uint64_t)io.tag_w << 32;
                gu64* wr = (gu64*)(io.rec_w + 2ull * j);
                // (absolute S: out of the lane frame)
                __hip_atomic_store(wr, tg | (uint32_t)(sext_lo(H2[R - 1]) + O[0] - dl * lane), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(wr + 1, tg | (uint32_t)(sext_hi(H2[R - 1]) + O[1] - dl * lane), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        // column m_h reached by some lane this step (uniform window test)
        if (!LOCAL && t + 1 >= io.m[0] && t + 1 < io.m[0] + kWave) capture(0, j, active);
        if (!LOCAL && t + 1 >= io.m[1] && t + 1 < io.m[1] + kWave) capture(1, j, active);
        if constexpr (CK) {
            io.cbuf[(t & 15u) * kWave + (uint32_t)lane] = ck_h(H2[R - 1], R - 1, t);  // (flushed by run_steps)
        } else if (CIGAR) {
            const uint32_t off = (t * kWave + (uint32_t)lane) * 4u;
            if (t < Tmax0) *(uint32_t*)((char*)prow0 + off) = __builtin_amdgcn_perm(acc0, acc1, 0x06020400u);
            if (t < Tmax1) *(uint32_t*)((char*)prow1 + off) = __builtin_amdgcn_perm(acc0, acc1, 0x07030501u);
        }
    };
    const uint32_t ramp_end = min(nl - 1, steps);
    uint32_t t = 0, next_reload = 64;
    auto run_steps = [&](uint32_t t_end, auto masked_tag) {
        while (t < t_end) {
            if (t == next_reload) {
                reload(t);
                next_reload += 64;
            }
            uint32_t blk = min(t_end, next_reload);
            if constexpr (CK) blk = min(blk, (t | 15u) + 1u);  // (the flushes outside the step body)
            for (; t + 1 < blk; t += 2) {  // steps in pairs (as ta_dual.hip)
                step(t, masked_tag);
                step(t + 1, masked_tag);
            }
            if (t < blk) step(t++, masked_tag);
            if constexpr (CK) {
                if ((t & 15u) == 0 || t == steps) ck_flush(t - 1, (t & 15u) == 0);
            }
        }
    };
    run_steps(ramp_end, std::true_type{});
    run_steps(M, std::false_type{});
    run_steps(steps, std::true_type{});

    FlexOut out;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        PassOut& o = out.o[h];
        o = PassOut{INT_MIN, 0, 0, INT_MIN, 0, 0};
        if (LOCAL) {
            // larger H, then the first lane (smaller rows); its key has the row, its column the j
            const int v = bestk[h] == INT_MIN ? -1 : (bestk[h] >> 4);
            const int mx = wave_max(v);
            const int fl = first_lane(v == mx);
            if (mx >= 0) {
                const int kf = rdlane(bestk[h], fl);
                o.h = mx;
                o.i = row_base + (uint32_t)fl * R + (uint32_t)(15 - (kf & 15)) + 1;
                o.j = (uint32_t)rdlane((int)bestj[h], fl);
            }
        } else if (MODE == kSemi) {
            // column m_h: H = S + ma*m_h for every row, so S orders them; first lane, then first row
            const int mx = wave_max(capv[h]);
            const int fl = first_lane(capv[h] == mx && capv[h] != INT_MIN);
            if (mx != INT_MIN) {
                o.h = mx + (ma - rowb) * (int)io.m[h];
                o.i = row_base + (uint32_t)fl * R + (uint32_t)rdlane(capr[h], fl) + 1;
                o.j = io.m[h];
            }
            if (last_pass) {
                o.row_h = rdlane(rb[h], nlh[h] - 1);  // INT_MIN: no column (m_h = 0 never reaches here)
                o.row_j = (uint32_t)rdlane((int)rbj[h], nlh[h] - 1);
            }
        } else if (last_pass) {
            o.corner = rdlane(capv[h], nlh[h] - 1) + (ma - rowb) * (int)io.m[h];
        }
    }
    return out;
}

template <int MODE, bool CIGAR, bool CLS>
__device__ __forceinline__ FlexOut flex_pass_nv(const FillArgs& a, const FlexIo& io, uint32_t pass, bool last_pass,
                                                bool tdash, int lane) {
    const uint32_t nrows = min((uint32_t)kPassRows, io.n[0] - pass * kPassRows);
    const uint32_t nv = nrows - ((nrows + kRows - 1) / kRows - 1) * kRows;
    if (nv == kRows) return flex_pass<MODE, CIGAR, kRows, CLS>(a, io, pass, last_pass, tdash, lane);
#define TA_NV_CASE(k) \
    case k: return flex_pass<MODE, CIGAR, k, CLS>(a, io, pass, last_pass, tdash, lane);
    switch (nv) {
        TA_NV_CASE(1) TA_NV_CASE(2) TA_NV_CASE(3) TA_NV_CASE(4) TA_NV_CASE(5) TA_NV_CASE(6) TA_NV_CASE(7)
        TA_NV_CASE(8) TA_NV_CASE(9) TA_NV_CASE(10) TA_NV_CASE(11) TA_NV_CASE(12) TA_NV_CASE(13) TA_NV_CASE(14)
        default: TA_NV_CASE(15)
    }
#undef TA_NV_CASE
}

#ifndef TA_FLEX_WAVES
#define TA_FLEX_WAVES 4
#endif
constexpr uint32_t kSkip = 0xFFFFFFFFu;  // PassOut.i of a couple handed to the int32 fill

// One wave per (couple, pass).  flex order: 2 pair ids per couple, pair A
// (larger n) first; same pass count and n mod 16 (a single long pair may be
// coupled with itself).  A wave takes the next ticket; the chunk's tasks are
// in pass-major order (every couple's pass 0, then every pass 1, ...; the host's
// flex_tasks), so pass p-1 of its couple belongs to a wave that took an earlier
// ticket and is running: every poll ends.  Pass-major also means a pass starts
// long after its predecessor, instead of all passes of a couple starting
// together and each waiting for the one above.
template <int MODE, bool CIGAR>
__device__ __forceinline__ void flex_fill_body(FillArgs a) {
    const int lane = threadIdx.x & 63;
    constexpr bool CK = kFlexCk && CIGAR;
    __shared__ uint32_t cbuf_all[CK ? kWavesPerBlock * 16 * kWave : 1];
    __shared__ uint4 lst_all[kWavesPerBlock * 64];  // (flex_pass: the per-step operands)
    uint32_t tk = 0;
    if (lane == 0) tk = atomicAdd(a.ticket, 1u);
    tk = (uint32_t)__builtin_amdgcn_readfirstlane((int)tk);
    if (tk >= a.n_tasks) return;
    const uint32_t code = a.tasks[a.task_off[a.begin] + tk];  // this chunk's tasks, pass-major
    const uint32_t w = code >> 6, pass = code & 63u;
    const uint32_t g = a.task_off[w] + pass;  // plan-global task index (couple-major): its PassOut
    uint32_t p[2];
    p[0] = a.order[2 * w];
    p[1] = a.order[2 * w + 1];
    FlexIo io;
    bool tdash = false, qdash = false, qother = false;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        io.n[h] = a.qlen[p[h]];
        io.m[h] = a.tlen[p[h]];
        io.Q[h] = a.qbytes + a.qoff[p[h]];
        io.T[h] = a.tbytes + a.toff[p[h]];
        io.ptrs[h] = CIGAR ? a.ptrs + a.ptr_off[p[h]] : nullptr;
        for (uint32_t k = (uint32_t)lane; k < io.m[h]; k += 64) tdash |= io.T[h][k] == '-';
        for (uint32_t k = (uint32_t)lane; k < io.n[h]; k += 64) {
            const uint32_t c = io.Q[h][k];
            qdash |= c == '-';
            qother |= !is_acgt(c);
        }
    }
    PassOut* po = static_cast<PassOut*>(a.pout) + 2ull * g;
    // per-row up gains ('-' in a query) -- and with checkpoints any '-', whose free gap
    // steps the recomputing walk does not model: the int32 fill takes the couple (pass
    // 0's wave hands it over); CK: the walk's flag, 1 handed back, 2 a pair of this fill
    const bool back = __ballot(qdash) || (CK && __ballot(tdash));
    if (CK && a.pflag && lane == 0 && pass == 0) {
        a.pflag[p[0]] = back ? 1 : 2;
        a.pflag[p[1]] = back ? 1 : 2;
    }
    if (back) {
        if (lane == 0) {
            if (pass == 0) {
                const uint32_t k = (p[1] != p[0]) ? 2u : 1u;
                const uint32_t at = atomicAdd(a.fb_count, k);
                a.fb_list[at] = p[0];
                if (k == 2) a.fb_list[at + 1] = p[1];
            }
            po[0].i = kSkip;
            po[1].i = kSkip;
        }
        return;
    }
    tdash = __ballot(tdash) != 0;
    const uint32_t passes = n_passes(io.n[0]);
    const bool last_pass = pass + 1 == passes;
    const uint32_t M = max(io.m[0], io.m[1]);
    uint64_t* rec = reinterpret_cast<uint64_t*>(a.bnd + a.bnd_off[p[0]]);  // 2 buffers x 2(M+1) records
    const uint64_t rb = 2ull * (M + 1);
    io.rec_w = last_pass ? nullptr : rec + (pass & 1u) * rb;
    io.rec_r = pass ? rec + ((pass - 1u) & 1u) * rb : nullptr;
    // never 0, unique per launch and pass; the host zeroes the record buffers
    // before each launch, so a record carries this tag only once written here
    io.tag_w = a.epoch * 64u + pass + 1u;
    io.tag_r = a.epoch * 64u + pass;
    io.err = a.err;
    io.cbuf = cbuf_all + (CK ? (threadIdx.x >> 6) * 16 * kWave : 0);
    io.lst = lst_all + (threadIdx.x >> 6) * 64;
    const FlexOut o = __ballot(qother) == 0 ? flex_pass_nv<MODE, CIGAR, true>(a, io, pass, last_pass, tdash, lane)
                                            : flex_pass_nv<MODE, CIGAR, false>(a, io, pass, last_pass, tdash, lane);
    if (lane == 0) {
        po[0] = o.o[0];
        po[1] = o.o[1];
    }
}

template <int MODE, bool CIGAR>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(TA_FLEX_WAVES))) void flex_fill_kernel(FillArgs a) {
    flex_fill_body<MODE, CIGAR>(a);
}
#if TA_FLEX_CK
// the checkpoint fill under a name of its own (rocprof, profiles/*_by_kernel.json)
template <int MODE>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(TA_FLEX_WAVES))) void flex_fill_ck_kernel(FillArgs a) {
    flex_fill_body<MODE, true>(a);
}
#endif

// After the fill: fold each couple's per-pass results in pass order (the
// upper pass wins ties; semi: row n after column m, :265-278).
template <int MODE>
__global__ void flex_combine_kernel(FillArgs a) {
    const uint32_t w = a.begin + blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= a.begin + a.count) return;
    const uint32_t g0 = a.task_off[w], passes = a.task_off[w + 1] - g0;
    const PassOut* po = static_cast<const PassOut*>(a.pout) + 2ull * g0;
    if (po[0].i == kSkip) return;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t p = a.order[2 * w + h];
        const uint32_t n = a.qlen[p], m = a.tlen[p];
        int best_h = (MODE == kSemi) ? 0 : INT_MIN, corner = 0;
        uint32_t best_i = 0, best_j = (MODE == kSemi) ? m : 0;
        for (uint32_t k = 0; k < passes; ++k) {
            const PassOut& o = po[2 * k + h];
            if (MODE != kGlobal && o.h > best_h) {  // strict: the upper pass wins ties (row-major, :186)
                best_h = o.h;
                best_i = o.i;
                best_j = o.j;
            }
            if (MODE == kSemi && k + 1 == passes && o.row_h > best_h) {
                best_h = o.row_h;
                best_i = n;
                best_j = o.row_j;
            }
            if (MODE == kGlobal && k + 1 == passes) corner = o.corner;
        }
        if (h == 1 && p == a.order[2 * w]) break;  // a pair coupled with itself
        a.score[p] = (MODE == kGlobal) ? corner : best_h;
        a.target_begin[p] = (MODE == kLocal) ? best_j + 1 : 0;  // :197-199
        a.goal_i[p] = (MODE == kGlobal) ? n : best_i;
        a.goal_j[p] = (MODE == kGlobal) ? m : best_j;
    }
}

#endif  // TA_FLEX_MODE
}  // namespace

#ifdef TA_FLEX_MODE
#if TA_FLEX_CK
template <>
hipError_t launch_flex_ck<TA_FLEX_MODE>(const FillArgs& a, hipStream_t s) {
    static_assert(TA_FLEX_CIGAR, "checkpoints replace the codes");
#else
template <>
hipError_t launch_flex_mode<TA_FLEX_MODE, (TA_FLEX_CIGAR != 0)>(const FillArgs& a, hipStream_t s) {
#endif
    if (!a.count) return hipSuccess;
#if TA_FLEX_CIGAR && !TA_FLEX_CK
    if (a.blk == 2) return launch_flex_ck<TA_FLEX_MODE>(a, s);  // (checkpoint plans)
#endif
#if TA_FLEX_CK
    if (a.n_tasks)
        hipLaunchKernelGGL(flex_fill_ck_kernel<TA_FLEX_MODE>, dim3((a.n_tasks + kWavesPerBlock - 1) / kWavesPerBlock),
                           dim3(kBlock), 0, s, a);
#else
    if (a.n_tasks)
        hipLaunchKernelGGL((flex_fill_kernel<TA_FLEX_MODE, TA_FLEX_CIGAR != 0>),
                           dim3((a.n_tasks + kWavesPerBlock - 1) / kWavesPerBlock), dim3(kBlock), 0, s, a);
#endif
    hipLaunchKernelGGL((flex_combine_kernel<TA_FLEX_MODE>), dim3((a.count + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}
#endif

}  // namespace ta
