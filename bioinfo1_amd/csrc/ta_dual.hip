// bioinfo1_amd/csrc/ta_dual.hip -- the DP fill for TWO pairs per wave in
// packed 16-bit lanes (gfx950 v_pk_* ops), for batches of equal-length pairs
// whose scores fit int16.  Same results as fill_kernel (ta_kernels.hip) and
// the same 2-bit pointer codes, so the traceback is shared.
//
// Each 32-bit register holds pair A in bits 15:0 and pair B in bits 31:16.
// The stored value is not H itself but a biased S chosen so that the
// diagonal candidate costs ONE v_pk_mad_i16 (e * (mi-ma) + S_diag, with
// e = min(q ^ t, 1) per half) and the other two at most one v_pk_add each:
//   global / semi:  S = H - ma*j + gap*(j - i)   (the up candidate is the
//                   value above itself, the left one S + 2*gap - ma)
//   local:          S = 16*H + (1 - 16*ma)*j - i
//     (the -i term tags the row: within a step S - Zbase + 15 = 16H + 15 - r
//      is the reference's row-major first-max key; the clamp H >= 0 becomes
//      S >= (1-16ma)j - i, a per-lane-per-step base minus the row index)
// A cell's inputs move exactly as in fill_kernel (lane skew, DPP wave_shr:1).
// The pointer codes never leave the VALU: each compare is the sign of a
// saturating packed subtraction, v_perm_b32 spreads the sign bits of both
// pairs to bytes and v_bfi_b32 inserts them into two row-group accumulators,
// which two more v_perm_b32 per step turn into the per-pair bit-plane dwords
// of ta_internal.h (Code).  No lane masks, no SALU, no v_addc chains.
// Local mode stores the raw compares too (no STOP code): the local walk
// tracks the cell cost and stops where it reaches 0 (ta_device.h WalkSeq).
#include "ta_device.h"
#include "ta_packed.h"

namespace ta {
namespace {

#ifdef TA_DUAL_MODE

struct DualOut {
    PassOut o[2];
};

// BLK: steps staged in LDS between flushes (16: 8 KB per wave; 8: 4 KB, half-block stores;
// 0: no staging, one scattered dword store per step and pair, merged in L2)
#ifndef TA_DUAL_STAGE
#define TA_DUAL_STAGE 16
#endif
constexpr int kDualStage = TA_DUAL_STAGE;
static_assert(kDualStage == 0 || kDualStage == 8 || kDualStage == 16, "dual BLK staging");
constexpr int kDualStageL = kDualStage ? kDualStage : 16;  // (array sizes and masks when staged)
// the local gains as 32-bit adds in the M3 frame (dual_pass SW); 0: v_pk_add_u16
#ifndef TA_SWAR
#define TA_SWAR 1
#endif
// CK (with TA_DUAL_BLK, a translation unit of its own): checkpoints instead of
// codes -- each stripe's bottom row every step and its 16 rows every 16 steps
// (ta_layout.h ck_row_index / ck_col_index), from which the walk recomputes
// the codes of the cells around its path (ta_walk_ck.hip)
#ifndef TA_DUAL_CK
#define TA_DUAL_CK 0
#endif
#if defined(TA_DUAL_BLK) && TA_DUAL_CK
constexpr bool kDualCk = true;
#else
constexpr bool kDualCk = false;
#endif
static_assert(!kDualCk || kDualStage != 0, "the checkpoint fill stages each step's bottom row in LDS");

struct DualIo {
    const uint8_t* Q[2];
    const uint8_t* T[2];
    uint32_t* ptrs[2];
    int32_t* B;  // packed boundary row (pair A's allocation)
    // One wave per (couple, pass) (multi-pass chunks): pass p's
    // bottom row goes to 8-byte records tag << 32 | packed value in pair A's
    // allocation (two buffers by pass parity), written with relaxed agent-scope
    // stores; pass p + 1 polls 64 columns at a time until every record carries
    // the tag it expects (the data is its own flag, as ta_flex.hip).  Null: the
    // in-place row B of a wave that sweeps all passes itself.
    uint64_t* rec_w;
    const uint64_t* rec_r;
    uint32_t tag_w, tag_r;
    uint32_t* err;
    // blocked layout (BLK): this wave's LDS staging of 16 steps, [pair][step][lane]
    uint32_t* cbuf;
    // CLS: this wave's per-step operands of the current 64 steps, entry k for step 64c + k:
    // both pairs' tables of the target byte and the row above (dual_pass LST)
    uint4* lst;
    uint32_t nb;  // blk_count(m)
};

typedef __attribute__((address_space(1))) unsigned long long gu64d;

// columns 64k + lane + 1 of the previous pass's bottom row (packed pairs)
__device__ __forceinline__ int dual_poll_chunk(const DualIo& io, uint32_t m, uint32_t k, int lane) {
    const uint32_t j = k * 64u + (uint32_t)lane + 1u;
    const gu64d* r = (const gu64d*)(io.rec_r + j);
    int v = 0;
    for (uint32_t spins = 0;; ++spins) {
        bool ok = true;
        if (j <= m) {
            const uint64_t x = __hip_atomic_load(r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = (uint32_t)(x >> 32) == io.tag_r;
            v = (int)(uint32_t)x;
        }
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
        if (spins > (1u << 22)) {  // bounded: the kernel always ends
            if (lane == 0) atomicOr(io.err, 1u);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    return v;
}

// One pass of both pairs; see run_pass (ta_kernels.hip) for the shared structure.
// M3 (local only): every value carries the offset `off` (local_max3_offset)
// so that the clamp folds into a three-input max and the stripe's row max is
// a tree of three-input maxima (v_pk_maximum3_f16 on non-negative int16).
// CLS: both queries hold only A, C, G, T -- mismatch flags by table lookup
// (ta_packed.h mismatch_table / row_selector), one v_perm per row.
// BLK: codes in the blocked layout (ta_layout.h blk_index): each step's two
// dwords go to this wave's LDS staging, and every 16 steps each lane writes its
// stripe's 16 steps of both pairs as 64 contiguous bytes (4 x 16-byte stores).
template <int MODE, bool CIGAR, int NV, bool M3, bool CLS, bool BLK = false>
__device__ __forceinline__ DualOut dual_pass(const FillArgs& a, const DualIo& io, uint32_t n, uint32_t m,
                                             uint32_t pass, bool last_pass, int lane, int off = 0) {
    constexpr int R = kRows;
    constexpr bool LOCAL = MODE == kLocal;
    static_assert(!M3 || LOCAL, "three-input maxima: local mode only");
    if constexpr (!M3) off = 0;
    const int ma = a.match, mi = a.mismatch, gap = a.gap;
    const int init = (MODE == kGlobal) ? gap : 0;
    constexpr bool CK = BLK && kDualCk;
    constexpr bool CODES = CIGAR && !CK;
    // EQ (M3 without codes): the equal-gain frame z = -1 (ta_layout.h local_max3_z):
    // H = max(diag + 16s - 2, max(left, up) + 16gap - 1, clamp), the diagonal gain
    // from a byte table (CLS) -- five instructions a row instead of six
    constexpr bool EQ = M3 && !CODES;
    const int zstep = local_max3_z(ma, EQ);  // local: S(0, j) = zstep * j
    const uint32_t KD = rep16(LOCAL ? 16 * (mi - ma) : (mi - ma));
    // left gain (no '-' in these targets); global / semi: the up gain is 0 (the
    // -gap*i term of S), so the left one carries gap twice
    const uint32_t GL = rep16(LOCAL ? 16 * gap + zstep : 2 * gap - ma);
    const uint32_t GUG = rep16(LOCAL ? 16 * gap - 1 : 0);  // up gain (no '-' in these queries)
    // SW (with M3): the two gains as ONE 32-bit add each (ta_packed.h swar_add):
    // every value and candidate of the M3 frame lies in [0, 0x7BFF]
    // (local_max3_offset), so the low half never borrows from the high one
    constexpr bool SW = M3 && TA_SWAR;
    uint32_t GLk = swar_k(LOCAL ? 16 * gap + zstep : 2 * gap - ma), GUGk = swar_k(16 * gap - 1);
    asm volatile("" : "+s"(GLk), "+s"(GUGk));  // SGPR operands (a literal would double the encoding)
    uint32_t ONE = 0x00010001u;
    asm volatile("" : "+s"(ONE));  // opaque: keeps v_pk_min_u16 (see pk_min_u16)
    // EQ: the diagonal gain 16s - 2 as table bytes + 128 (class_table: byte k = ub, or
    // ua for the class-k letter), added with the bias as ONE v_add3_u32 (the walk's TAB
    // sweep, ta_walk_ck.hip); without the tables (not CLS) the mismatch delta then + GM
    const uint32_t ua = (uint32_t)(16 * ma - 2 + 128), ub = (uint32_t)(16 * mi - 2 + 128);
    const uint32_t T0 = ub * 0x01010101u, TX = ua ^ ub;
    const uint32_t GM = rep16(16 * ma - 2);
    uint32_t KN = swar_k(-128);
    asm volatile("" : "+s"(KN));
    const uint32_t Tmax = pass_steps(m);
    const uint32_t row_base = pass * kPassRows;
    const uint32_t nrows = min((uint32_t)kPassRows, n - row_base);
    const uint32_t nl = (nrows + R - 1) / R;
    const bool has_next = !last_pass;
    // UZ (with M3): lane l keeps its values in the frame S + dl*l (dl = zstep + 16),
    // which makes the clamp base of a step the same in every lane: the bases
    // and the argmax column then live in SGPRs (SALU work) instead of VALU
    // registers, for one packed add per step on the value handed down (each
    // hand-off crosses one lane).  local_max3_offset bounds the frame too.
    constexpr bool UZ = M3;
    const int dl = UZ ? zstep + 16 : 0;
    const uint32_t D2 = rep16(dl);

    uint32_t q2[R], H2[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i0 = row_base + (uint32_t)lane * R + r;
        if constexpr (CLS) q2[r] = i0 < n ? row_selector(io.Q[0][i0], io.Q[1][i0]) : row_selector(0, 0);
        else q2[r] = i0 < n ? ((uint32_t)io.Q[0][i0] | ((uint32_t)io.Q[1][i0] << 16)) : 0u;
        H2[r] = rep16(LOCAL ? off - (int)(i0 + 1) + dl * lane : wmul(i0 + 1, init - gap));  // S(i, 0)
    }
    const uint32_t ia = row_base + (uint32_t)lane * R;  // row above the stripe
    uint32_t recv = rep16(LOCAL ? off - (int)ia + dl * lane : wmul(ia, init - gap));
    uint32_t tc2 = 0, tA = 0x01010101u, tB = 0x01010101u;
    const uint32_t nv_lane = (uint32_t)lane < nl - 1 ? R : ((uint32_t)lane == nl - 1 ? NV : 0);
    // Per-lane running values, both pairs packed, advanced once per step:
    //   Zp = local clamp base Zb = zstep*j - (ia + 1) for this lane's column j
    //   jj = j (= t - lane + 1); semi: row n holds H = S + ma*j
    // (all at t = -1 here).  Running bests are updated branch-free: the sign
    // of a saturating packed difference, spread over its half by v_perm,
    // selects the new column with one v_bfi; the value is a packed max.
    uint32_t Zp = rep16(off + zstep * (0 - lane) - (int)(ia + 1));
    int zu = off - (int)row_base - 1;  // UZ: the clamp base of row 0 in the lane frame (t = -1)
    const uint32_t ZS2 = rep16(zstep);
    uint32_t jj = rep16(-lane);
    const uint32_t MAG2 = rep16(ma - gap);
    // local: best key S - Zb = 16H - r (r = row in the stripe), -16 = no cell yet
    uint32_t bestK = rep16(-16), bestj = 0;
    uint32_t rowbest = rep16(-32768), rowbest_j = 0;  // semi: best of row n, its column

    // LST (CLS): a step's wave-uniform operands -- the two pairs' tables of the new target
    // byte and the row above -- come from one LDS read of a 64-entry list each lane fills for
    // its column every 64 steps, instead of three v_readlane and the SALU table arithmetic;
    // the DPP hand-offs then take the read registers as their lane-0 value (no v_mov)
    // (not in the code fill of blocked plans: its 32 KB of staging per block leave no room
    // for the list at 5 waves per SIMD)
    constexpr bool LST = CLS && (!BLK || kDualCk);
    uint32_t tcur[2], tnext[2];
    auto tbyte = [&](int h, uint32_t c) -> uint32_t {  // target byte of step 64c + lane
        const uint32_t k = c * 64u + (uint32_t)lane;
        return k < m ? (uint32_t)io.T[h][k] : 0u;
    };
    auto table = [&](uint32_t b) -> uint32_t { return EQ ? class_table(b, T0, TX) : mismatch_table(b); };
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        tcur[h] = LST ? tbyte(h, 0) : load_tchunk(io.T[h], m, 0, lane);
        tnext[h] = LST ? tbyte(h, 1) : load_tchunk(io.T[h], m, 1, lane);
    }
    // The row above the pass, 64 columns per chunk (lane k: column 64c + k + 1):
    // the boundary row S(0, j) in pass 0, the previous pass's bottom row after.
    // UZ: minus dl, which the hand-off adds back in lane 0 too.
    auto top_chunk = [&](uint32_t c) -> int {
        if (pass > 0)
            return (int)pk_sub((uint32_t)(io.rec_r ? dual_poll_chunk(io, m, c, lane) : load_bchunk(io.B, m, c, lane)), D2);
        const int j = (int)(c * 64u + (uint32_t)lane + 1u);
        return (int)rep16(LOCAL ? off + zstep * j - dl : (init - ma + gap) * j);
    };
    int bcur = top_chunk(0), bnext = top_chunk(1);
    if constexpr (LST) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // (after the last pass's reads)
        io.lst[lane] = make_uint4(table(tcur[0]), table(tcur[1]), (uint32_t)bcur, 0u);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    const uint32_t steps = m + nl - 1;
    uint32_t* prow0 = CIGAR ? io.ptrs[0] + (BLK ? (uint64_t)pass * io.nb * (kBlkSteps * kWave) : (uint64_t)pass * Tmax * kWave) : nullptr;
    uint32_t* prow1 = CIGAR ? io.ptrs[1] + (BLK ? (uint64_t)pass * io.nb * (kBlkSteps * kWave) : (uint64_t)pass * Tmax * kWave) : nullptr;
    // BLK: the staged kDualStage steps ending at step t (inclusive) -> their
    // place in block t / 16, [b][lane][16], of both pairs
    // CK: the bottom rows staged for the 16 steps ending at t, split by pair, and
    // at a block's end (full) all 16 rows after its last step
    auto ck_flush = [&](uint32_t t, bool full) {
        const uint32_t b = t >> 4;
        uint32_t x[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) x[q] = io.cbuf[q * kWave + lane];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t sel = h ? 0x07060302u : 0x05040100u;
            uint32_t* dr = (h ? prow1 : prow0) + ((uint64_t)b * kWave + (uint32_t)lane) * 8u;
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 2; ++q)
                *reinterpret_cast<uint4*>(dr + 4 * q) =
                    make_uint4(__builtin_amdgcn_perm(x[8 * q + 1], x[8 * q], sel), __builtin_amdgcn_perm(x[8 * q + 3], x[8 * q + 2], sel),
                               __builtin_amdgcn_perm(x[8 * q + 5], x[8 * q + 4], sel), __builtin_amdgcn_perm(x[8 * q + 7], x[8 * q + 6], sel));
            if (full) {
                uint32_t* dc = dr + (uint64_t)io.nb * kWave * 8u;
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    *reinterpret_cast<uint4*>(dc + 4 * q) =
                        make_uint4(__builtin_amdgcn_perm(H2[8 * q + 1], H2[8 * q], sel), __builtin_amdgcn_perm(H2[8 * q + 3], H2[8 * q + 2], sel),
                                   __builtin_amdgcn_perm(H2[8 * q + 5], H2[8 * q + 4], sel), __builtin_amdgcn_perm(H2[8 * q + 7], H2[8 * q + 6], sel));
            }
        }
    };
    auto blk_flush = [&](uint32_t t) {
        const uint64_t at = ((uint64_t)(t >> 4) * kWave + (uint32_t)lane) * kBlkSteps + (t & 15u & ~(uint32_t)(kDualStageL - 1));
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint32_t* dst = (h ? prow1 : prow0) + at;
            const uint32_t* src = io.cbuf + h * (kDualStageL * kWave) + lane;
#pragma unroll
            for (int q = 0; q < kDualStageL / 4; ++q) {
                // (one 16-byte piece at a time: the step loop's registers are all live here)
                __builtin_amdgcn_sched_barrier(0);
                uint4 v;
                v.x = src[(4 * q + 0) * kWave];
                v.y = src[(4 * q + 1) * kWave];
                v.z = src[(4 * q + 2) * kWave];
                v.w = src[(4 * q + 3) * kWave];
                *reinterpret_cast<uint4*>(dst + 4 * q) = v;
            }
        }
    };

    // Chunk reloads (every 256 steps: target bytes; every 64: the row above)
    // are hoisted out of the step loop by run_steps.
    auto reload = [&](uint32_t t) {
        if constexpr (LST) {
            // chunk t / 64's list (the reads of the last chunk's steps were issued before)
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            io.lst[lane] = make_uint4(table(tnext[0]), table(tnext[1]), (uint32_t)bnext, 0u);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
            for (int h = 0; h < 2; ++h) tnext[h] = tbyte(h, (t >> 6) + 1);
            bnext = top_chunk((t >> 6) + 1);
            return;
        }
        if ((t & 255u) == 0) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                tcur[h] = tnext[h];
                tnext[h] = load_tchunk(io.T[h], m, (t >> 8) + 1, lane);
            }
        }
        bcur = bnext;
        bnext = top_chunk((t >> 6) + 1);
    };
    auto step = [&](uint32_t t, auto masked_tag) {
        constexpr bool MASKED = decltype(masked_tag)::value;
        const uint32_t prev = recv;
        if constexpr (LST) {
            const uint4 e = io.lst[t & 63u];  // (one address for the wave: a broadcast)
            recv = (uint32_t)wave_shr1((int)e.z, (int)H2[R - 1]);
            tA = (uint32_t)wave_shr1((int)e.x, (int)tA);
            tB = (uint32_t)wave_shr1((int)e.y, (int)tB);
        } else {
            const uint32_t top = (uint32_t)rdlane(bcur, t & 63u);
            const uint32_t sh = (t & 3u) * 8;
            const uint32_t wa = (uint32_t)rdlane((int)tcur[0], (t >> 2) & 63u);
            const uint32_t wb = (uint32_t)rdlane((int)tcur[1], (t >> 2) & 63u);
            const uint32_t newc = ((wa >> sh) & 0xFFu) | (((wb >> sh) & 0xFFu) << 16);
            recv = (uint32_t)wave_shr1((int)top, (int)H2[R - 1]);
            if constexpr (CLS) {
                tA = (uint32_t)wave_shr1((int)table((wa >> sh) & 0xFFu), (int)tA);
                tB = (uint32_t)wave_shr1((int)table((wb >> sh) & 0xFFu), (int)tB);
            } else {
                tc2 = (uint32_t)wave_shr1((int)newc, (int)tc2);
            }
        }
        if constexpr (UZ) recv = pk_add(recv, D2);
        if constexpr (UZ) {
            zu += zstep;
        } else {
            Zp = pk_add(Zp, ZS2);
            if (MODE != kSemi) jj = pk_add(jj, ONE);  // (semi: at its use, last pass only)
        }

        const int j = (int)t - lane + 1;
        const bool active = !MASKED || (((uint32_t)lane < nl) & (j >= 1) & (j <= (int)m));
        // rows 0-7 / 8-15: bytes [I_A, I_B, D_A, D_B], row r at bit 7 - r%8
        uint32_t acc0 = 0, acc1 = 0;
        if (active) {
            auto e_of = [&](int r) {  // 0 on a match, 1 otherwise
                if constexpr (CLS) return mismatch_flags(tA, tB, q2[r]);
                else return pk_min_u16(q2[r] ^ tc2, ONE);
            };
            // the diagonal candidate of row r from the value diagonally above it
            auto diag_of = [&](int r, uint32_t dv) -> uint32_t {
                if constexpr (EQ && CLS) return dv + mismatch_flags(tA, tB, q2[r]) + KN;  // (v_add3_u32)
                else if constexpr (EQ) return pk_add(pk_mad_i16(e_of(r), KD, dv), GM);
                else return pk_mad_i16(e_of(r), KD, dv);
            };
            uint32_t dnext = diag_of(0, prev);
            uint32_t upv = recv;
            uint32_t Z = Zp;
            // M3: the clamp bases of rows 2k, 2k+1 in the halves of W[k] (op_sel picks one)
            uint32_t W[R / 2];
            if constexpr (M3) {
                // wave-uniform (SALU): halves zu - 2k, zu - 2k - 1, all >= 0 (no borrows)
                W[0] = ((uint32_t)zu & 0xFFFFu) * 0x10001u - 0x10000u;
#pragma unroll
                for (int k = 1; k < R / 2; ++k) W[k] = W[0] - 0x20002u * (uint32_t)k;
            }
            static_for<0, R>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                const uint32_t old = H2[r];
                const uint32_t diag = dnext;
                if constexpr (r + 1 < R) dnext = diag_of(r + 1, old);
                if constexpr (EQ) {
                    // left and up share the gain: max first, one add (M3 values are in
                    // [0, 0x7BFF], so the max is the integers')
                    const uint32_t lu = pk_max(old, upv);
                    const uint32_t hv = pk_max3_pos_bc<r & 1>(diag, SW ? swar_add(lu, GLk) : pk_add(lu, GL), W[r / 2]);
                    H2[r] = hv;
                    upv = hv;
                    return;
                }
                const uint32_t left = SW ? swar_add(old, GLk) : pk_add(old, GL);
                const uint32_t up = LOCAL ? (SW ? swar_add(upv, GUGk) : pk_add(upv, GUG)) : upv;
                const uint32_t m1 = pk_max(diag, left);
                uint32_t hv;
                if constexpr (M3) hv = pk_max3_pos_bc<r & 1>(m1, up, W[r / 2]);  // clamp folded in, :185
                else hv = LOCAL ? pk_max(pk_max(m1, up), Z) : pk_max(m1, up);
                if (CODES) {
                    // raw compares (D wins over I in the walk; local walks track the
                    // cost instead of reading a STOP code, ta_device.h WalkSeq)
                    const uint32_t wd = pk_sub_sat(m1, up);    // sign: up > max(diag, left)  (DELETE)
                    const uint32_t wi = pk_sub_sat(diag, left);  // sign: left > diag           (INSERT)
                    uint32_t& acc = (r < 8) ? acc0 : acc1;
                    acc = bfi(0x01010101u << (7 - (r & 7)), sign_bytes(wd, wi), acc);
                }
                H2[r] = hv;
                upv = hv;
                if (LOCAL && !M3 && r + 1 < R) Z = pk_sub(Z, ONE);
            });
            if (LOCAL) {
                // balanced trees (a serial packed-max chain stalls one cycle per link)
                uint32_t lo, hi_rows = 0;
                if constexpr (M3) {
                    lo = max3_reduce<NV>(H2);
                    if constexpr (NV != R) hi_rows = max3_reduce<R - NV>(H2 + NV);
                } else {
                    lo = tree_max<0, NV>(H2);
                    if constexpr (NV != R) hi_rows = tree_max<NV, R>(H2);
                }
                uint32_t sk = lo;
                if (NV != R) {
                    const uint32_t full = pk_max(lo, hi_rows);
                    sk = ((uint32_t)lane == nl - 1) ? lo : full;
                }
                // key = S - Zb = 16H - r per half; strict '>' keeps the first column (:186)
                if constexpr (UZ) {
                    // the column as the step t + 1 (uniform); j = t + 1 - lane at the end
                    const uint32_t key = pk_sub(sk, ((uint32_t)zu & 0xFFFFu) * 0x10001u);
                    const uint32_t msk = half_mask(pk_sub_sat(bestK, key));
                    bestj = (((t + 1u) * 0x10001u) & msk) | (bestj & ~msk);
                    bestK = pk_max(bestK, key);
                } else {
                    const uint32_t key = pk_sub(sk, Zp);
                    bestj = bfi(half_mask(pk_sub_sat(bestK, key)), jj, bestj);
                    bestK = pk_max(bestK, key);
                }
            }
            if (MODE == kSemi && (NV != R || last_pass)) {  // row n: H = S + (ma-gap)*j + gap*n, strict '>' (:271-278)
                // j of this lane's column, formed here rather than carried through
                // the passes that never read it; + gap*n is added at the end
                const uint32_t jl = rep16((int)t + 1 - lane);
                const uint32_t v = pk_mad_i16(jl, MAG2, H2[NV - 1]);
                rowbest_j = bfi(half_mask(pk_sub_sat(rowbest, v)), jl, rowbest_j);
                rowbest = pk_max(rowbest, v);
            }
            if (has_next && (uint32_t)lane == nl - 1) {
                const uint32_t bv = UZ ? pk_sub(H2[R - 1], rep16(dl * lane)) : H2[R - 1];
                if (io.rec_w)
                    __hip_atomic_store((gu64d*)(io.rec_w + j), ((uint64_t)io.tag_w << 32) | bv, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                else
                    io.B[j] = (int32_t)bv;
            }
        }
        if constexpr (CK) {
            io.cbuf[(t & 15u) * kWave + (uint32_t)lane] = H2[R - 1];  // (flushed by run_steps)
        } else if (CIGAR) {
            // per pair: [I rows 8-15, I rows 0-7, D rows 8-15, D rows 0-7] (ta_internal.h Code)
            const uint32_t cA = __builtin_amdgcn_perm(acc0, acc1, 0x06020400u);
            const uint32_t cB = __builtin_amdgcn_perm(acc0, acc1, 0x07030501u);
            if constexpr (BLK) {
                if constexpr (kDualStage == 0) {
                    const uint32_t off = (uint32_t)blk_index(0, t, (uint32_t)lane, io.nb);  // (within the pass)
                    prow0[off] = cA;
                    prow1[off] = cB;
                } else {
                    const uint32_t sl = (t & (uint32_t)(kDualStage - 1)) * kWave + (uint32_t)lane;
                    io.cbuf[sl] = cA;
                    io.cbuf[kDualStage * kWave + sl] = cB;  // (flushed by run_steps)
                }
            } else {
                // 32-bit byte offset from the uniform row base (SGPR base + VGPR offset stores)
                const uint32_t off = (t * kWave + (uint32_t)lane) * 4u;
                *(uint32_t*)((char*)prow0 + off) = cA;
                *(uint32_t*)((char*)prow1 + off) = cB;
            }
        }
    };
    const uint32_t ramp_end = min(nl - 1, steps);
    uint32_t t = 0, next_reload = 64;
    // Steps in pairs: the loop-carried DPP registers alternate between the two
    // copies instead of being copied back every step.
    auto run_steps = [&](uint32_t t_end, auto masked_tag) {
        while (t < t_end) {
            if (t == next_reload) {
                reload(t);
                next_reload += 64;
            }
            uint32_t blk = min(t_end, next_reload);
            // BLK: stop at each 16-step block end, flushing outside the step body
            // (a branch inside it costs the whole step loop spills)
            if constexpr (BLK && kDualStage) blk = min(blk, (t | (uint32_t)(kDualStage - 1)) + 1u);
            for (; t + 1 < blk; t += 2) {
                step(t, masked_tag);
                step(t + 1, masked_tag);
            }
            if (t < blk) step(t++, masked_tag);
            if constexpr (CK) {
                if ((t & 15u) == 0 || t == steps) ck_flush(t - 1, (t & 15u) == 0);
            } else if constexpr (BLK && kDualStage) {
                if ((t & (uint32_t)(kDualStageL - 1)) == 0 || t == steps) blk_flush(t - 1);
            }
        }
    };
    run_steps(ramp_end, std::true_type{});
    run_steps(m, std::false_type{});
    run_steps(steps, std::true_type{});

    DualOut out;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        PassOut& o = out.o[h];
        o = PassOut{INT_MIN, 0, 0, INT_MIN, 0, 0};
        if (LOCAL) {
            const int K = (h ? hi16(bestK) : lo16(bestK)) + 15;  // 16H + 15 - r, < 0: no cell
            const int v = ((uint32_t)lane >= nl || K < 0) ? -1 : (K >> 4);
            const int mx = wave_max(v);
            const int fl = first_lane(v == mx);
            const int Kf = rdlane(K, fl);
            const uint32_t jf = (uint32_t)rdlane((int)(h ? (bestj >> 16) : (bestj & 0xFFFFu)), fl) - (UZ ? (uint32_t)fl : 0u);
            o.h = mx;
            o.i = row_base + (uint32_t)fl * R + (uint32_t)(15 - (Kf & 15)) + 1;
            o.j = jf;
        } else if (MODE == kSemi) {
            // column m: H = S + (ma-gap)*m + gap*i; first lane, then first row (:265-270)
            int cv = INT_MIN;
            uint32_t cr = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int sv = (h ? hi16(H2[r]) : lo16(H2[r])) + gap * (int)(row_base + (uint32_t)lane * R + r + 1);
                if ((uint32_t)r < nv_lane && sv > cv) {
                    cv = sv;
                    cr = r;
                }
            }
            const int mx = wave_max(cv);
            const int fl = first_lane(cv == mx && nv_lane > 0);
            o.h = mx + (ma - gap) * (int)m;
            o.i = row_base + (uint32_t)fl * R + (uint32_t)rdlane((int)cr, fl) + 1;
            o.j = m;
            if (last_pass) {
                const int rb = rdlane(h ? hi16(rowbest) : lo16(rowbest), nl - 1);
                o.row_h = rb == -32768 ? INT_MIN : rb + gap * (int)n;  // -32768: never set
                o.row_j = (uint32_t)rdlane((int)(h ? (rowbest_j >> 16) : (rowbest_j & 0xFFFFu)), nl - 1);
            }
        } else {
            if (last_pass) {
                int hv[R];
#pragma unroll
                for (int r = 0; r < R; ++r) hv[r] = h ? hi16(H2[r]) : lo16(H2[r]);
                o.corner = rdlane(select_row<R>(hv, nrows - (nl - 1) * R - 1), nl - 1) + (ma - gap) * (int)m + gap * (int)n;
            }
        }
    }
    return out;
}

template <int MODE, bool CIGAR, bool CLS, bool BLK = false>
__device__ __forceinline__ DualOut dual_pass_nv(const FillArgs& a, const DualIo& io, uint32_t n, uint32_t m,
                                                uint32_t pass, bool last_pass, int lane) {
    const uint32_t nrows = min((uint32_t)kPassRows, n - pass * kPassRows);
    const uint32_t nv = nrows - ((nrows + kRows - 1) / kRows - 1) * kRows;
    if constexpr (MODE == kLocal) {
        // (the fills without codes use the equal-gain frame, dual_pass EQ)
        constexpr bool eq = !CIGAR || (BLK && kDualCk);
        const int off = local_max3_offset(n, m, a.match, a.mismatch, a.gap, eq);  // wave-uniform
        if (off >= 0) {
            if (nv == kRows)
                return dual_pass<MODE, CIGAR, kRows, true, CLS, BLK>(a, io, n, m, pass, last_pass, lane, off);
#define TA_NV_CASE(k) \
    case k: return dual_pass<MODE, CIGAR, k, true, CLS, BLK>(a, io, n, m, pass, last_pass, lane, off);
            switch (nv) {
                TA_NV_CASE(1) TA_NV_CASE(2) TA_NV_CASE(3) TA_NV_CASE(4) TA_NV_CASE(5) TA_NV_CASE(6) TA_NV_CASE(7)
                TA_NV_CASE(8) TA_NV_CASE(9) TA_NV_CASE(10) TA_NV_CASE(11) TA_NV_CASE(12) TA_NV_CASE(13) TA_NV_CASE(14)
                default: TA_NV_CASE(15)
            }
#undef TA_NV_CASE
        }
    }
    if (MODE == kGlobal || nv == kRows)
        return dual_pass<MODE, CIGAR, kRows, false, CLS, BLK>(a, io, n, m, pass, last_pass, lane);
#define TA_NV_CASE(k) \
    case k: return dual_pass<MODE, CIGAR, k, false, CLS, BLK>(a, io, n, m, pass, last_pass, lane);
    switch (nv) {
        TA_NV_CASE(1) TA_NV_CASE(2) TA_NV_CASE(3) TA_NV_CASE(4) TA_NV_CASE(5) TA_NV_CASE(6) TA_NV_CASE(7)
        TA_NV_CASE(8) TA_NV_CASE(9) TA_NV_CASE(10) TA_NV_CASE(11) TA_NV_CASE(12) TA_NV_CASE(13) TA_NV_CASE(14)
        default: TA_NV_CASE(15)
    }
#undef TA_NV_CASE
}

// dual_order: 2 pair ids per wave (both pairs have the same n and m and fit int16)
// 5 waves/SIMD: local+CIGAR needs ~105 VGPRs unconstrained (occupancy 4); at
// 96 the allocator spills two pass-invariant pointers, reloaded off the
// per-cell path.
#ifndef TA_DUAL_WAVES
#define TA_DUAL_WAVES 5
#endif
constexpr uint32_t kDualSkip = 0xFFFFFFFFu;  // PassOut.i of a couple handed to the int32 fill

// Chunks of multi-pass couples (a.ticket set) run one wave per (couple, pass):
// ticket t is level t / count of couple t % count; the level is the pass
// (pass-major) or, end-aligned (ta_planner.cpp order_pass_tasks), the pass
// plus the chunk's pass count minus the couple's, so the pass a wave polls
// belongs to a wave that took an earlier ticket and is running;
// each wave writes its pass's PassOut and dual_combine_kernel folds them.
// Otherwise one wave per couple sweeps its passes.
template <int MODE, bool CIGAR, bool BLK = false>
__device__ __forceinline__ void dual_fill_body(const FillArgs& a) {
    const int lane = threadIdx.x & 63;
    // BLK: code staging per wave (kDualStage steps x 64 lanes x 2 pairs)
    // (CK: the bottom row of each step, both pairs in one dword)
    constexpr int kStageDw = kDualCk ? 16 * kWave : 2 * kDualStage * kWave;
    __shared__ uint32_t cbuf_all[(BLK && kDualStage) ? kWavesPerBlock * kStageDw : 1];
    __shared__ uint4 lst_all[(BLK && !kDualCk) ? 1 : kWavesPerBlock * 64];  // (dual_pass LST)
    uint32_t widx, p_only = 0;
    const bool pipe = a.ticket != nullptr;
    if (pipe) {
        uint32_t tk = 0;
        if (lane == 0) tk = atomicAdd(a.ticket, 1u);
        tk = (uint32_t)__builtin_amdgcn_readfirstlane((int)tk);
        if (tk >= a.n_tasks) return;
        p_only = tk / a.count;  // the level; the pass once the couple's pass count is known
        widx = tk - p_only * a.count;
    } else {
        widx = wave_id();
        if (widx >= a.count) return;
    }
    uint32_t p[2];
    p[0] = a.order[2 * (a.begin + widx)];
    p[1] = a.order[2 * (a.begin + widx) + 1];
    const uint32_t n = a.qlen[p[0]], m = a.tlen[p[0]];
    const uint32_t passes = n_passes(n);
    if (pipe && a.end_aligned) {
        const uint32_t shift = a.n_tasks / a.count - passes;  // levels before this couple's pass 0
        if (p_only < shift) return;
        p_only -= shift;
    }
    if (pipe && p_only >= passes) return;
    PassOut* po = pipe ? static_cast<PassOut*>(a.pout) + 2ull * ((uint64_t)p_only * a.count + widx) : nullptr;
    DualIo io;
    io.rec_w = nullptr;
    io.rec_r = nullptr;
    io.tag_w = io.tag_r = 0;
    io.err = a.err;
    io.cbuf = cbuf_all + ((BLK && kDualStage) ? (threadIdx.x >> 6) * kStageDw : 0);
    io.lst = lst_all + (threadIdx.x >> 6) * 64;
    io.nb = blk_count(m);
    bool dash = false, qother = false;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        io.Q[h] = a.qbytes + a.qoff[p[h]];
        io.T[h] = a.tbytes + a.toff[p[h]];
        io.ptrs[h] = CIGAR ? a.ptrs + a.ptr_off[p[h]] : nullptr;
        for (uint32_t k = (uint32_t)lane; k < m; k += 64) dash |= io.T[h][k] == '-';
        for (uint32_t k = (uint32_t)lane; k < n; k += 64) {
            const uint32_t c = io.Q[h][k];
            dash |= c == '-';
            qother |= !is_acgt(c);
        }
    }
    const bool cls = __ballot(qother) == 0;  // queries of A, C, G, T only: table mismatch flags
    const bool any_dash = __ballot(dash) != 0;
    if (a.pflag && lane == 0 && (!pipe || p_only == 0)) {  // blk plans: the band walk skips handed-back pairs
        a.pflag[p[0]] = any_dash ? 1 : 0;
        a.pflag[p[1]] = any_dash ? 1 : 0;
    }
    // A '-' (a free gap step, team_alignment.cpp:25-28) changes the up gain per
    // row (query) or the left gain per step (target); those variants would cost
    // this kernel ~30 VGPRs and per-step selects for input real reads never
    // contain, so such couples go to the int32 fill (launched right after,
    // same workspace).
    if (any_dash) {
        if (lane == 0) {
            if (!pipe || p_only == 0) {
                // a self-coupled pair (p[0] == p[1], ta_planner.cpp) is handed back once:
                // two int32 waves on one pair would share its in-place boundary row
                const uint32_t k = (p[1] != p[0]) ? 2u : 1u;
                const uint32_t at = atomicAdd(a.fb_count, k);
                a.fb_list[at] = p[0];
                if (k == 2) a.fb_list[at + 1] = p[1];
            }
            if (pipe) {
                po[0].i = kDualSkip;
                po[1].i = kDualSkip;
            }
        }
        return;
    }
    io.B = (passes > 1) ? a.bnd + a.bnd_off[p[0]] : nullptr;
    if (pipe) {
        // tags never 0, unique per launch and pass (passes < 64: dual couples fit
        // int16); the host zeroes the records before each launch
        uint64_t* rec = reinterpret_cast<uint64_t*>(io.B);
        const uint64_t rb = (uint64_t)m + 1;
        io.rec_w = (p_only + 1 == passes) ? nullptr : rec + (p_only & 1u) * rb;
        io.rec_r = p_only ? rec + ((p_only - 1u) & 1u) * rb : nullptr;
        io.tag_w = a.epoch * 64u + p_only + 1u;
        io.tag_r = a.epoch * 64u + p_only;
        const bool last_pass = p_only + 1 == passes;
        const DualOut o = cls ? dual_pass_nv<MODE, CIGAR, true, BLK>(a, io, n, m, p_only, last_pass, lane)
                              : dual_pass_nv<MODE, CIGAR, false, BLK>(a, io, n, m, p_only, last_pass, lane);
        if (lane == 0) {
            po[0] = o.o[0];
            po[1] = o.o[1];
        }
        return;
    }
    int best_h[2], corner[2] = {0, 0};
    uint32_t best_i[2], best_j[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        best_h[h] = (MODE == kSemi) ? 0 : INT_MIN;
        best_i[h] = 0;
        best_j[h] = (MODE == kSemi) ? m : 0;
    }
    for (uint32_t pass = 0; pass < passes; ++pass) {
        const bool last_pass = pass + 1 == passes;
        const DualOut o = cls ? dual_pass_nv<MODE, CIGAR, true, BLK>(a, io, n, m, pass, last_pass, lane)
                              : dual_pass_nv<MODE, CIGAR, false, BLK>(a, io, n, m, pass, last_pass, lane);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (MODE != kGlobal && o.o[h].h > best_h[h]) {
                best_h[h] = o.o[h].h;
                best_i[h] = o.o[h].i;
                best_j[h] = o.o[h].j;
            }
            if (MODE == kSemi && last_pass && o.o[h].row_h > best_h[h]) {
                best_h[h] = o.o[h].row_h;
                best_i[h] = n;
                best_j[h] = o.o[h].row_j;
            }
            if (MODE == kGlobal && last_pass) corner[h] = o.o[h].corner;
        }
        if (!last_pass) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
    if (CIGAR && a.fused) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t gi = (MODE == kGlobal) ? n : best_i[h], gj = (MODE == kGlobal) ? m : best_j[h];
        if (CIGAR && a.fused) {
            uint64_t st;
            uint32_t len;
            const WalkSeq seq{io.Q[h], io.T[h], best_h[h], a.match, a.mismatch, a.gap};
            traceback_pair<MODE>(io.ptrs[h], n, m, gi, gj, a.slots + a.slot_off[p[h]], cigar_slot_bytes(n, m), lane,
                                 &st, &len, seq);
            if (lane == 0) {
                a.cigar_start[p[h]] = a.slot_off[p[h]] + st;
                a.cigar_len[p[h]] = len;
            }
        }
        if (lane == 0) {
            a.score[p[h]] = (MODE == kGlobal) ? corner[h] : best_h[h];
            a.target_begin[p[h]] = (MODE == kLocal) ? best_j[h] + 1 : 0;
            a.goal_i[p[h]] = gi;
            a.goal_j[p[h]] = gj;
        }
    }
}

template <int MODE, bool CIGAR, bool BLK = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(TA_DUAL_WAVES))) void dual_fill_kernel(FillArgs a) {
    dual_fill_body<MODE, CIGAR, BLK>(a);
}
#if defined(TA_DUAL_BLK) && TA_DUAL_CK
// the checkpoint fill under a name of its own (rocprof, profiles/*_by_kernel.json)
template <int MODE>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(TA_DUAL_WAVES))) void dual_fill_ck_kernel(FillArgs a) {
    dual_fill_body<MODE, true, true>(a);
}
#endif

inline dim3 dual_grid(uint32_t waves) { return dim3((waves + kWavesPerBlock - 1) / kWavesPerBlock); }

// After a pipelined dual fill: fold each couple's per-pass results in pass
// order (the upper pass wins ties; semi: row n after column m, :265-278;
// global: the last pass's corner).
template <int MODE>
__global__ void dual_combine_kernel(FillArgs a) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= a.count) return;
    const PassOut* po = static_cast<const PassOut*>(a.pout);
    if (po[2ull * w].i == kDualSkip) return;
    const uint32_t n = a.qlen[a.order[2 * (a.begin + w)]], m = a.tlen[a.order[2 * (a.begin + w)]];
    const uint32_t passes = n_passes(n);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t p = a.order[2 * (a.begin + w) + h];
        int best_h = (MODE == kSemi) ? 0 : INT_MIN, corner = 0;
        uint32_t best_i = 0, best_j = (MODE == kSemi) ? m : 0;
        for (uint32_t k = 0; k < passes; ++k) {
            const PassOut& o = po[2ull * ((uint64_t)k * a.count + w) + h];
            if (MODE != kGlobal && o.h > best_h) {
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
        if (h == 1 && p == a.order[2 * (a.begin + w)]) break;  // a pair coupled with itself
        a.score[p] = (MODE == kGlobal) ? corner : best_h;
        a.target_begin[p] = (MODE == kLocal) ? best_j + 1 : 0;
        a.goal_i[p] = (MODE == kGlobal) ? n : best_i;
        a.goal_j[p] = (MODE == kGlobal) ? m : best_j;
    }
}

#endif  // TA_DUAL_MODE
}  // namespace

#ifdef TA_DUAL_MODE
#if defined(TA_DUAL_BLK) && TA_DUAL_CK
template <>
hipError_t launch_dual_ck<TA_DUAL_MODE>(const FillArgs& a, hipStream_t s) {
#elif defined(TA_DUAL_BLK)
hipError_t launch_dual_blk(const FillArgs& a, hipStream_t s) {
#else
template <>
hipError_t launch_dual_mode<TA_DUAL_MODE, (TA_DUAL_CIGAR != 0)>(const FillArgs& a, hipStream_t s) {
#endif
    if (!a.count) return hipSuccess;
#if defined(TA_DUAL_BLK) && TA_DUAL_CK  // (the checkpoint layout)
    hipLaunchKernelGGL(dual_fill_ck_kernel<TA_DUAL_MODE>, dual_grid(a.ticket ? a.n_tasks : a.count), dim3(kBlock), 0, s,
                       a);
#elif defined(TA_DUAL_BLK)  // (its own translation unit: the blocked-layout local fill)
    hipLaunchKernelGGL((dual_fill_kernel<TA_DUAL_MODE, true, true>), dual_grid(a.ticket ? a.n_tasks : a.count),
                       dim3(kBlock), 0, s, a);
#else
#if TA_DUAL_CIGAR
    if (a.blk == 2) return launch_dual_ck<TA_DUAL_MODE>(a, s);  // (checkpoint plans: any mode)
#endif
#if TA_DUAL_MODE == 1 && TA_DUAL_CIGAR
    if (a.blk) return launch_dual_blk(a, s);
#endif
    hipLaunchKernelGGL((dual_fill_kernel<TA_DUAL_MODE, TA_DUAL_CIGAR != 0>), dual_grid(a.ticket ? a.n_tasks : a.count),
                       dim3(kBlock), 0, s, a);
#endif
    if (a.ticket)
        hipLaunchKernelGGL(dual_combine_kernel<TA_DUAL_MODE>, dim3((a.count + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}
#endif

}  // namespace ta
