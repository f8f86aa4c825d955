// bioinfo1_amd/csrc/ta_packed.h -- packed two-pair (2 x int16 per dword)
// helpers shared by the dual fill (ta_dual.hip) and the flexible dual fill
// (ta_flex.hip): v_pk_* arithmetic through clang vector builtins, the
// sign-byte pointer-code packing and the branch-free select.
#pragma once

#include "ta_device.h"

namespace ta {
namespace {

__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) {
    typedef short s2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(s2, a) + __builtin_bit_cast(s2, b));
}
__device__ __forceinline__ uint32_t pk_sub(uint32_t a, uint32_t b) {
    typedef short s2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(s2, a) - __builtin_bit_cast(s2, b));
}
__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b) {
    typedef short s2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s2, a), __builtin_bit_cast(s2, b)));
}
// max over v[B..E) as a balanced tree
template <int B, int E>
__device__ __forceinline__ uint32_t tree_max(const uint32_t* v) {
    if constexpr (E - B == 1) return v[B];
    else return pk_max(tree_max<B, (B + E) / 2>(v), tree_max<(B + E) / 2, E>(v));
}
// max of three packed values whose halves all lie in [0, 0x7BFF]: read as
// f16 bit patterns they are finite non-negative numbers ordered like the
// integers, and clang fuses the nested maxima into one v_pk_maximum3_f16
// (gfx950; there is no packed i16 max3).  The result is one of the inputs'
// bit patterns.
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_max3_pos(uint32_t a, uint32_t b, uint32_t c) {
    const h2v x = __builtin_bit_cast(h2v, a), y = __builtin_bit_cast(h2v, b), z = __builtin_bit_cast(h2v, c);
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_maximum(__builtin_elementwise_maximum(x, y), z));
}
// pk_max3_pos(a, b, one half of w in both halves): the broadcast folds into
// the instruction's op_sel (two rows' clamp bases share one register)
template <int HALF>
__device__ __forceinline__ uint32_t pk_max3_pos_bc(uint32_t a, uint32_t b, uint32_t w) {
    const h2v x = __builtin_bit_cast(h2v, a), y = __builtin_bit_cast(h2v, b), z = __builtin_bit_cast(h2v, w);
    const h2v zz = __builtin_shufflevector(z, z, HALF, HALF);
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_maximum(__builtin_elementwise_maximum(x, y), zz));
}
// max over v[0..N) of such values: triples per level, ceil((N-1)/2) instructions
template <int N>
__device__ __forceinline__ uint32_t max3_reduce(const uint32_t* v) {
    if constexpr (N == 1) {
        return v[0];
    } else if constexpr (N == 2) {
        return pk_max(v[0], v[1]);
    } else {
        constexpr int M = (N + 2) / 3;
        uint32_t w[M];
#pragma unroll
        for (int k = 0; k < N / 3; ++k) w[k] = pk_max3_pos(v[3 * k], v[3 * k + 1], v[3 * k + 2]);
        if constexpr (N % 3 == 1) w[M - 1] = v[N - 1];
        if constexpr (N % 3 == 2) w[M - 1] = pk_max(v[N - 2], v[N - 1]);
        return max3_reduce<M>(w);
    }
}
// Mismatch flags from a per-step table, for queries of the bytes A, C, G, T
// only (the reference compares raw bytes; any other target byte can then
// match no query byte).  class: 'A' 0, 'C' 1, 'T' 2, 'G' 3 = (c >> 1) & 3.
// The table of target byte c has byte k = 0 if c is the class-k letter,
// else 1; row r's selector picks pair A's flag from table A (bytes 0-3),
// pair B's from table B (4-7) and zeros above them: one v_perm_b32 per row
// instead of xor + min.  The tables are built on the SALU from the
// wave-uniform new target byte and ride the lane skew with DPP.
__device__ __forceinline__ bool is_acgt(uint32_t c) {
    return c == ((0x47544341u >> (8u * ((c >> 1) & 3u))) & 0xFFu);
}
// The general table: byte k = mis, or hit when c is the class-k letter, as
// t0 = mis * 0x01010101 and x = hit ^ mis (the local equal-gain frame's gain
// bytes 16 s - 2 + 128, ta_layout.h local_eq_gains).
__device__ __forceinline__ uint32_t class_table(uint32_t c, uint32_t t0, uint32_t x) {
    // (a select of the bits, not a bool shifted: keeps the whole table on the SALU)
    const uint32_t sh = 8u * ((c >> 1) & 3u);
    return t0 ^ ((c == ((0x47544341u >> sh) & 0xFFu)) ? x << sh : 0u);
}
__device__ __forceinline__ uint32_t mismatch_table(uint32_t c) { return class_table(c, 0x01010101u, 1u); }
__device__ __forceinline__ uint32_t row_selector(uint32_t qa, uint32_t qb) {
    return ((qa >> 1) & 3u) | 0x0C00u | ((4u + ((qb >> 1) & 3u)) << 16) | 0x0C000000u;
}
__device__ __forceinline__ uint32_t mismatch_flags(uint32_t ta, uint32_t tb, uint32_t sel) {
    return __builtin_amdgcn_perm(tb, ta, sel);
}
// Packed helpers through clang vector builtins (inline asm costs an s_nop:
// the hazard recognizer cannot see into it).  pk_min_u16 must get a
// non-constant operand: min(x, 1) with a literal 1 is expanded into compares.
typedef unsigned short u2 __attribute__((ext_vector_type(2)));
typedef short s2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u2, a), __builtin_bit_cast(u2, b)));
}
// a * b + c per half (v_pk_mad_u16: the low 16 bits are the same as i16)
__device__ __forceinline__ uint32_t pk_mad_i16(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(s2v, a) * __builtin_bit_cast(s2v, b) + __builtin_bit_cast(s2v, c));
}
// a - b per half, saturating (v_pk_sub_i16 clamp): its sign bits (15, 31) are the per-half a < b
__device__ __forceinline__ uint32_t pk_sub_sat(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(s2v, a), __builtin_bit_cast(s2v, b)));
}
// Pointer bits without lane masks: the sign bits of two compare words are
// spread to whole bytes by v_perm_b32 (selectors 8..11 replicate the sign of
// bytes 1, 3, 5, 7), giving [I_A, I_B, D_A, D_B] as 0x00/0xFF bytes, and one
// bit-insert (v_bitop3_b32 on gfx950) drops them into bit (7 - r%8) of the
// row group's accumulator.
constexpr uint32_t kSignBytes = 0x0B0A0908u;
__device__ __forceinline__ uint32_t sign_bytes(uint32_t dword_d, uint32_t dword_i) {
    return __builtin_amdgcn_perm(dword_d, dword_i, kSignBytes);
}
// Bit select (a & mask) | (b & ~mask).  TA_BITOP3 (default): v_bitop3_b32
// (gfx950, truth table 0xCA), which issues at ~2.5 cycles per wave64
// instruction where v_bfi_b32 takes ~4.2 (profiles/r03_valu_rates.txt).  Not
// the C++ form: from that hipcc builds and/or trees over all 8 rows of a group,
// which keeps their sign bytes live (spills at 5 waves).
#ifndef TA_BITOP3
#define TA_BITOP3 1
#endif
__device__ __forceinline__ uint32_t bfi(uint32_t mask, uint32_t a, uint32_t b) {
    uint32_t r;
    // (inline asm, not __builtin_amdgcn_bitop3_b32: hipcc merges the builtin's
    // chains into trees like the C++ form's, 15,988 spilled VGPRs in the dual fill)
#if TA_BITOP3
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(r) : "s"(mask), "v"(a), "v"(b));
#else
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(mask), "v"(a), "v"(b));
#endif
    return r;
}
// Packed add of a per-half constant v through ONE 32-bit add (v_add_u32:
// ~2.9 cycles per wave64 instruction against ~4.4 for v_pk_add_u16), exact
// when every half of a and of the result lies in [0, 0x10000): then the low
// half never borrows from or carries into the high one.  k = swar_k(v) =
// v * 65537 (the low half's wrap-around carry pre-subtracted from the high
// half when v < 0).  Used where values are range-proved non-negative int16
// (ta_layout.h local_max3_offset).
__device__ __forceinline__ uint32_t swar_k(int v) { return (uint32_t)(v * 65537); }
__device__ __forceinline__ uint32_t swar_add(uint32_t a, uint32_t k) { return a + k; }

// each half shifted right by 4 (v_pk_lshrrev_b16)
__device__ __forceinline__ uint32_t pk_lshr4(uint32_t a) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u2, a) >> (u2){4, 4});
}
// (a & m) | (b & ~m) with a per-lane mask (bfi above takes a wave-uniform one)
__device__ __forceinline__ uint32_t vsel(uint32_t m, uint32_t a, uint32_t b) { return (a & m) | (b & ~m); }

// 0xFFFF in each half whose sign bit (15 / 31) is set
__device__ __forceinline__ uint32_t half_mask(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x09090808u); }
__device__ __forceinline__ uint32_t rep16(int v) { return ((uint32_t)v & 0xFFFFu) | ((uint32_t)v << 16); }
__device__ __forceinline__ int lo16(uint32_t x) { return (int)(int16_t)(x & 0xFFFFu); }
__device__ __forceinline__ int hi16(uint32_t x) { return (int)(int16_t)(x >> 16); }


}  // namespace
}  // namespace ta
