// scripts/exp/ubench/valu_rates.hip -- cycles per wave-instruction for the VALU
// ops the DP kernels use (MI355X).  Each kernel runs 8 independent chains of
// one op per wave, 8 waves per SIMD, and reports the chip-wide rate.
// Build + run on the GPU box: hipcc -O3 --offload-arch=gfx950 valu_rates.hip -o vr && ./vr
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHAINS 8
#define ITERS 4096
#define OPK(name, asmop)                                                                  \
    __global__ void name(uint32_t* out, uint32_t seed) {                                  \
        uint32_t v[CHAINS];                                                               \
        for (int c = 0; c < CHAINS; ++c) v[c] = seed + threadIdx.x * 7u + c;             \
        uint32_t k = seed | 0x00010001u;                                                  \
        for (int i = 0; i < ITERS; ++i) {                                                 \
            _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) asm volatile(asmop : "+v"(v[c]) : "v"(k)); \
        }                                                                                 \
        uint32_t s = 0;                                                                   \
        for (int c = 0; c < CHAINS; ++c) s ^= v[c];                                       \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                   \
    }
// the same with SGPR clobbers (ops that write an SGPR or read a fixed SGPR pair)
#define OPKS(name, asmop)                                                                 \
    __global__ void name(uint32_t* out, uint32_t seed) {                                  \
        uint32_t v[CHAINS];                                                               \
        for (int c = 0; c < CHAINS; ++c) v[c] = seed + threadIdx.x * 7u + c;             \
        uint32_t k = seed | 0x00010001u;                                                  \
        asm volatile("s_mov_b64 s[0:1], 0x5555" ::: "s0", "s1");                         \
        for (int i = 0; i < ITERS; ++i) {                                                 \
            _Pragma("unroll") for (int c = 0; c < CHAINS; ++c)                            \
                asm volatile(asmop : "+v"(v[c]) : "v"(k) : "s0", "s1", "s2", "vcc");      \
        }                                                                                 \
        uint32_t s = 0;                                                                   \
        for (int c = 0; c < CHAINS; ++c) s ^= v[c];                                       \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                   \
    }
OPK(k_add_u32, "v_add_u32 %0, %0, %1")
OPK(k_max_i32, "v_max_i32 %0, %0, %1")
OPK(k_max3_i32, "v_max3_i32 %0, %0, %1, %0")
OPK(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")
OPK(k_pk_max_i16, "v_pk_max_i16 %0, %0, %1")
OPK(k_pk_min_u16, "v_pk_min_u16 %0, %0, %1")
OPK(k_pk_mad_i16, "v_pk_mad_i16 %0, %0, %1, %0")
OPK(k_perm, "v_perm_b32 %0, %0, %1, %0")
OPK(k_xor, "v_xor_b32 %0, %0, %1")
OPKS(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
OPKS(k_addc, "v_addc_co_u32 %0, vcc, %0, %0, vcc")
OPK(k_bfe, "v_bfe_u32 %0, %0, %1, 2")
OPK(k_lshl_or, "v_lshl_or_b32 %0, %0, 1, %1")
OPK(k_pk_fma_f32_probe, "v_pk_add_u16 %0, %0, %1 op_sel_hi:[1,1]")
// the dual fill's remaining per-cell ops (ta_dual.hip): saturating packed subtract,
// f16 three-input maximum on int16 bit patterns, bit-field insert, packed mad, DPP hand-off
OPK(k_pk_sub_i16_clamp, "v_pk_sub_i16 %0, %0, %1 clamp")
OPK(k_pk_max3_f16, "v_pk_maximum3_f16 %0, %0, %1, %0")
OPK(k_bfi, "v_bfi_b32 %0, %1, %0, %1")
OPK(k_pk_mad_u16, "v_pk_mad_u16 %0, %0, %1, %0")
OPK(k_pk_max_i16_opsel, "v_pk_max_i16 %0, %0, %1 op_sel:[0,1] op_sel_hi:[1,1]")
OPK(k_mov, "v_mov_b32 %0, %1\n v_add_u32 %0, %0, %1")
OPK(k_dpp_shr, "v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf")
OPK(k_fma_f32, "v_fma_f32 %0, %0, %1, %0")
// the rest of the fills' / walks' opcodes (scripts/valu_roof.py weights them by the census)
OPK(k_or, "v_or_b32 %0, %0, %1")
OPK(k_and, "v_and_b32 %0, %0, %1")
OPK(k_lshlrev, "v_lshlrev_b32 %0, 3, %0")
OPK(k_lshrrev, "v_lshrrev_b32 %0, 3, %0")
OPK(k_sub, "v_sub_u32 %0, %0, %1")
OPK(k_min_u32, "v_min_u32 %0, %0, %1")
OPK(k_max_u32, "v_max_u32 %0, %0, %1")
OPK(k_bitop3, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0x6c")
OPK(k_and_or, "v_and_or_b32 %0, %0, %1, %0")
OPK(k_or3, "v_or3_b32 %0, %0, %1, %0")
OPK(k_add3, "v_add3_u32 %0, %0, %1, %0")
OPK(k_xad, "v_xad_u32 %0, %0, %1, %0")
OPK(k_lshl_add, "v_lshl_add_u32 %0, %0, 1, %1")
OPK(k_mad_u24, "v_mad_u32_u24 %0, %0, %1, %0")
OPK(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
OPKS(k_cndmask_s, "v_cndmask_b32_e64 %0, %0, %1, s[0:1]")
OPKS(k_cmp_cnd, "v_cmp_gt_u32_e64 s[0:1], %0, %1\n v_cndmask_b32_e64 %0, %0, %1, s[0:1]")
OPKS(k_readlane, "v_readlane_b32 s2, %0, 5\n v_add_u32 %0, s2, %0")
OPK(k_pk_lshl, "v_pk_lshlrev_b16 %0, 1, %0")
OPK(k_pk_sub_u16, "v_pk_sub_u16 %0, %0, %1")
OPK(k_sdwa_add, "v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD")
// mixed issue: one 32-bit + one packed 16-bit op (counted as 2 wave-instructions below)
OPK(k_mix, "v_add_u32 %0, %0, %1\n v_pk_add_u16 %0, %0, %1")

int main() {
    int dev = 0;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, dev);
    const int cus = p.multiProcessorCount;
    const int waves_per_simd = 8, block = 256;
    const int blocks = cus * 4 * waves_per_simd * 64 / block;
    uint32_t* out;
    hipMalloc(&out, (size_t)blocks * block * 4);
    struct K { const char* n; void (*f)(uint32_t*, uint32_t); } ks[] = {
        {"v_add_u32", k_add_u32}, {"v_max_i32", k_max_i32}, {"v_max3_i32", k_max3_i32},
        {"v_pk_add_u16", k_pk_add_u16}, {"v_pk_max_i16", k_pk_max_i16}, {"v_pk_min_u16", k_pk_min_u16},
        {"v_pk_mad_i16", k_pk_mad_i16}, {"v_perm_b32", k_perm}, {"v_xor_b32", k_xor},
        {"v_cndmask_b32", k_cndmask}, {"v_addc_co_u32", k_addc}, {"v_bfe_u32", k_bfe},
        {"v_lshl_or_b32", k_lshl_or}, {"v_pk_add_u16(opsel)", k_pk_fma_f32_probe},
        {"v_pk_sub_i16 clamp", k_pk_sub_i16_clamp}, {"v_pk_maximum3_f16", k_pk_max3_f16}, {"v_bfi_b32", k_bfi},
        {"v_pk_mad_u16", k_pk_mad_u16}, {"v_pk_max_i16(op_sel)", k_pk_max_i16_opsel},
        {"v_mov_b32+v_add_u32 (x2)", k_mov}, {"v_mov_b32_dpp wave_shr:1", k_dpp_shr}, {"v_fma_f32", k_fma_f32},
        {"v_add_u32+v_pk_add_u16 (x2)", k_mix},
        {"v_or_b32", k_or}, {"v_and_b32", k_and}, {"v_lshlrev_b32", k_lshlrev}, {"v_lshrrev_b32", k_lshrrev},
        {"v_sub_u32", k_sub}, {"v_min_u32", k_min_u32}, {"v_max_u32", k_max_u32}, {"v_bitop3_b32", k_bitop3},
        {"v_and_or_b32", k_and_or}, {"v_or3_b32", k_or3}, {"v_add3_u32", k_add3}, {"v_xad_u32", k_xad},
        {"v_lshl_add_u32", k_lshl_add}, {"v_mad_u32_u24", k_mad_u24}, {"v_mul_lo_u32", k_mul_lo},
        {"v_cndmask_b32_e64", k_cndmask_s}, {"v_cmp_gt_u32+v_cndmask (x2)", k_cmp_cnd},
        {"v_readlane_b32+v_add_u32 (x2)", k_readlane}, {"v_pk_lshlrev_b16", k_pk_lshl},
        {"v_pk_sub_u16", k_pk_sub_u16}, {"v_add_u32_sdwa", k_sdwa_add}};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    printf("CUs %d, clock %d kHz, %d waves/SIMD\n", cus, p.clockRate, waves_per_simd);
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(block), 0, 0, out, 1u);
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(block), 0, 0, out, (uint32_t)r);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double per = (k.f == k_mov || k.f == k_mix || k.f == k_cmp_cnd || k.f == k_readlane) ? 2.0 : 1.0;
        const double winstr = per * 5.0 * blocks * (block / 64) * (double)ITERS * CHAINS;
        const double per_simd_per_s = winstr / (ms * 1e-3) / (cus * 4);
        printf("%-22s %8.3f ms  %.3f Gwave-instr/s/SIMD  => %.2f cycles/wave-instr at 2.4 GHz\n", k.n, ms,
               per_simd_per_s / 1e9, 2.4e9 / per_simd_per_s);
    }
    return 0;
}
