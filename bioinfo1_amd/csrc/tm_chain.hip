// bioinfo1_amd/csrc/tm_chain.hip -- seed chaining (FindLIS) on gfx950.
//
// Restates FindLIS (/root/reference/team_mapper.cpp:283-316) exactly:
//   lis[i]  = 1 + max lis[j] over j < i with r_i > r_j, f_i != f_j and the
//             unsigned differences f_i - f_j, r_i - r_j both below 5000
//             (so 0 < f_i - f_j < 5000 and 0 < r_i - r_j < 5000);
//   prev[i] = the smallest such j reaching that max (the reference updates
//             only on a strict improvement while j ascends);
//   chain   = walk prev from the FIRST index of the maximal lis.
// One workgroup (256 threads) per hit list.  i runs sequentially; for each i
// the 256 threads scan the candidate j's in parallel and a (lis, -j) max
// reduction picks prev[i] -- one barrier per i.  The candidate range uses the
// list's order: over the prefix where f is non-decreasing (all hits of the
// leading and full-window minimizers) every eligible j lies in the window
// f_j > f_i - 5000, tracked by a moving lower bound; hits after that prefix
// (trailing end-minimizers) scan all earlier j.  Lists up to kCapBig hits live
// in LDS (f, r, lis, prev); longer lists run the same code on global scratch.
// (kCapSmall / kCapBig: two LDS sizes, see chain_kernel.)
// The wave that owns i-1's result keeps it in registers, so iteration i needs
// no second barrier before reading lis[i-1].
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "tm_internal.h"

namespace tmap {

namespace {

constexpr int kChainBlock = 256;
constexpr int kCapSmall = 3072;  // hits per list staged in LDS: 36 KB, 4 workgroups per CU
constexpr int kCapBig = 12288;   // 144 KB, 1 workgroup per CU (gfx950: up to 160 KB per workgroup)

template <class FT, class LT>
__device__ __forceinline__ void lis_list(int n, const FT* F, const FT* R, LT* LIS, LT* PREV, uint64_t* red, int* sorted_end,
                         uint32_t* out) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // length of the prefix over which f is non-decreasing
    if (tid == 0) *sorted_end = n;
    __syncthreads();
    for (int j = tid; j + 1 < n; j += kChainBlock)
        if (F[j + 1] < F[j]) atomicMin(sorted_end, j + 1);
    __syncthreads();
    const int S = *sorted_end;
    int lo = 0;
    uint32_t best_len = 0;
    int best_i = 0;
    // element i-1 in registers (uniform)
    uint32_t pf = 0, pr = 0, plis = 0;
    for (int i = 0; i < n; ++i) {
        const uint32_t fi = F[i], ri = R[i];
        int jlo = 0;
        if (i < S) {
            while (lo < i && fi - (uint32_t)F[lo] >= 5000u) ++lo;  // f non-decreasing: later j only closer
            jlo = lo;
        }
        uint32_t bl = 0;
        int bj = -1;
        for (int j = jlo + tid; j < i - 1; j += kChainBlock) {
            const uint32_t lj = LIS[j];
            const bool ok = (fi - (uint32_t)F[j] - 1u) < 4999u && (ri - (uint32_t)R[j] - 1u) < 4999u;
            if (ok && lj > bl) {
                bl = lj;
                bj = j;
            }
        }
        if (i >= 1 && tid == 0 && i - 1 >= jlo) {  // j = i-1 from registers (smallest j wins ties in the reduce)
            const bool ok = (fi - pf - 1u) < 4999u && (ri - pr - 1u) < 4999u;
            if (ok && plis > bl) {
                bl = plis;
                bj = i - 1;
            }
        }
        // key: larger lis first, then smaller j
        unsigned long long key = bj < 0 ? 0ull : ((unsigned long long)bl << 32) | (0xffffffffu - (uint32_t)bj);
        for (int d = 32; d >= 1; d >>= 1) {
            const unsigned long long o = __shfl_xor(key, d, 64);
            key = o > key ? o : key;
        }
        uint64_t* rb = red + (i & 1) * 4;
        if (lane == 0) rb[wave] = key;
        __syncthreads();
        uint64_t k = rb[0];
        for (int q = 1; q < kChainBlock / 64; ++q) k = rb[q] > k ? rb[q] : k;
        const uint32_t li = (k ? (uint32_t)(k >> 32) : 0u) + 1u;
        const int pj = k ? (int)(0xffffffffu - (uint32_t)k) : -1;
        if (tid == 0) {
            LIS[i] = (LT)li;
            PREV[i] = (LT)(pj < 0 ? 0xffffffffu : (uint32_t)pj);
        }
        if (li > best_len) {  // std::max_element: first maximum
            best_len = li;
            best_i = i;
        }
        pf = fi;
        pr = ri;
        plis = li;
    }
    __syncthreads();
    if (tid == 0) {
        int f = best_i;
        if (n) {
            for (;;) {
                const uint32_t p = (uint32_t)PREV[f];
                if (p == (uint32_t)(LT)0xffffffffu) break;
                f = (int)p;
            }
        }
        out[0] = n ? best_len : 0;
        out[1] = n ? (uint32_t)F[f] : 0;
        out[2] = n ? (uint32_t)R[f] : 0;
        out[3] = n ? (uint32_t)F[best_i] : 0;
        out[4] = n ? (uint32_t)R[best_i] : 0;
    }
}

// Lists with lo < n <= CAP run in LDS; with CAP == kCapBig the kernel also
// takes every longer list (global scratch).  Two instantiations: a small-LDS
// one (4 workgroups per CU) for the common lists and a large-LDS one for the
// long reads' lists.
template <int CAP>
__global__ __launch_bounds__(kChainBlock) void chain_kernel(uint32_t n_lists, int lo_excl,
                                                            const uint64_t* __restrict__ off,
                                                            const uint32_t* __restrict__ f,
                                                            const uint32_t* __restrict__ r,
                                                            uint32_t* __restrict__ g_lis, uint32_t* __restrict__ g_prev,
                                                            uint32_t* __restrict__ out) {
    __shared__ uint32_t sF[CAP], sR[CAP];
    __shared__ uint16_t sL[CAP], sP[CAP];
    __shared__ uint64_t red[8];
    __shared__ int sorted_end;
    const uint32_t l = blockIdx.x;
    if (l >= n_lists) return;
    const uint64_t b = off[l];
    const int n = (int)(off[l + 1] - b);
    if (n <= lo_excl || (CAP != kCapBig && n > CAP)) return;  // another instantiation's list
    if (n <= CAP) {
        for (int j = threadIdx.x; j < n; j += kChainBlock) {
            sF[j] = f[b + j];
            sR[j] = r[b + j];
        }
        __syncthreads();
        lis_list<uint32_t, uint16_t>(n, sF, sR, sL, sP, red, &sorted_end, out + 5ull * l);
    } else {
        lis_list<uint32_t, uint32_t>(n, f + b, r + b, g_lis + b, g_prev + b, red, &sorted_end, out + 5ull * l);
    }
}

}  // namespace

int chain_device(tm_context* ctx, uint32_t n_lists, const uint64_t* d_off, uint64_t total_hits, const uint32_t* d_f,
                 const uint32_t* d_r, uint32_t* d_out) {
    if (!n_lists) return TM_OK;
    TM_HIP(ctx, ctx->c_lis.reserve(total_hits * 4 + 4));
    TM_HIP(ctx, ctx->c_prev.reserve(total_hits * 4 + 4));
    chain_kernel<kCapSmall><<<n_lists, kChainBlock, 0, ctx->stream>>>(
        n_lists, -1, d_off, d_f, d_r, ctx->c_lis.as<uint32_t>(), ctx->c_prev.as<uint32_t>(), d_out);
    TM_HIP(ctx, hipGetLastError());
    chain_kernel<kCapBig><<<n_lists, kChainBlock, 0, ctx->stream>>>(
        n_lists, kCapSmall, d_off, d_f, d_r, ctx->c_lis.as<uint32_t>(), ctx->c_prev.as<uint32_t>(), d_out);
    TM_HIP(ctx, hipGetLastError());
    return TM_OK;
}

}  // namespace tmap

extern "C" int tm_chain_batch(tm_context* ctx, uint32_t n_lists, const uint64_t* off, const uint32_t* fpos,
                              const uint32_t* rpos, uint32_t* chain_len, uint32_t* first_f, uint32_t* first_r,
                              uint32_t* last_f, uint32_t* last_r) {
    if (!ctx) return TM_ERR_ARG;
    if (!n_lists) return TM_OK;
    if (!off || !chain_len || !first_f || !first_r || !last_f || !last_r)
        return tmap::fail(ctx, TM_ERR_ARG, "null argument");
    const uint64_t total = off[n_lists];
    if (total && (!fpos || !rpos)) return tmap::fail(ctx, TM_ERR_ARG, "null hits");
    for (uint32_t l = 0; l < n_lists; ++l)
        if (off[l + 1] < off[l]) return tmap::fail(ctx, TM_ERR_ARG, "offsets not ascending");
    TM_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    TM_HIP(ctx, ctx->c_off.reserve((n_lists + 1) * 8ull));
    TM_HIP(ctx, ctx->c_f.reserve(total * 4 + 4));
    TM_HIP(ctx, ctx->c_r.reserve(total * 4 + 4));
    TM_HIP(ctx, ctx->c_out.reserve(n_lists * 20ull));
    TM_HIP(ctx, hipMemcpyAsync(ctx->c_off.p, off, (n_lists + 1) * 8ull, hipMemcpyHostToDevice, s));
    if (total) {
        TM_HIP(ctx, hipMemcpyAsync(ctx->c_f.p, fpos, total * 4, hipMemcpyHostToDevice, s));
        TM_HIP(ctx, hipMemcpyAsync(ctx->c_r.p, rpos, total * 4, hipMemcpyHostToDevice, s));
    }
    if (int rc = tmap::chain_device(ctx, n_lists, ctx->c_off.as<uint64_t>(), total, ctx->c_f.as<uint32_t>(),
                                  ctx->c_r.as<uint32_t>(), ctx->c_out.as<uint32_t>()))
        return rc;
    std::vector<uint32_t> o(5ull * n_lists);
    TM_HIP(ctx, hipMemcpyAsync(o.data(), ctx->c_out.p, n_lists * 20ull, hipMemcpyDeviceToHost, s));
    TM_HIP(ctx, hipStreamSynchronize(s));
    for (uint32_t l = 0; l < n_lists; ++l) {
        chain_len[l] = o[5 * l];
        first_f[l] = o[5 * l + 1];
        first_r[l] = o[5 * l + 2];
        last_f[l] = o[5 * l + 3];
        last_r[l] = o[5 * l + 4];
    }
    return TM_OK;
}
