// bioinfo1_amd/csrc/tm_match.hip -- seed matching against the reference
// minimizer index, and the reverse-complement of the reference, on gfx950.
//
// Matching restates team_mapper.cpp:631-646 (FASTA reads) and 718-731 (FASTQ
// reads): for each deduplicated read minimizer, in order, every position of
// its hash in the forward index (ascending, the std::set order) becomes a
// forward hit (read pos, ref pos); reverse hits come from the reverse index,
// for FASTA reads only when the hash is also in the forward index.  The index
// is CSR in HBM: sorted unique hashes, offsets, positions.  Two passes over
// the minimizers (count, then write at the scanned offsets) keep the hit
// lists in exactly the reference's order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "tm_internal.h"
#include "tm_match.h"

namespace tmap {

namespace {

__device__ __forceinline__ int find_key(const uint32_t* __restrict__ keys, uint32_t nk, uint32_t h) {
    uint32_t lo = 0, hi = nk;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (keys[mid] < h) lo = mid + 1;
        else hi = mid;
    }
    return (lo < nk && keys[lo] == h) ? (int)lo : -1;
}

__global__ void count_hits_kernel(uint64_t n, const uint32_t* __restrict__ mh, DevIndexView fi, DevIndexView ri,
                                  int fastq_rules, uint32_t* __restrict__ cnt_f, uint32_t* __restrict__ cnt_r,
                                  int32_t* __restrict__ key_f, int32_t* __restrict__ key_r) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    const uint32_t h = mh[g];
    const int a = find_key(fi.keys, fi.n_keys, h);
    const int b = (fastq_rules || a >= 0) ? find_key(ri.keys, ri.n_keys, h) : -1;
    cnt_f[g] = a >= 0 ? fi.koff[a + 1] - fi.koff[a] : 0;
    cnt_r[g] = b >= 0 ? ri.koff[b + 1] - ri.koff[b] : 0;
    key_f[g] = a;
    key_r[g] = b;
}

__global__ void write_hits_kernel(uint64_t n, const uint32_t* __restrict__ mpos, DevIndexView fi, DevIndexView ri,
                                  const int32_t* __restrict__ key_f, const int32_t* __restrict__ key_r,
                                  const uint32_t* __restrict__ off_f, const uint32_t* __restrict__ off_r,
                                  uint64_t rev_base, uint32_t* __restrict__ hf, uint32_t* __restrict__ hr) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    const uint32_t p = mpos[g];
    int a = key_f[g];
    if (a >= 0) {
        uint64_t o = off_f[g];
        for (uint32_t x = fi.koff[a]; x < fi.koff[a + 1]; ++x, ++o) {
            hf[o] = p;
            hr[o] = fi.pos[x];
        }
    }
    a = key_r[g];
    if (a >= 0) {
        uint64_t o = rev_base + off_r[g];
        for (uint32_t x = ri.koff[a]; x < ri.koff[a + 1]; ++x, ++o) {
            hf[o] = p;
            hr[o] = ri.pos[x];
        }
    }
}

// list offsets: forward list of read r, then reverse lists after all forward hits
__global__ void list_off_kernel(uint32_t n_reads, const uint64_t* __restrict__ kept_off, uint64_t n_min,
                                const uint32_t* __restrict__ off_f, const uint32_t* __restrict__ off_r,
                                uint64_t tot_f, uint64_t tot_r, uint64_t* __restrict__ list_off) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r > n_reads) return;
    const uint64_t g = kept_off[r];
    list_off[r] = g < n_min ? off_f[g] : tot_f;
    list_off[n_reads + r] = tot_f + (g < n_min ? off_r[g] : tot_r);
}

__global__ void revcomp_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint64_t L) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L) return;
    const uint8_t c = in[L - 1 - i];  // team_mapper.cpp:47-63: A<->T, C<->G, others unchanged
    out[i] = c == 'A' ? 'T' : c == 'T' ? 'A' : c == 'G' ? 'C' : c == 'C' ? 'G' : c;
}

__global__ void widen_kernel(uint32_t n, const uint32_t* __restrict__ in, uint64_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i];
}

// one workgroup per segment: bytes src[start[p] .. + len[p]) -> dst[off[p] ..)
__global__ void gather_segments_kernel(const char* __restrict__ src, const uint64_t* __restrict__ start,
                                       const uint32_t* __restrict__ len, const uint64_t* __restrict__ off,
                                       char* __restrict__ dst) {
    const uint32_t p = blockIdx.x;
    const char* a = src + start[p];
    char* b = dst + off[p];
    for (uint32_t i = threadIdx.x; i < len[p]; i += blockDim.x) b[i] = a[i];
}

}  // namespace

int compact_segments(tm_context* ctx, uint32_t n, const char* d_src, const uint64_t* d_start, const uint32_t* d_len,
                     DevBuf& d_off, DevBuf& d_dst, DevBuf& tmp, uint64_t& total) {
    hipStream_t s = ctx->stream;
    total = 0;
    if (!n) return TM_OK;
    TM_HIP(ctx, d_off.reserve((n + 1) * 8ull));
    size_t tb = 0;
    TM_HIP(ctx, hipcub::DeviceScan::InclusiveSum(nullptr, tb, d_off.as<uint64_t>(), d_off.as<uint64_t>() + 1, (int)n, s));
    const size_t tb_al = (tb + 255) & ~(size_t)255;
    TM_HIP(ctx, tmp.reserve(tb_al + n * 8ull));
    uint64_t* len64 = reinterpret_cast<uint64_t*>(tmp.as<char>() + tb_al);  // scan input, apart from its output
    widen_kernel<<<(n + 255) / 256, 256, 0, s>>>(n, d_len, len64);
    TM_HIP(ctx, hipGetLastError());
    TM_HIP(ctx, hipcub::DeviceScan::InclusiveSum(tmp.p, tb, len64, d_off.as<uint64_t>() + 1, (int)n, s));
    TM_HIP(ctx, hipMemsetAsync(d_off.p, 0, 8, s));
    TM_HIP(ctx, hipMemcpyAsync(&total, d_off.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, s));
    TM_HIP(ctx, hipStreamSynchronize(s));
    TM_HIP(ctx, d_dst.reserve(total + 1));
    gather_segments_kernel<<<n, 256, 0, s>>>(d_src, d_start, d_len, d_off.as<uint64_t>(), d_dst.as<char>());
    TM_HIP(ctx, hipGetLastError());
    return TM_OK;
}

hipError_t launch_revcomp(const uint8_t* in, uint8_t* out, uint64_t L, hipStream_t s) {
    if (!L) return hipSuccess;
    revcomp_kernel<<<(uint32_t)((L + 255) / 256), 256, 0, s>>>(in, out, L);
    return hipGetLastError();
}

int match_device(tm_context* ctx, uint32_t n_reads, const MinimizerOut& m, const DevIndexView& fi,
                 const DevIndexView& ri, int fastq_rules, MatchOut& out) {
    hipStream_t s = ctx->stream;
    const uint64_t n = m.kept;
    TM_HIP(ctx, out.cnt_f.reserve(n * 4 + 4));
    TM_HIP(ctx, out.cnt_r.reserve(n * 4 + 4));
    TM_HIP(ctx, out.off_f.reserve(n * 4 + 4));
    TM_HIP(ctx, out.off_r.reserve(n * 4 + 4));
    TM_HIP(ctx, out.key_f.reserve(n * 4 + 4));
    TM_HIP(ctx, out.key_r.reserve(n * 4 + 4));
    TM_HIP(ctx, out.list_off.reserve((2ull * n_reads + 1) * 8));
    out.tot_f = out.tot_r = 0;
    if (n) {
        count_hits_kernel<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(
            n, m.khash.as<uint32_t>(), fi, ri, fastq_rules, out.cnt_f.as<uint32_t>(), out.cnt_r.as<uint32_t>(),
            out.key_f.as<int32_t>(), out.key_r.as<int32_t>());
        TM_HIP(ctx, hipGetLastError());
        size_t tmp = 0;
        TM_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, out.cnt_f.as<uint32_t>(), out.off_f.as<uint32_t>(),
                                                     (int)n, s));
        TM_HIP(ctx, out.cub_tmp.reserve(tmp));
        TM_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(out.cub_tmp.p, tmp, out.cnt_f.as<uint32_t>(),
                                                     out.off_f.as<uint32_t>(), (int)n, s));
        TM_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(out.cub_tmp.p, tmp, out.cnt_r.as<uint32_t>(),
                                                     out.off_r.as<uint32_t>(), (int)n, s));
        uint32_t last[4];
        TM_HIP(ctx, hipMemcpyAsync(&last[0], out.off_f.as<uint32_t>() + n - 1, 4, hipMemcpyDeviceToHost, s));
        TM_HIP(ctx, hipMemcpyAsync(&last[1], out.cnt_f.as<uint32_t>() + n - 1, 4, hipMemcpyDeviceToHost, s));
        TM_HIP(ctx, hipMemcpyAsync(&last[2], out.off_r.as<uint32_t>() + n - 1, 4, hipMemcpyDeviceToHost, s));
        TM_HIP(ctx, hipMemcpyAsync(&last[3], out.cnt_r.as<uint32_t>() + n - 1, 4, hipMemcpyDeviceToHost, s));
        TM_HIP(ctx, hipStreamSynchronize(s));
        out.tot_f = (uint64_t)last[0] + last[1];
        out.tot_r = (uint64_t)last[2] + last[3];
    }
    const uint64_t tot = out.tot_f + out.tot_r;
    TM_HIP(ctx, out.hf.reserve(tot * 4 + 4));
    TM_HIP(ctx, out.hr.reserve(tot * 4 + 4));
    if (n) {
        write_hits_kernel<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(
            n, m.kpos.as<uint32_t>(), fi, ri, out.key_f.as<int32_t>(), out.key_r.as<int32_t>(),
            out.off_f.as<uint32_t>(), out.off_r.as<uint32_t>(), out.tot_f, out.hf.as<uint32_t>(),
            out.hr.as<uint32_t>());
        TM_HIP(ctx, hipGetLastError());
    }
    list_off_kernel<<<(n_reads + 1 + 255) / 256, 256, 0, s>>>(n_reads, m.kept_off.as<uint64_t>(), n,
                                                              out.off_f.as<uint32_t>(), out.off_r.as<uint32_t>(),
                                                              out.tot_f, out.tot_r, out.list_off.as<uint64_t>());
    TM_HIP(ctx, hipGetLastError());
    return TM_OK;
}

}  // namespace tmap
