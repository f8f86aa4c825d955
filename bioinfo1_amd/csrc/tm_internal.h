// bioinfo1_amd/csrc/tm_internal.h -- shared pieces of the mapper stages
// (include/team_mapper_c.h): the context, device buffers, minimizer entry
// geometry, and the device-level stage functions the driver chains together.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/team_align_c.h"
#include "../../include/team_mapper_c.h"

namespace tmap {

constexpr uint32_t kMaxK = 15;
constexpr uint32_t kMaxW = 64;
constexpr int kMinTile = 1024;  // minimizer entries per workgroup
constexpr int kMinBlock = 256;
constexpr int kStages = 8;  // tm_stage_times: upload, minimizers, matching, chaining, windows+plan, align, results, total

// Entries KMER::Minimize emits for a sequence of length L
// (team_minimizers.cpp:146-222): w-1 leading end-minimizers (the reference
// does not check L there), one per full window (i = w-1 .. L-k), and one
// trailing end-minimizer per u in [k, w+k-2] with u <= L.
__host__ __device__ inline uint32_t n_lead(uint32_t L, uint32_t k, uint32_t w) { return (w == 0 || L < k) ? 0 : w - 1; }
__host__ __device__ inline uint32_t n_full(uint32_t L, uint32_t k, uint32_t w) {
    return (w == 0 || L < k || L - k + 1 < w) ? 0 : L - k + 1 - (w - 1);
}
__host__ __device__ inline uint32_t n_tail(uint32_t L, uint32_t k, uint32_t w) {
    if (w == 0 || L < k) return 0;
    return (w - 1 < L - k + 1) ? w - 1 : L - k + 1;
}
__host__ __device__ inline uint64_t n_entries(uint32_t L, uint32_t k, uint32_t w) {
    return (uint64_t)n_lead(L, k, w) + n_full(L, k, w) + n_tail(L, k, w);
}

// Grow-only device allocation.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t bytes);
    void release();
    template <class T>
    T* as() const {
        return static_cast<T*>(p);
    }
};

struct MinTile {
    uint32_t seq;    // sequence id
    uint32_t first;  // first entry of the tile (entry index within the sequence)
};

// Minimizers of a device-resident batch.  Results stay on the device:
//   full lists  : hash/pos at entry_off[s] .. entry_off[s+1] (every emitted entry)
//   dedup lists : khash/kpos at kept_off[s] .. kept_off[s+1] (first occurrences)
struct MinimizerOut {
    DevBuf entry_off, tiles, hash, pos, keep, scan, kept_off, khash, kpos, cub_tmp;
    uint64_t total = 0, kept = 0;
    std::vector<uint64_t> h_entry_off;
};

// One strand of the reference index in HBM (CSR): keys[n_keys] sorted unique
// hashes, koff[n_keys+1], pos[koff[n_keys]] ascending per key (1-based).
struct DevIndexView {
    const uint32_t* keys;
    const uint32_t* koff;
    const uint32_t* pos;
    uint32_t n_keys;
};

// Seed hits: hf/hr[list_off[l] .. list_off[l+1]); l < n_reads forward lists,
// then the reverse lists.
struct MatchOut {
    DevBuf cnt_f, cnt_r, off_f, off_r, key_f, key_r, hf, hr, list_off, cub_tmp;
    uint64_t tot_f = 0, tot_r = 0;
};

}  // namespace tmap

struct tm_context {
    int device = 0;
    hipStream_t stream = nullptr;
    ta_context* ta = nullptr;  // alignment batches (libteam_alignment) on the same device
    std::string last_error;
    tmap::DevBuf bytes, off, len;  // staging for the host-memory entry points
    tmap::MinimizerOut mins;
    tmap::MatchOut match;
    tmap::DevBuf c_off, c_f, c_r, c_out, c_prev, c_lis;
    // tm_map_batch
    tmap::DevBuf m_qoff, m_toff, m_score, m_tb, m_slots, m_cstart, m_clen, m_coff, m_cdst;
    double stage_ms[tmap::kStages] = {};
    uint64_t stage_cells = 0;
    uint64_t plan_stats[5] = {};  // tm_align_plan_stats
};

namespace tmap {

int fail(tm_context* ctx, int code, const std::string& msg);

#define TM_HIP(ctx, expr)                                                                                     \
    do {                                                                                                      \
        hipError_t e_ = (expr);                                                                               \
        if (e_ != hipSuccess) return ::tmap::fail((ctx), TM_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// Stage 1 (tm_minimizers.hip): minimizers of n sequences already on the device
// (d_bytes + d_off/d_len), host copy of the lengths in h_len.
int minimize_device(tm_context* ctx, uint32_t n, const uint8_t* d_bytes, const uint64_t* d_off, const uint32_t* d_len,
                    const uint32_t* h_len, uint32_t k, uint32_t w, bool dedup, MinimizerOut& out);

// Stage 3 (tm_chain.hip): FindLIS over n lists; per list 5 uint32 outputs
// (len, first f, first r, last f, last r) at d_out[5*l ..].
int chain_device(tm_context* ctx, uint32_t n_lists, const uint64_t* d_off, uint64_t total_hits, const uint32_t* d_f,
                 const uint32_t* d_r, uint32_t* d_out);

}  // namespace tmap
