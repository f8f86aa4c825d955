// bioinfo1_amd/csrc/ta_layout.h -- geometry of the fill and of the HBM
// workspace, shared by the kernels (hipcc) and the host planner
// (ta_planner.cpp, which also builds with plain g++ for the CPU sanitizer
// tests).  No HIP runtime types here.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define TA_HD __host__ __device__
#else
#define TA_HD
#endif

namespace ta {

// One wave64 per pair; lane l owns kRows consecutive query rows; a "pass" is
// the 64*kRows = 1024 rows one wave covers at once.
constexpr int kRows = 16;
constexpr int kWave = 64;
constexpr int kPassRows = kRows * kWave;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;

enum Mode : int { kGlobal = 0, kLocal = 1, kSemi = 2 };

// Steps of one pass over an m-column target: m + 63 (lane skew).
TA_HD inline uint32_t pass_steps(uint32_t m) { return m + kWave - 1; }
TA_HD inline uint32_t n_passes(uint32_t n) { return (n + kPassRows - 1) / kPassRows; }
// Pointer-matrix dwords for an n x m pair: passes x steps x 64 lanes.
TA_HD inline uint64_t ptr_dwords(uint32_t n, uint32_t m) {
    return (n == 0 || m == 0) ? 0 : (uint64_t)n_passes(n) * pass_steps(m) * kWave;
}
// Pass-boundary row (int32 per column) needed only when the query spans > 1 pass.
TA_HD inline uint64_t bnd_words(uint32_t n, uint32_t m) {
    return n_passes(n) > 1 ? (uint64_t)m + 1 + kWave : 0;
}
// Upper bound on any run-length CIGAR of an n x m pair (team_alignment.cpp:145-160).
TA_HD inline uint64_t cigar_slot_bytes(uint32_t n, uint32_t m) {
    return 2ull * ((uint64_t)n + m) + 2;
}

}  // namespace ta
