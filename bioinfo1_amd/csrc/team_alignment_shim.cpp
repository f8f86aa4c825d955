// bioinfo1_amd/csrc/team_alignment_shim.cpp -- the drop-in team::Align.
//
// Exports the reference's C++ entry point with the identical signature and
// mangled name (include/team_alignment.hpp; reference
// team_alignment.hpp:14-23 / team_alignment.cpp:49-56) so team_mapper.cpp's
// four call sites (team_mapper.cpp:666, 674, 755, 763) link unchanged.  The
// call is forwarded as a one-pair batch to the extern "C" ABI, which runs the
// HIP kernels; there is no CPU fallback.  Error behaviour mirrors the
// reference: std::invalid_argument with the same two messages; a missing or
// failing GPU raises std::runtime_error (the mapper's catch (std::exception&)
// at team_mapper.cpp:680-683 handles both).
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/team_align_c.h"
#include "../../include/team_alignment.hpp"

namespace {

// One context (device stream + grow-only device and pinned staging buffers)
// per calling thread: Align is re-entrant in the reference and the mapper
// calls it from OpenMP threads.  After the first calls a call allocates
// nothing: one pinned upload, the fill kernel (which walks its own pair),
// one download, one synchronisation (ta_host_batch.h).
struct ThreadCtx {
    ta_context* ctx = nullptr;
    std::vector<char> arena;  // CIGAR bytes of the last call (grow-only)
    ~ThreadCtx() { ta_context_destroy(ctx); }
};

thread_local ThreadCtx tc;

ta_context* thread_context() {
    if (!tc.ctx) {
        int r = ta_context_create(0, &tc.ctx);
        if (r != TA_OK) throw std::runtime_error("team::Align: no usable gfx950 GPU (" + std::string(ta_status_string(r)) + ")");
    }
    return tc.ctx;
}

}  // namespace

namespace team {

int Align(const char* query, unsigned int query_len, const char* target, unsigned int target_len,
          AlignmentType type, int match, int mismatch, int gap, std::string* cigar, unsigned int* target_begin) {
    const int t = static_cast<int>(type);
    if (t != TA_GLOBAL && t != TA_LOCAL && t != TA_SEMI_GLOBAL)
        throw std::invalid_argument("Unknown AlignmentType provided.");  // team_alignment.cpp:73
    ta_context* ctx = thread_context();
    const uint64_t qoff = 0, toff = 0;
    const uint32_t ql = query_len, tl = target_len;
    int32_t score = 0;
    uint32_t tb = 0;
    std::vector<char>& arena = tc.arena;
    if (cigar && arena.size() < ta_cigar_slot_bytes(ql, tl)) arena.resize(ta_cigar_slot_bytes(ql, tl));
    uint64_t coff = 0;
    uint32_t clen = 0;
    int r = ta_align_batch(ctx, 1, query, &qoff, &ql, target, &toff, &tl, t, match, mismatch, gap, cigar != nullptr,
                           &score, &tb, arena.data(), arena.size(), &coff, &clen);
    if (r == TA_ERR_BAD_TYPE || r == TA_ERR_CIGAR) throw std::invalid_argument(ta_status_string(r));
    if (r != TA_OK)
        throw std::runtime_error(std::string("team::Align: ") + ta_status_string(r) + ": " + ta_last_error(ctx));
    if (target_begin) *target_begin = tb;
    if (cigar) cigar->assign(arena.data() + coff, clen);  // assigned, not appended (:160)
    return score;
}

}  // namespace team
