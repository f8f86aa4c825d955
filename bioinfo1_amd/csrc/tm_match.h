// bioinfo1_amd/csrc/tm_match.h -- device views of the reference minimizer
// index and the seed-matching stage (tm_match.hip).
#pragma once

#include "tm_internal.h"

namespace tmap {

hipError_t launch_revcomp(const uint8_t* in, uint8_t* out, uint64_t L, hipStream_t s);
int match_device(tm_context* ctx, uint32_t n_reads, const MinimizerOut& m, const DevIndexView& fi,
                 const DevIndexView& ri, int fastq_rules, MatchOut& out);

}  // namespace tmap
