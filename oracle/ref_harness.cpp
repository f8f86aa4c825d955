// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A C-callable wrapper around the UNMODIFIED reference team::Align, compiled
// by oracle/Makefile directly from /root/reference/team_alignment/
// team_alignment.cpp into oracle/_ref/libref_align.so (git-ignored).  It is
// used (1) by tests/golden/make_golden.py to produce the committed golden
// vectors and (2) by bench.py's cpu_baseline leg ("kind": "reference").
// No reference source is copied into this repository.
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "team_alignment.hpp"

namespace {
int copy_err(const char* what, char* errbuf, size_t errcap) {
  if (errbuf && errcap) {
    std::strncpy(errbuf, what, errcap - 1);
    errbuf[errcap - 1] = 0;
  }
  // 1: unknown type, 2: cigar walk error (the two messages the reference throws)
  return std::strstr(what, "AlignmentType") ? 1 : 2;
}
}  // namespace

extern "C" int ref_align(const char* q, unsigned n, const char* t, unsigned m, int type, int match,
                         int mismatch, int gap, int want_cigar, int* score, unsigned* target_begin,
                         char* cigar, size_t cigar_cap, size_t* cigar_len, char* errbuf, size_t errcap) {
  try {
    std::string c;
    unsigned tb = 0;
    int s = team::Align(q, n, t, m, static_cast<team::AlignmentType>(type), match, mismatch, gap,
                        want_cigar ? &c : nullptr, &tb);
    if (want_cigar) {
      if (c.size() > cigar_cap) return 4;
      std::memcpy(cigar, c.data(), c.size());
      *cigar_len = c.size();
    } else {
      *cigar_len = 0;
    }
    *score = s;
    *target_begin = tb;
    return 0;
  } catch (const std::invalid_argument& e) {
    return copy_err(e.what(), errbuf, errcap);
  }
}

// Batch form for the CPU baseline: OpenMP over pairs, schedule(dynamic), the
// way team_mapper.cpp:596 intends.  CIGARs go to per-pair slots.
extern "C" int ref_align_batch(unsigned n_pairs, const char* qb, const uint64_t* qoff, const uint32_t* qlen,
                               const char* tbytes, const uint64_t* toff, const uint32_t* tlen, int type,
                               int match, int mismatch, int gap, int want_cigar, int n_threads,
                               int32_t* scores, uint32_t* tbs, char* arena, const uint64_t* slot_off,
                               const uint64_t* slot_cap, uint32_t* cigar_lens, int32_t* status) {
  int bad = 0;
#ifdef _OPENMP
  if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic) reduction(+ : bad)
#endif
  for (long p = 0; p < (long)n_pairs; ++p) {
    int s = 0;
    unsigned tb = 0;
    size_t cl = 0;
    char err[128];
    int r = ref_align(qb + qoff[p], qlen[p], tbytes + toff[p], tlen[p], type, match, mismatch, gap,
                      want_cigar, &s, &tb, want_cigar ? arena + slot_off[p] : nullptr,
                      want_cigar ? slot_cap[p] : 0, &cl, err, sizeof err);
    status[p] = r;
    scores[p] = s;
    tbs[p] = tb;
    cigar_lens[p] = (uint32_t)cl;
    if (r) ++bad;
  }
  return bad;
}
