// include/team_alignment.hpp -- drop-in interface for the MI355X team_alignment
// library.
//
// Declares exactly what the reference header declares
// (/root/reference/team_alignment/team_alignment.hpp:7-28): namespace team,
// the AlignmentType enum (underlying int; global=0, local=1, semiGlobal=2) and
// Align() with its default arguments.  A caller such as team_mapper.cpp
// compiles and links against libteam_alignment.so unchanged: the exported
// symbol is the same mangled name,
//   _ZN4team5AlignEPKcjS1_jNS_13AlignmentTypeEiiiPNSt7__cxx1112basic_stringIcSt11char_traitsIcESaIcEEEPj
// Behaviour (score, CIGAR bytes, *target_begin, the two std::invalid_argument
// messages) is bit-exact with the reference; the DP runs on the GPU through the
// extern "C" batch ABI in team_align_c.h.
#ifndef TEAM_ALIGNMENT_HPP
#define TEAM_ALIGNMENT_HPP

#include <string>

namespace team {

enum class AlignmentType {
    global,     // Needleman-Wunsch
    local,      // Smith-Waterman
    semiGlobal  // free leading/trailing gaps ("Gotoh" in the reference comment; linear gap)
};

int Align(const char* query, unsigned int query_len, const char* target, unsigned int target_len,
          AlignmentType type, int match, int mismatch, int gap, std::string* cigar = nullptr,
          unsigned int* target_begin = nullptr);

}  // namespace team

#endif  // TEAM_ALIGNMENT_HPP
