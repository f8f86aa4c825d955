// TEST-ONLY (tests/test_abi.py).  The surface of the bioparser library -- an
// un-vendored git submodule of the reference, absent from its checkout -- that
// /root/reference/team_mapper.cpp uses (:187-188, :230-235, :401-402,
// :534-551): Parser<T>::Create<FastaParser | FastqParser>(path) and
// Parse(bytes).  It exists only so that the unmodified team_mapper.cpp
// compiles and links against libteam_alignment.so with nothing undefined.  It
// parses nothing (every Parse throws), so the executable pins no results and is
// never used as an oracle.
#pragma once

// (standard headers the real bioparser headers bring in, which team_mapper.cpp
// relies on transitively: std::sort, std::reverse, std::max_element, strcmp)
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace bioparser {

template <class T>
class Parser {
public:
    virtual ~Parser() = default;
    template <template <class> class P>
    static std::unique_ptr<Parser<T>> Create(const std::string& path) {
        return std::unique_ptr<Parser<T>>(new P<T>(path));
    }
    virtual std::vector<std::unique_ptr<T>> Parse(std::uint64_t bytes, bool shorten_names = true) = 0;
};

template <class T>
class SurfaceParser : public Parser<T> {
public:
    explicit SurfaceParser(const std::string&) {}
    std::vector<std::unique_ptr<T>> Parse(std::uint64_t, bool = true) override {
        // (opaque to the optimiser, so that the mapper's code after a parse -- its
        // team::Align calls -- stays in the executable; the variable is never set)
        if (std::getenv("BIOPARSER_TEST_SURFACE_EMPTY")) return {};
        throw std::invalid_argument("[bioparser test surface] parses nothing");
    }
};

}  // namespace bioparser
