// tests/cpp/shim_caller.cpp -- a team_mapper.cpp-shaped caller of the drop-in
// team::Align (include/team_alignment.hpp), linked against
// libteam_alignment.so exactly as the reference mapper links team_alignment
// (CMakeLists.txt:32-36).  Reads cases "type match mismatch gap qhex thex"
// from stdin; prints "score tb cigarhex" or "ERR <what()>" per case, like the
// mapper's try/catch at team_mapper.cpp:663-683.  With argv[1] == "threads"
// the cases are run from argv[2] (default 4) threads at once (the mapper's
// OpenMP loop).
#include <cstdio>
#include <iostream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "team_alignment.hpp"

static std::string unhex(const std::string& h) {
    std::string s;
    for (size_t i = 0; i + 1 < h.size(); i += 2) s.push_back((char)std::stoi(h.substr(i, 2), nullptr, 16));
    return s;
}
static std::string hex(const std::string& s) {
    static const char* d = "0123456789abcdef";
    std::string o;
    for (unsigned char c : s) {
        o.push_back(d[c >> 4]);
        o.push_back(d[c & 15]);
    }
    return o;
}

struct Case {
    int type, m, n, g;
    std::string q, t, out;
};

static void run(Case& c) {
    std::string cigar;
    unsigned tb = 12345;
    try {
        int s = team::Align(c.q.data(), (unsigned)c.q.size(), c.t.data(), (unsigned)c.t.size(),
                            static_cast<team::AlignmentType>(c.type), c.m, c.n, c.g, &cigar, &tb);
        unsigned tb2 = 0;
        int s2 = team::Align(c.q.data(), (unsigned)c.q.size(), c.t.data(), (unsigned)c.t.size(),
                             static_cast<team::AlignmentType>(c.type), c.m, c.n, c.g, nullptr, &tb2);
        if (s2 != s || tb2 != tb) {
            c.out = "MISMATCH score-only";
            return;
        }
        c.out = std::to_string(s) + " " + std::to_string(tb) + " " + (cigar.empty() ? "-" : hex(cigar));
    } catch (const std::exception& e) {
        c.out = std::string("ERR ") + e.what();
    }
}

int main(int argc, char** argv) {
    std::vector<Case> cases;
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream is(line);
        Case c;
        std::string qh, th;
        is >> c.type >> c.m >> c.n >> c.g >> qh >> th;
        c.q = qh == "-" ? "" : unhex(qh);
        c.t = th == "-" ? "" : unhex(th);
        cases.push_back(c);
    }
    if (argc > 1 && std::string(argv[1]) == "threads") {
        const int T = argc > 2 ? std::stoi(argv[2]) : 4;  // concurrent calls are combined into batches
        std::vector<std::thread> th;
        for (int w = 0; w < T; ++w)
            th.emplace_back([&, w, T] {
                for (size_t i = w; i < cases.size(); i += (size_t)T) run(cases[i]);
            });
        for (auto& t : th) t.join();
    } else {
        for (auto& c : cases) run(c);
    }
    for (auto& c : cases) std::cout << c.out << "\n";
    return 0;
}
