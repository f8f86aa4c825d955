// tests/cpp/shim_caller.cpp -- a team_mapper.cpp-shaped caller of the drop-in
// team::Align (include/team_alignment.hpp), linked against
// libteam_alignment.so exactly as the reference mapper links team_alignment
// (CMakeLists.txt:32-36).  Reads cases "type match mismatch gap qhex thex"
// from stdin; prints "score tb cigarhex" or "ERR <what()>" per case, like the
// mapper's try/catch at team_mapper.cpp:663-683.  With argv[1] == "threads"
// the cases are run from argv[2] (default 4) threads at once (the mapper's
// OpenMP loop).
#include <cstdio>
#include <cstring>
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

// (weak: defined only by the CPU stand-in tests/cpp/stub_ta.cpp; the GPU tests
// link this caller against the real library and never run "devices")
extern "C" __attribute__((weak)) void stub_set_current_device(int);
extern "C" __attribute__((weak)) int stub_last_device();
extern "C" int ta_set_thread_device(int);

// "devices": which device a thread's calls run on (include/team_align_c.h,
// ta_set_thread_device): its current device as of its first call, kept across
// a later device switch, re-read after ta_set_thread_device(-1), and a pinned
// device ahead of the current one -- on the server path (even query lengths,
// stub_ta.cpp) and on the batch path (odd ones).
int run_devices() {
    if (!stub_set_current_device || !stub_last_device) {
        std::printf("devices: needs the CPU stand-in (stub_ta.cpp)\n");
        return 2;
    }
    int bad = 0;
    auto call = [&](const char* q, int want, const char* what) {
        std::string cig;
        unsigned tb = 0;
        team::Align(q, (unsigned)std::strlen(q), "ACGTACGT", 8, team::AlignmentType::local, 1, -1, -1, &cig, &tb);
        if (stub_last_device() != want) {
            std::printf("%s: device %d, want %d\n", what, stub_last_device(), want);
            ++bad;
        }
    };
    for (const char* q : {"ACGT", "ACG"}) {  // server path, batch path
        std::thread([&] {
            stub_set_current_device(1);
            call(q, 1, "first call");
            stub_set_current_device(2);
            call(q, 1, "after a device switch (kept)");
            if (ta_set_thread_device(-1) != 0) ++bad;
            call(q, 2, "after ta_set_thread_device(-1)");
            if (ta_set_thread_device(3) != 0) ++bad;
            stub_set_current_device(0);
            call(q, 3, "pinned");
            if (ta_set_thread_device(99) == 0) ++bad;  // no such device
            call(q, 3, "pinned after a refused choice");
        }).join();
        std::thread([&] { call(q, 0, "another thread"); }).join();
    }
    std::printf("devices %s\n", bad ? "FAIL" : "ok");
    return bad ? 1 : 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "devices") return run_devices();
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
