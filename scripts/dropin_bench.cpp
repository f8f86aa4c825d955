// scripts/dropin_bench.cpp -- single-call throughput / latency of the drop-in
// team::Align, the way team_mapper.cpp calls it (one pair per call, from
// several threads: team_mapper.cpp:596 / 666-678).  The SAME source is linked
// twice: against libteam_alignment.so (build.sh -> build/dropin_amd) and
// against the reference's own team_alignment.cpp compiled from
// /root/reference (oracle/Makefile -> oracle/_ref/dropin_ref), so both numbers
// come from identical callers and identical pairs; the score checksum of the
// two runs must agree.
//
// usage: dropin_bench THREADS SECONDS SHAPES [MODE] [CIGAR]
//   SHAPES: comma list of NxM (query x target), e.g. 5x9,200x200,1000x1000
//   MODE: 0 global, 1 local (default), 2 semiGlobal; CIGAR: 1 (default) or 0
// Prints one JSON line per shape.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "team_alignment.hpp"

namespace {

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// a read window and a related reference window (~10 % substitutions)
std::pair<std::string, std::string> make_pair_(uint32_t n, uint32_t m, uint64_t seed) {
    static const char* A = "ACGT";
    uint64_t s = seed;
    std::string q(n, 'A'), t(m, 'A');
    for (auto& c : q) c = A[splitmix(s) >> 62];
    for (uint32_t j = 0; j < m; ++j) {
        const uint64_t r = splitmix(s);
        t[j] = (j < n && (r & 1023) >= 100) ? q[j] : A[r >> 62];
    }
    return {q, t};
}

struct Res {
    std::vector<double> lat_us;
    uint64_t calls = 0;
    int64_t checksum = 0;
};

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s THREADS SECONDS SHAPES [MODE] [CIGAR]\n", argv[0]);
        return 2;
    }
    const int threads = std::max(1, std::atoi(argv[1]));
    const double seconds = std::atof(argv[2]);
    const int mode = argc > 4 ? std::atoi(argv[4]) : 1;
    const bool want_cigar = argc > 5 ? std::atoi(argv[5]) != 0 : true;
    std::stringstream shapes(argv[3]);
    std::string sh;
    while (std::getline(shapes, sh, ',')) {
        const uint32_t n = (uint32_t)std::stoul(sh.substr(0, sh.find('x')));
        const uint32_t m = (uint32_t)std::stoul(sh.substr(sh.find('x') + 1));
        constexpr int kPairs = 64;
        std::vector<std::pair<std::string, std::string>> pairs;
        for (int k = 0; k < kPairs; ++k) pairs.push_back(make_pair_(n, m, 0xD809 ^ (uint64_t)k));
        // score checksum over the 64 pairs (identical for both builds)
        int64_t want = 0;
        for (auto& pq : pairs)
            want += team::Align(pq.first.data(), n, pq.second.data(), m, static_cast<team::AlignmentType>(mode), 1,
                                -1, -1, nullptr, nullptr);
        std::vector<Res> res(threads);
        std::atomic<int> ready{0};
        std::atomic<bool> go{false};
        std::vector<std::thread> th;
        for (int w = 0; w < threads; ++w)
            th.emplace_back([&, w] {
                Res& r = res[w];
                std::string cigar;
                unsigned tb = 0;
                for (int k = 0; k < 3; ++k)  // warm up: per-thread context, staging buffers
                    team::Align(pairs[k].first.data(), n, pairs[k].second.data(), m,
                                static_cast<team::AlignmentType>(mode), 1, -1, -1, want_cigar ? &cigar : nullptr, &tb);
                ++ready;
                while (!go.load()) std::this_thread::yield();
                const auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double>(seconds);
                for (uint64_t k = (uint64_t)w;; k += (uint64_t)threads) {
                    const auto& pq = pairs[k % kPairs];
                    const auto t0 = std::chrono::steady_clock::now();
                    const int s = team::Align(pq.first.data(), n, pq.second.data(), m,
                                              static_cast<team::AlignmentType>(mode), 1, -1, -1,
                                              want_cigar ? &cigar : nullptr, &tb);
                    const auto t1 = std::chrono::steady_clock::now();
                    r.lat_us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
                    r.checksum += s + (int64_t)cigar.size();
                    ++r.calls;
                    if (t1 >= t_end && r.calls >= 3) break;
                }
            });
        while (ready.load() < threads) std::this_thread::yield();
        const auto t0 = std::chrono::steady_clock::now();
        go = true;
        for (auto& t : th) t.join();
        const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::vector<double> lat;
        uint64_t calls = 0;
        for (auto& r : res) {
            lat.insert(lat.end(), r.lat_us.begin(), r.lat_us.end());
            calls += r.calls;
        }
        std::sort(lat.begin(), lat.end());
        auto pct = [&](double p) { return lat.empty() ? 0.0 : lat[std::min(lat.size() - 1, (size_t)(p * lat.size()))]; };
        std::printf("{\"shape\": \"%ux%u\", \"mode\": %d, \"cigar\": %s, \"threads\": %d, \"calls\": %llu, "
                    "\"wall_s\": %.3f, \"calls_per_s\": %.1f, \"gcups\": %.5f, \"lat_us_p50\": %.1f, "
                    "\"lat_us_p99\": %.1f, \"score_checksum\": %lld}\n",
                    n, m, mode, want_cigar ? "true" : "false", threads, (unsigned long long)calls, wall,
                    calls / wall, (double)calls * n * m / wall / 1e9, pct(0.5), pct(0.99), (long long)want);
        std::fflush(stdout);
    }
    return 0;
}
