// tests/cpp/sanitize_driver.cpp -- host code of the build under the CPU
// sanitizers (tests/test_host_sanitizers.py builds this with
// -fsanitize=address,undefined and with -fsanitize=thread).  Modes:
//   oracle CASES     the C restatement (oracle/align_oracle.c) and the affine
//                    definition (oracle/affine_oracle.c) on the golden cases
//                    "type match mismatch gap qhex thex score tb cigarhex|-|ERR"
//                    (stdin-style file): results, path check, affine(open 0) == linear
//   planner SEED N T the host planner (bioinfo1_amd/csrc/ta_planner.cpp) on N
//                    random batches from T threads at once: every pair planned
//                    exactly once, chunk / workspace / task invariants
//   fastx PATH Q     the FASTA/FASTQ reader (tm_fastx.cpp): record count + checksum
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../bioinfo1_amd/csrc/ta_planner.h"
#include "../../bioinfo1_amd/csrc/tm_fastx.h"

extern "C" {
int oracle_align(const char* q, unsigned n, const char* t, unsigned m, int type, int match, int mismatch, int gap,
                 int want_cigar, int* score_out, unsigned* target_begin_out, char* cigar_out, size_t cigar_cap,
                 size_t* cigar_len);
int oracle_align_affine(const char* q, unsigned n, const char* t, unsigned m, int type, int match, int mismatch,
                        int open, int extend, int want_cigar, int* score_out, unsigned* target_begin_out,
                        char* cigar_out, size_t cigar_cap, size_t* cigar_len);
int oracle_cigar_check(const char* q, unsigned n, const char* t, unsigned m, int type, int match, int mismatch,
                       int gap, const char* cig, size_t clen, int score, unsigned target_begin);
}

namespace {

int fails = 0;
#define CHECK(c)                                                             \
    do {                                                                     \
        if (!(c)) {                                                          \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                         \
        }                                                                    \
    } while (0)

std::string unhex(const std::string& h) {
    std::string s;
    if (h == "-") return s;
    for (size_t i = 0; i + 1 < h.size(); i += 2) s.push_back((char)std::stoi(h.substr(i, 2), nullptr, 16));
    return s;
}

int run_oracle(const char* path) {
    std::ifstream in(path);
    std::string line;
    int n_cases = 0;
    while (std::getline(in, line)) {
        std::istringstream is(line);
        int type, ma, mi, g, want_score;
        unsigned want_tb;
        std::string qh, th, ws, wtb, wc;
        is >> type >> ma >> mi >> g >> qh >> th >> ws >> wtb >> wc;
        const std::string q = unhex(qh), t = unhex(th);
        std::vector<char> buf(2 * (q.size() + t.size()) + 2);
        int score = 0;
        unsigned tb = 0;
        size_t clen = 0;
        const int r = oracle_align(q.data(), (unsigned)q.size(), t.data(), (unsigned)t.size(), type, ma, mi, g, 1,
                                   &score, &tb, buf.data(), buf.size(), &clen);
        ++n_cases;
        if (ws == "ERR") {
            CHECK(r != 0);
            continue;
        }
        want_score = std::stoi(ws);
        want_tb = (unsigned)std::stoul(wtb);
        CHECK(r == 0);
        CHECK(score == want_score);
        CHECK(tb == want_tb);
        CHECK(std::string(buf.data(), clen) == unhex(wc));
        CHECK(oracle_cigar_check(q.data(), (unsigned)q.size(), t.data(), (unsigned)t.size(), type, ma, mi, g,
                                 buf.data(), clen, score, tb) == 0);
        // the affine definition with gap_open = 0 is team::Align with gap = gap_extend
        std::vector<char> abuf(buf.size());
        int as = 0;
        unsigned atb = 0;
        size_t alen = 0;
        const int ar = oracle_align_affine(q.data(), (unsigned)q.size(), t.data(), (unsigned)t.size(), type, ma, mi,
                                           0, g, 1, &as, &atb, abuf.data(), abuf.size(), &alen);
        if (ar == 0) {
            CHECK(as == score);
            CHECK(atb == tb);
            CHECK(std::string(abuf.data(), alen) == std::string(buf.data(), clen));
        }
    }
    std::printf("oracle cases %d fails %d\n", n_cases, fails);
    return fails ? 1 : 0;
}

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void check_linear(const ta::Plan& pl, uint64_t budget) {
    const uint32_t P = pl.n_pairs;
    std::vector<int> seen(P, 0);
    for (uint32_t x : pl.order) {
        CHECK(x < P);
        if (x < P) ++seen[x];
    }
    for (uint32_t p = 0; p < P; ++p) CHECK(seen[p] == 1);
    // units partition the pairs: singles + duals + flex (a self-coupled flex pair counts once)
    std::vector<int> unit(P, 0);
    for (uint32_t x : pl.singles) ++unit[x];
    for (size_t k = 0; k + 1 < pl.duals.size(); k += 2) {  // a lone pair may be coupled with itself
        ++unit[pl.duals[k]];
        if (pl.duals[k + 1] != pl.duals[k]) ++unit[pl.duals[k + 1]];
    }
    for (size_t k = 0; k + 1 < pl.flexes.size(); k += 2) {
        ++unit[pl.flexes[k]];
        if (pl.flexes[k + 1] != pl.flexes[k]) ++unit[pl.flexes[k + 1]];
    }
    for (uint32_t p = 0; p < P; ++p) CHECK(unit[p] == 1);
    uint64_t count = 0, s = 0, d = 0, f = 0;
    for (const auto& c : pl.chunks) {
        CHECK(c.begin == count);
        CHECK(c.sbegin == s && c.dbegin == d && c.fbegin == f);
        count += c.count;
        s += c.scount;
        d += c.dcount;
        f += c.fcount;
        CHECK(c.ptr_dwords <= pl.ws_ptr_dwords);
        CHECK(c.bnd_words <= pl.ws_bnd_words);
        // a chunk exceeds the budget only when it holds a single unit
        if (c.ptr_dwords * 4 > budget) CHECK(c.scount + c.dcount + c.fcount == 1);
        for (uint32_t k = c.begin; k < c.begin + c.count; ++k) {
            const uint32_t x = pl.order[k];
            const uint64_t need = pl.want_cigar ? ta::ptr_dwords_any(pl.qlen[x], pl.tlen[x], pl.blk) : 0;
            CHECK(pl.ptr_off[x] + need <= c.ptr_dwords);
            CHECK(pl.bnd_off[x] + ta::bnd_words(pl.qlen[x], pl.tlen[x]) <= c.bnd_words);
        }
    }
    CHECK(count == P && s == pl.singles.size() && d * 2 == pl.duals.size() && f * 2 == pl.flexes.size());
    // flex tasks: every (couple, pass) exactly once per chunk, pass-major
    CHECK(pl.flex_task_off.size() == pl.flexes.size() / 2 + 1);
    std::set<uint32_t> tasks(pl.flex_tasks.begin(), pl.flex_tasks.end());
    CHECK(tasks.size() == pl.flex_tasks.size());
    for (const auto& c : pl.chunks) {
        std::set<uint32_t> done;  // a task's predecessor (same couple, pass - 1) has an earlier ticket
        for (uint32_t k = pl.flex_task_off[c.fbegin]; k < pl.flex_task_off[c.fbegin + c.fcount]; ++k) {
            const uint32_t w = pl.flex_tasks[k] / 64, ps = pl.flex_tasks[k] % 64;
            CHECK(w >= c.fbegin && w < c.fbegin + c.fcount);
            if (ps) CHECK(done.count(pl.flex_tasks[k] - 1) == 1);
            done.insert(pl.flex_tasks[k]);
            CHECK(ps < pl.flex_task_off[w + 1] - pl.flex_task_off[w]);
        }
    }
    // pipelined int32 tasks: every (single, pass) of a chunk with spasses > 1
    // exactly once, pass-major; its pair holds two record buffers
    bool piped = false;
    for (const auto& c : pl.chunks) piped |= c.spasses > 1;
    CHECK(piped == !pl.single_task_off.empty());
    if (piped) {
        CHECK(pl.single_task_off.size() == pl.singles.size() + 1);
        CHECK(!pl.fused);
        for (const auto& c : pl.chunks) {
            if (c.spasses < 2) continue;
            std::set<uint64_t> seen_tasks;
            uint32_t maxp = 0;
            for (uint32_t w = c.sbegin; w < c.sbegin + c.scount; ++w) {
                const uint32_t x = pl.singles[w];
                const uint32_t want = pl.qlen[x] && pl.tlen[x] ? ta::n_passes(pl.qlen[x]) : 0;
                CHECK(pl.single_task_off[w + 1] - pl.single_task_off[w] == want);
                maxp = std::max(maxp, want);
                if (want > 1) CHECK(pl.bnd_off[x] + 4ull * (pl.tlen[x] + 1) <= c.bnd_words && pl.bnd_off[x] % 2 == 0);
            }
            CHECK(maxp == c.spasses);
            for (uint32_t k = pl.single_task_off[c.sbegin]; k < pl.single_task_off[c.sbegin + c.scount]; ++k) {
                const uint64_t code = pl.single_tasks[k];
                const uint32_t w = (uint32_t)(code >> 32), ps = (uint32_t)code;
                CHECK(w >= c.sbegin && w < c.sbegin + c.scount);
                if (ps) CHECK(seen_tasks.count(code - 1) == 1);  // predecessor ticketed earlier
                if (w < pl.singles.size()) CHECK(ps < pl.single_task_off[w + 1] - pl.single_task_off[w]);
                seen_tasks.insert(code);
            }
            CHECK(seen_tasks.size() == pl.single_task_off[c.sbegin + c.scount] - pl.single_task_off[c.sbegin]);
        }
    }
    for (size_t k = 0; k + 1 < pl.duals.size(); k += 2) {
        CHECK(pl.qlen[pl.duals[k]] == pl.qlen[pl.duals[k + 1]]);
        CHECK(pl.tlen[pl.duals[k]] == pl.tlen[pl.duals[k + 1]]);
        CHECK(ta::n_passes(pl.qlen[pl.duals[k]]) < 64);  // hand-off tags epoch * 64 + pass + 1 (ta_dual.hip)
    }
    for (size_t k = 0; k + 1 < pl.flexes.size(); k += 2) CHECK(ta::n_passes(pl.qlen[pl.flexes[k]]) < 64);
    uint64_t so = 0;
    for (uint32_t p = 0; p < P; ++p) {
        CHECK(pl.slot_off[p] == so);
        so += ta::cigar_slot_bytes(pl.qlen[p], pl.tlen[p]);
    }
    CHECK(so == pl.slots_bytes);
}

void check_affine(const ta::AffinePlan& pl) {
    const uint32_t P = pl.n_pairs;
    std::vector<int> seen(P, 0);
    for (uint32_t x : pl.order)
        if (x < P) ++seen[x];
    for (uint32_t p = 0; p < P; ++p) CHECK(seen[p] == 1);
    uint64_t count = 0;
    for (const auto& c : pl.chunks) {
        CHECK(c.begin == count);
        count += c.count;
        CHECK(c.ptr_entries <= pl.ws_ptr_entries);
    }
    CHECK(count == P);
    for (size_t k = 0; k + 1 < pl.duals.size(); k += 2) CHECK(ta::n_passes(pl.qlen[pl.duals[k]]) < 64);
    bool piped = false;
    for (const auto& c : pl.chunks) piped |= c.spasses > 1;
    CHECK(piped == !pl.single_task_off.empty());
    if (piped) {
        CHECK(pl.single_task_off.size() == pl.singles.size() + 1);
        for (const auto& c : pl.chunks) {
            if (c.spasses < 2) continue;
            std::set<uint64_t> seen_tasks;
            for (uint32_t w = c.sbegin; w < c.sbegin + c.scount; ++w) {
                const uint32_t x = pl.singles[w];
                if (ta::n_passes(pl.qlen[x]) > 1 && pl.tlen[x])
                    CHECK(pl.bnd_off[x] + 4ull * (pl.tlen[x] + 1) <= c.bnd_entries);
            }
            for (uint32_t k = pl.single_task_off[c.sbegin]; k < pl.single_task_off[c.sbegin + c.scount]; ++k) {
                const uint32_t w = (uint32_t)(pl.single_tasks[k] >> 32), ps = (uint32_t)pl.single_tasks[k];
                CHECK(w >= c.sbegin && w < c.sbegin + c.scount);
                if (ps) CHECK(seen_tasks.count(pl.single_tasks[k] - 1) == 1);  // predecessor ticketed earlier
                if (w < pl.singles.size()) CHECK(ps < pl.single_task_off[w + 1] - pl.single_task_off[w]);
                seen_tasks.insert(pl.single_tasks[k]);
            }
            CHECK(seen_tasks.size() == pl.single_task_off[c.sbegin + c.scount] - pl.single_task_off[c.sbegin]);
        }
    }
}

void plan_worker(uint64_t seed, int iters) {
    uint64_t s = seed;
    for (int it = 0; it < iters; ++it) {
        const int kind = (int)(splitmix(s) % 5);
        const uint32_t P = kind == 4 ? 2 + (uint32_t)(splitmix(s) % 3) : (uint32_t)(splitmix(s) % 300);
        std::vector<uint32_t> q(P), t(P);
        for (uint32_t p = 0; p < P; ++p) {
            switch (kind) {
                case 0: q[p] = t[p] = 1000; break;                                                 // config 2
                case 1: q[p] = (uint32_t)(splitmix(s) % 3000); t[p] = (uint32_t)(splitmix(s) % 3000); break;  // ragged
                case 2: q[p] = 1 + (uint32_t)(splitmix(s) % 20000); t[p] = q[p] + (uint32_t)(splitmix(s) % 500); break;
                case 3: q[p] = (uint32_t)(splitmix(s) % 4) * 1024 + 7; t[p] = 300 + (uint32_t)(splitmix(s) % 3); break;
                default: q[p] = 63 * 1024 + 1 + (uint32_t)(splitmix(s) % 3) * 1024; t[p] = 40; break;  // 63..65 passes
            }
        }
        const int type = (int)(splitmix(s) % 3);
        // (kind 4: all-zero scoring, whose values fit int16 at any length: only the pass bound stops couples)
        const int ma = kind == 4 ? 0 : 1 + (int)(splitmix(s) % 3), mi = kind == 4 ? 0 : -(int)(splitmix(s) % 3),
                  g = kind == 4 ? 0 : -(int)(splitmix(s) % 3);
        const uint64_t budget = (splitmix(s) & 1) ? (1ull << 40) : 4096ull + splitmix(s) % (64ull << 20);
        const uint32_t flags = (uint32_t)(splitmix(s) % 8) | ((splitmix(s) & 1) ? 32u : 0u) | ((splitmix(s) & 1) ? 64u : 0u);
        const bool cig = splitmix(s) % 4 != 0;
        ta::Plan pl;
        const uint32_t quantum = (splitmix(s) & 1) ? 1024u : (uint32_t)(splitmix(s) % 9);
        ta::build_plan(pl, P, q.data(), t.data(), type, ma, mi, g, cig, budget, flags, quantum);
        check_linear(pl, budget);
        ta::AffinePlan ap;
        ta::build_affine_plan(ap, P, q.data(), t.data(), type, ma, mi, -2, g, cig, budget, flags & 97u, quantum);
        check_affine(ap);
    }
}

// Small host batches (the drop-in call's combined batches, ta_align_batch)
// plan as ONE chunk under their own budget (ta_host_batch.h batch_budget), in
// both code layouts.
void check_small_batches() {
    const uint32_t shapes[][2] = {{1000, 1000}, {200, 200}, {5, 9}, {1000, 700}, {3000, 2500}};
    for (const auto& sh : shapes)
        for (uint32_t P : {1u, 2u, 3u, 8u, 16u, 33u})
            for (int type = 0; type < 3; ++type)
                for (uint32_t flags : {0u, 128u, 256u, 512u}) {  // TA_PLAN_NO_BLK, TA_PLAN_NO_CK, TA_PLAN_CK
                    std::vector<uint32_t> q(P, sh[0]), t(P, sh[1]);
                    const uint64_t budget = std::max<uint64_t>(ta::host_batch_code_bytes(P, q.data(), t.data(), 4), 1);
                    ta::Plan pl;
                    ta::build_plan(pl, P, q.data(), t.data(), type, 1, -1, -1, true, budget, flags, 1024);
                    check_linear(pl, budget);
                    CHECK(pl.chunks.size() == 1);
                    if (pl.chunks.size() != 1)
                        std::printf("small batch %u x %ux%u type %d flags %u: %zu chunks\n", P, sh[0], sh[1], type, flags,
                                    pl.chunks.size());
                    // every pair in the packed kernels (an odd one coupled with itself) when it fits
                    // int16 and is not tiny (or TA_PLAN_CK); band walks (blocked layout) from 8 local pairs up
                    // under TA_PLAN_NO_CK
                    const bool packed = ((uint64_t)sh[0] * sh[1] >= 4096 || flags == 512u) &&
                                        ta::fits_int16(type, sh[0], sh[1], 1, -1, -1);
                    // (n_dual_pairs counts two per couple, a self-coupled pair included)
                    if (packed) CHECK(pl.singles.empty() && pl.n_dual_pairs == 2 * ((P + 1) / 2));
                    // (tiny pairs of an even batch still couple with each other; only a lone one stays int32)
                    const bool all_packed = ta::fits_int16(type, sh[0], sh[1], 1, -1, -1) && (packed || P % 2 == 0);
                    // global / semi: checkpoints (blocked region sizes) whenever they are taken
                    const bool edge_ck = all_packed && type != ta::kLocal && flags == 512u;
                    // pairs past int16 in the dual kernel: flexible couples (self-coupled when alone),
                    // with checkpoints under TA_PLAN_CK when their H fits (ta_planner.cpp flex_ck_fits)
                    const bool flex_ck = flags == 512u && !ta::fits_int16(type, sh[0], sh[1], 1, -1, -1) &&
                                         ta::flex_ck_fits(type, sh[0], sh[1], 1, -1, -1);
                    // local: blocked codes only under TA_PLAN_NO_CK, or with checkpoints (TA_PLAN_CK)
                    CHECK(pl.blk == ((all_packed && type == ta::kLocal && P >= 8 && (flags == 256u || flags == 512u) &&
                                      sh[0] + sh[1] <= 6000) ||
                                     edge_ck || flex_ck));
                    // checkpoints and recomputing walks: small batches only with TA_PLAN_CK (gap -1 <= 0)
                    CHECK(pl.ck == (pl.blk && flags == 512u));
                    if (pl.ck) CHECK(pl.walk_group == 64);
                }
}

int run_planner(uint64_t seed, int iters, int threads) {
    check_small_batches();
    std::vector<std::thread> th;
    for (int w = 0; w < threads; ++w) th.emplace_back(plan_worker, seed + (uint64_t)w * 7919, iters);
    for (auto& x : th) x.join();
    std::printf("planner iters %d threads %d fails %d\n", iters, threads, fails);
    return fails ? 1 : 0;
}

int run_fastx(const char* path, bool fastq) {
    tmap::FastxFile f;
    std::string err;
    if (!tmap::read_fastx(path, fastq, f, err)) {
        std::printf("fastx error %s\n", err.c_str());
        return 0;  // a wrong-format read is a clean failure, not a sanitizer finding
    }
    uint64_t h = 1469598103934665603ull;
    for (const auto& r : f.records) {
        CHECK(r.off + r.len <= f.seq.size());
        for (char c : r.name) h = (h ^ (uint8_t)c) * 1099511628211ull;
        h = (h ^ r.len) * 1099511628211ull;
    }
    std::printf("fastx records %zu bases %zu hash %llx\n", f.records.size(), f.seq.size(), (unsigned long long)h);
    return fails ? 1 : 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc >= 3 && std::strcmp(argv[1], "oracle") == 0) return run_oracle(argv[2]);
    if (argc >= 5 && std::strcmp(argv[1], "planner") == 0)
        return run_planner(std::strtoull(argv[2], nullptr, 10), std::atoi(argv[3]), std::atoi(argv[4]));
    if (argc >= 4 && std::strcmp(argv[1], "fastx") == 0) return run_fastx(argv[2], std::atoi(argv[3]) != 0);
    std::fprintf(stderr, "usage: %s oracle CASES | planner SEED N THREADS | fastx PATH FASTQ\n", argv[0]);
    return 2;
}
