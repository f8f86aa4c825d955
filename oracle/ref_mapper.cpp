/*
 * oracle/ref_mapper.cpp -- CPU checker for the mapper rows of SURVEY §8f.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (bioinfo1_amd/) links or
 * calls this file; tests/, tests/golden/make_mapper_golden.py and bench.py's
 * cpu_baseline leg use it as the checker.
 *
 * Built by oracle/Makefile into oracle/_ref/ together with the UNMODIFIED
 * reference sources team_minimizers/team_minimizers.cpp (KMER::Minimize) and
 * team_alignment/team_alignment.cpp (Align), compiled in place from
 * /root/reference.  The reference driver team_mapper.cpp itself cannot be
 * compiled here (it includes bioparser, an un-vendored dependency that is
 * absent: SURVEY §8c), so its glue is RESTATED below, each step citing the
 * team_mapper.cpp lines it follows.  Minimizers and alignments come from the
 * reference's own code; index / dedup / matching / chaining / PAF formatting
 * are the restatement ("parity pinned by the reference's Minimize and Align,
 * glue restated").
 *
 * Differences that are deliberate and documented:
 *  - reads are processed sequentially and printed in input order (the
 *    reference's OpenMP loop, team_mapper.cpp:596, prints in completion
 *    order);
 *  - FASTA/FASTQ are read by a small restatement of bioparser's rules
 *    (name cut at the first blank, sequence lines concatenated with trailing
 *    white space stripped; a FASTA file fails the FASTQ parse).
 *
 * Exposes:
 *  - extern "C" ref_minimize(): one team::KMER::Minimize call;
 *  - extern "C" ref_find_lis(): the restated FindLIS;
 *  - main() (with -DREF_MAPPER_MAIN): the restated mapper CLI, PAF on stdout.
 */
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <set>
#include <sstream>
#include <stdexcept>
#include <string>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "team_alignment.hpp"
#include "team_minimizers.hpp"

using Mini = std::tuple<unsigned int, unsigned int, bool>;
using Hit = std::pair<unsigned int, unsigned int>;  // (fragment pos, reference pos), 1-based

extern "C" int ref_minimize(const char* seq, unsigned len, unsigned k, unsigned w, int is_fwd, uint32_t* hash,
                            uint32_t* pos, uint8_t* strand, size_t cap, size_t* count, size_t* n_unique) {
    team::KMER km(is_fwd != 0);
    std::vector<Mini> v = km.Minimize(seq, len, k, w);
    *count = v.size();
    *n_unique = km.GetUniqueMinimizers().size();
    if (v.size() > cap) return 1;
    for (size_t i = 0; i < v.size(); ++i) {
        hash[i] = std::get<0>(v[i]);
        pos[i] = std::get<1>(v[i]);
        strand[i] = std::get<2>(v[i]) ? 1 : 0;
    }
    return 0;
}

namespace {

// team_mapper.cpp:26-42: keep the first occurrence of every (hash, pos, strand).
std::vector<Mini> first_occurrences(const std::vector<Mini>& in) {
    std::set<Mini> seen;
    std::vector<Mini> out;
    for (const Mini& m : in)
        if (seen.insert(m).second) out.push_back(m);
    return out;
}

// team_mapper.cpp:283-316.  lis[i] = 1 + max lis[j] over earlier j with a
// strictly larger reference position, a different fragment position and both
// unsigned differences below 5000; the first such j wins ties; the chain ends
// at the first maximal lis.
std::vector<Hit> find_lis(const std::vector<Hit>& h) {
    const size_t n = h.size();
    if (!n) return {};
    std::vector<int> lis(n, 1), prev(n, -1);
    for (size_t i = 1; i < n; ++i)
        for (size_t j = 0; j < i; ++j) {
            const bool ok = h[i].second > h[j].second && h[i].first != h[j].first &&
                            h[i].first - h[j].first < 5000u && h[i].second - h[j].second < 5000u;
            if (ok && lis[j] + 1 > lis[i]) {
                lis[i] = lis[j] + 1;
                prev[i] = (int)j;
            }
        }
    int best = (int)(std::max_element(lis.begin(), lis.end()) - lis.begin());
    std::vector<Hit> chain;
    for (int i = best; i >= 0; i = prev[i]) chain.push_back(h[i]);
    std::reverse(chain.begin(), chain.end());
    return chain;
}

}  // namespace

extern "C" int ref_find_lis(size_t n, const uint32_t* fpos, const uint32_t* rpos, uint32_t* out_f, uint32_t* out_r,
                            size_t* out_n) {
    std::vector<Hit> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = {fpos[i], rpos[i]};
    std::vector<Hit> c = find_lis(h);
    *out_n = c.size();
    for (size_t i = 0; i < c.size(); ++i) {
        out_f[i] = c[i].first;
        out_r[i] = c[i].second;
    }
    return 0;
}

#ifdef REF_MAPPER_MAIN
namespace {

struct Rec {
    std::string name, seq;
};

std::string rstrip(const std::string& s) {
    size_t e = s.size();
    while (e && std::isspace((unsigned char)s[e - 1])) --e;
    return s.substr(0, e);
}

std::string short_name(const std::string& header) {
    std::string h = rstrip(header.substr(1));
    size_t c = h.find_first_of(" \t");
    return c == std::string::npos ? h : h.substr(0, c);
}

std::vector<std::string> lines_of(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::invalid_argument("cannot open " + path);
    std::vector<std::string> out;
    std::string l;
    while (std::getline(f, l)) out.push_back(l);
    return out;
}

std::vector<Rec> read_fasta(const std::string& path) {
    std::vector<Rec> out;
    for (const std::string& l : lines_of(path)) {
        if (!l.empty() && l[0] == '>') {
            out.push_back({short_name(l), ""});
        } else {
            std::string s = rstrip(l);
            if (s.empty()) continue;
            if (out.empty()) throw std::invalid_argument("invalid FASTA");
            out.back().seq += s;
        }
    }
    for (const Rec& r : out)
        if (r.name.empty() || r.seq.empty()) throw std::invalid_argument("invalid FASTA");
    return out;
}

std::vector<Rec> read_fastq(const std::string& path) {
    std::vector<std::string> ls = lines_of(path);
    std::vector<Rec> out;
    size_t i = 0;
    while (i < ls.size()) {
        if (rstrip(ls[i]).empty()) {
            ++i;
            continue;
        }
        if (ls[i][0] != '@') throw std::invalid_argument("invalid FASTQ");
        Rec r{short_name(ls[i]), ""};
        ++i;
        while (i < ls.size() && (ls[i].empty() || ls[i][0] != '+')) r.seq += rstrip(ls[i++]);
        if (i >= ls.size()) throw std::invalid_argument("invalid FASTQ");
        ++i;
        size_t q = 0;
        while (i < ls.size() && q < r.seq.size()) q += rstrip(ls[i++]).size();
        if (q != r.seq.size() || r.seq.empty()) throw std::invalid_argument("invalid FASTQ");
        out.push_back(std::move(r));
    }
    return out;
}

std::string revcomp(const std::string& s) {  // team_mapper.cpp:47-63
    std::string r(s.rbegin(), s.rend());
    for (char& c : r) c = c == 'A' ? 'T' : c == 'T' ? 'A' : c == 'G' ? 'C' : c == 'C' ? 'G' : c;
    return r;
}

using Index = std::unordered_map<unsigned int, std::set<std::pair<unsigned int, bool>>>;

// team_mapper.cpp:432-471: the top `limit` hashes of `by_count` (sorted by
// descending frequency with std::sort over the unordered_map's iteration
// order, exactly the reference's container sequence) are banned.
std::vector<std::pair<unsigned int, int>> by_count(const std::unordered_map<unsigned int, int>& freq) {
    std::vector<std::pair<unsigned int, int>> v(freq.begin(), freq.end());
    std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.second > b.second; });
    return v;
}

}  // namespace

int main(int argc, char** argv) {
    team::AlignmentType type = team::AlignmentType::global;  // team_mapper.cpp:321-327
    int match = 1, mismatch = -1, gap = -1;
    unsigned k = 15, w = 5;
    double f = 0.001;
    bool want_cigar = false;
    std::string file1, file2;
    for (int i = 1; i < argc; ++i) {  // team_mapper.cpp:348-387
        std::string a = argv[i];
        auto next = [&]() { return std::string(argv[++i]); };
        if (a == "-a" && i + 1 < argc) {
            std::string t = next();
            if (t == "global") type = team::AlignmentType::global;
            else if (t == "local") type = team::AlignmentType::local;
            else if (t == "semiGlobal") type = team::AlignmentType::semiGlobal;
            else return 1;
        } else if (a == "-m" && i + 1 < argc) match = std::atoi(next().c_str());
        else if (a == "-n" && i + 1 < argc) mismatch = std::atoi(next().c_str());
        else if (a == "-g" && i + 1 < argc) gap = std::atoi(next().c_str());
        else if (a == "-k" && i + 1 < argc) k = (unsigned)std::atoi(next().c_str());
        else if (a == "-w" && i + 1 < argc) w = (unsigned)std::atoi(next().c_str());
        else if (a == "-f" && i + 1 < argc) f = std::stod(next());
        else if (a == "-c") want_cigar = true;
        else if (file1.empty()) file1 = a;
        else if (file2.empty()) file2 = a;
        else return 1;
    }
    if (file1.empty() || file2.empty()) return 1;

    const auto t0 = std::chrono::steady_clock::now();
    // reference + its reverse complement, minimizers and frequencies (:398-430)
    std::vector<Rec> refs = read_fasta(file1);
    const Rec& R = refs.front();
    const std::string& ref = R.seq;
    const std::string ref_rc = revcomp(ref);
    team::KMER kf(true);
    std::vector<Mini> mf = kf.Minimize(ref.c_str(), (unsigned)ref.size(), k, w);
    std::unordered_map<unsigned int, int> freq_f = kf.GetMinimizerFrequencies();
    team::KMER kr(false);
    std::vector<Mini> mr = kr.Minimize(ref_rc.c_str(), (unsigned)ref_rc.size(), k, w);
    std::unordered_map<unsigned int, int> freq_r = kr.GetMinimizerFrequencies();
    // both thresholds read the unique set left by the LAST Minimize call (the
    // reference keeps it in a namespace-level global): the reverse strand's
    const size_t uniq = kf.GetUniqueMinimizers().size();
    const int thr_f = static_cast<int>(f * uniq), thr_r = static_cast<int>(f * uniq);
    std::vector<std::pair<unsigned int, int>> vf = by_count(freq_f), vr = by_count(freq_r);
    std::unordered_set<unsigned int> ban_f, ban_r;
    for (int i = 0; i < std::min(thr_f, (int)vf.size()); ++i) ban_f.insert(vf[i].first);
    // the reverse ban list is filled from the FORWARD ranking (:463-465)
    for (int i = 0; i < std::min(thr_r, (int)vr.size()); ++i) ban_r.insert(vf[i].first);
    Index idx_f, idx_r;
    for (const Mini& m : mf)
        if (!ban_f.count(std::get<0>(m))) idx_f[std::get<0>(m)].insert({std::get<1>(m), std::get<2>(m)});
    for (const Mini& m : mr)
        if (!ban_r.count(std::get<0>(m))) idx_r[std::get<0>(m)].insert({std::get<1>(m), std::get<2>(m)});

    // fragments: FASTQ first, FASTA on failure (:533-556)
    bool fastq = true;
    std::vector<Rec> reads;
    try {
        reads = read_fastq(file2);
    } catch (const std::exception&) {
        fastq = false;
        try {
            reads = read_fasta(file2);
        } catch (const std::exception&) {
            std::cerr << "Given file is not in FASTA or FASTQ format! " << std::endl;
            return 1;
        }
    }

    const auto t1 = std::chrono::steady_clock::now();
    uint64_t cells = 0, mapped = 0;
    for (const Rec& rd : reads) {  // :596-698 (FASTA), :709-789 (FASTQ)
        team::KMER kq(true);
        if (!fastq) kq.SetFrequenciesCount(false);
        std::vector<Mini> qm = first_occurrences(kq.Minimize(rd.seq.c_str(), (unsigned)rd.seq.size(), k, w));
        std::vector<Hit> hf, hr;
        for (const Mini& m : qm) {
            const unsigned h = std::get<0>(m), p = std::get<1>(m);
            auto itf = idx_f.find(h);
            if (itf != idx_f.end())
                for (const auto& rp : itf->second) hf.emplace_back(p, rp.first);
            // FASTA path: reverse hits only for hashes present in the forward
            // index (:637-645); FASTQ path: independently (:721-730)
            if (fastq || itf != idx_f.end()) {
                auto itr = idx_r.find(h);
                if (itr != idx_r.end())
                    for (const auto& rp : itr->second) hr.emplace_back(p, rp.first);
            }
        }
        std::vector<Hit> cf = find_lis(hf), cr = find_lis(hr);
        const bool fwd = cf.size() >= cr.size();  // :650-656
        const std::vector<Hit>& c = fwd ? cf : cr;
        if (c.empty()) continue;
        const unsigned qb = c.front().first - 1, qe = c.back().first + k - 2;  // :660-663
        const unsigned tb = c.front().second - 1, te = c.back().second + k - 2;
        const std::string& T = fwd ? ref : ref_rc;
        std::string cigar;
        unsigned off = 0;
        int score;
        try {
            score = team::Align(rd.seq.c_str() + qb, qe - qb + 1, T.c_str() + tb, te - tb + 1, type, match, mismatch,
                                gap, want_cigar ? &cigar : nullptr, &off);
        } catch (const std::exception& e) {
            std::cerr << "ERROR: Exception during Align: " << e.what() << std::endl;
            continue;
        }
        cells += (uint64_t)(qe - qb + 1) * (te - tb + 1);
        ++mapped;
        // PAF-like line (:686-697): reverse hits are reported in forward coordinates
        std::cout << rd.name << "\t" << rd.seq.size() << "\t" << qb << "\t" << (qe + 1) << "\t" << (fwd ? "+" : "-")
                  << "\t" << R.name << "\t" << ref.size() << "\t"
                  << (fwd ? tb : (unsigned)(ref_rc.size() - te - 1)) << "\t"
                  << (fwd ? te + 1 : (unsigned)(ref_rc.size() - tb)) << "\t" << score << "\t" << (qe - qb + 1)
                  << "\t60";
        if (want_cigar) std::cout << "\tcg:Z:" << cigar;
        std::cout << std::endl;
    }
    if (std::getenv("REF_MAPPER_TIMING")) {
        const auto t2 = std::chrono::steady_clock::now();
        std::cerr << "ref_mapper_timing index_s=" << std::chrono::duration<double>(t1 - t0).count()
                  << " map_s=" << std::chrono::duration<double>(t2 - t1).count() << " reads=" << reads.size()
                  << " mapped=" << mapped << " aligned_cells=" << cells << std::endl;
    }
    return 0;
}
#endif
