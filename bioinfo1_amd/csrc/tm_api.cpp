// bioinfo1_amd/csrc/tm_api.cpp -- host side of the mapper ABI
// (include/team_mapper_c.h): contexts, the reference minimizer index, the
// batched mapper (minimizers -> seed hits -> FindLIS chains -> one
// team_alignment batch plan) and the file-level driver that writes the
// reference's PAF-like lines.  The per-read work runs in the HIP stages
// (tm_minimizers.hip, tm_match.hip, tm_chain.hip, libteam_alignment).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "tm_fastx.h"
#include "tm_internal.h"
#include "tm_match.h"

struct tm_index {
    tm_context* ctx = nullptr;
    std::string name;
    uint64_t len = 0;
    uint32_t k = 0, w = 0;
    tmap::DevBuf ref2;  // [forward | reverse complement], 2*len bytes
    struct Strand {
        tmap::DevBuf keys, koff, pos;
        uint32_t n_keys = 0;
        uint64_t n_pos = 0;
        uint32_t banned = 0;
        tmap::DevIndexView view() const {
            return {keys.as<uint32_t>(), koff.as<uint32_t>(), pos.as<uint32_t>(), n_keys};
        }
    } fwd, rev;
};

namespace {

using tmap::fail;

bool valid_kw(uint32_t k, uint32_t w) { return k >= 1 && k <= tmap::kMaxK && w >= 1 && w <= tmap::kMaxW; }

// team_mapper.cpp:432-446: hashes by descending frequency.  std::sort over the
// unordered_map's iteration order, with the map built by the same sequence of
// operator[] increments as the reference (KMER::Minimize, team_minimizers.cpp
// :160-167/190-196/214-220), so equal counts fall in the same order.
std::vector<std::pair<unsigned int, int>> ranked(const uint32_t* hashes, uint64_t n) {
    std::unordered_map<unsigned int, int> freq;
    for (uint64_t i = 0; i < n; ++i) freq[hashes[i]]++;
    std::vector<std::pair<unsigned int, int>> v(freq.begin(), freq.end());
    std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.second > b.second; });
    return v;
}

// CSR over the surviving (hash, position) pairs of one strand (the
// unordered_map<hash, set<(pos, strand)>> of team_mapper.cpp:449-471).
int build_strand(tm_context* ctx, tm_index::Strand& st, const uint32_t* h, const uint32_t* p, uint64_t n,
                 const std::unordered_set<unsigned int>& ban) {
    std::vector<uint64_t> kv;
    kv.reserve(n);
    for (uint64_t i = 0; i < n; ++i)
        if (!ban.count(h[i])) kv.push_back(((uint64_t)h[i] << 32) | p[i]);
    std::sort(kv.begin(), kv.end());
    kv.erase(std::unique(kv.begin(), kv.end()), kv.end());
    std::vector<uint32_t> keys, koff, pos(kv.size());
    for (size_t i = 0; i < kv.size(); ++i) {
        const uint32_t hh = (uint32_t)(kv[i] >> 32);
        if (keys.empty() || keys.back() != hh) {
            keys.push_back(hh);
            koff.push_back((uint32_t)i);
        }
        pos[i] = (uint32_t)kv[i];
    }
    koff.push_back((uint32_t)kv.size());
    st.n_keys = (uint32_t)keys.size();
    st.n_pos = kv.size();
    st.banned = (uint32_t)ban.size();
    hipStream_t s = ctx->stream;
    TM_HIP(ctx, st.keys.reserve(keys.size() * 4 + 4));
    TM_HIP(ctx, st.koff.reserve(koff.size() * 4 + 4));
    TM_HIP(ctx, st.pos.reserve(pos.size() * 4 + 4));
    if (!keys.empty()) TM_HIP(ctx, hipMemcpyAsync(st.keys.p, keys.data(), keys.size() * 4, hipMemcpyHostToDevice, s));
    TM_HIP(ctx, hipMemcpyAsync(st.koff.p, koff.data(), koff.size() * 4, hipMemcpyHostToDevice, s));
    if (!pos.empty()) TM_HIP(ctx, hipMemcpyAsync(st.pos.p, pos.data(), pos.size() * 4, hipMemcpyHostToDevice, s));
    TM_HIP(ctx, hipStreamSynchronize(s));
    return TM_OK;
}

}  // namespace

extern "C" {

const char* tm_status_string(int status) {
    switch (status) {
        case TM_OK: return "ok";
        case TM_ERR_BAD_TYPE: return "Unknown AlignmentType provided.";
        case TM_ERR_ARG: return "invalid argument";
        case TM_ERR_DEVICE: return "device error";
        case TM_ERR_CAPACITY: return "output buffer too small";
        case TM_ERR_INPUT: return "Given file is not in FASTA or FASTQ format!";
        default: return "unknown status";
    }
}

const char* tm_last_error(const tm_context* ctx) { return ctx ? ctx->last_error.c_str() : ""; }

int tm_context_create(int device, tm_context** out) {
    if (!out) return TM_ERR_ARG;
    *out = nullptr;
    ta_context* ta = nullptr;
    if (int r = ta_context_create(device, &ta)) return r == TA_ERR_DEVICE ? TM_ERR_DEVICE : TM_ERR_ARG;
    auto* c = new tm_context();
    c->device = device;
    c->ta = ta;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        tm_context_destroy(c);
        return TM_ERR_DEVICE;
    }
    *out = c;
    return TM_OK;
}

void tm_context_destroy(tm_context* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    tmap::MinimizerOut& m = c->mins;
    for (tmap::DevBuf* b : {&c->bytes, &c->off, &c->len, &m.entry_off, &m.tiles, &m.hash, &m.pos, &m.keep, &m.scan,
                          &m.kept_off, &m.khash, &m.kpos, &m.cub_tmp, &c->c_off, &c->c_f, &c->c_r, &c->c_out,
                          &c->c_prev, &c->c_lis, &c->m_qoff, &c->m_toff, &c->m_score, &c->m_tb, &c->m_slots,
                          &c->m_cstart, &c->m_clen, &c->m_coff, &c->m_cdst, &c->match.cnt_f, &c->match.cnt_r, &c->match.off_f,
                          &c->match.off_r, &c->match.key_f, &c->match.key_r, &c->match.hf, &c->match.hr,
                          &c->match.list_off, &c->match.cub_tmp})
        b->release();
    if (c->stream) (void)hipStreamDestroy(c->stream);
    ta_context_destroy(c->ta);
    delete c;
}

int tm_index_create(tm_context* ctx, const char* name, const char* seq, uint64_t len, uint32_t k, uint32_t w, double f,
                    tm_index** out) {
    if (!ctx || !out || (len && !seq)) return TM_ERR_ARG;
    *out = nullptr;
    if (!valid_kw(k, w)) return fail(ctx, TM_ERR_ARG, "unsupported k or w");
    if (len >= (1ull << 31)) return fail(ctx, TM_ERR_ARG, "reference longer than 2^31 bases");
    TM_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    auto* idx = new tm_index();
    idx->ctx = ctx;
    idx->name = name ? name : "";
    idx->len = len;
    idx->k = k;
    idx->w = w;
    auto bail = [&](int r) {
        tm_index_destroy(idx);
        return r;
    };
    if (idx->ref2.reserve(2 * len + 1) != hipSuccess) return bail(fail(ctx, TM_ERR_DEVICE, "hipMalloc reference"));
    if (len && (hipMemcpyAsync(idx->ref2.p, seq, len, hipMemcpyHostToDevice, s) != hipSuccess ||
                tmap::launch_revcomp(idx->ref2.as<uint8_t>(), idx->ref2.as<uint8_t>() + len, len, s) != hipSuccess))
        return bail(fail(ctx, TM_ERR_DEVICE, "reference upload / reverse complement"));
    // both strands' minimizers in one batch (team_mapper.cpp:413-427)
    const uint64_t h_off[2] = {0, len};
    const uint32_t h_len[2] = {(uint32_t)len, (uint32_t)len};
    if (ctx->off.reserve(16) != hipSuccess || ctx->len.reserve(8) != hipSuccess ||
        hipMemcpyAsync(ctx->off.p, h_off, 16, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(ctx->len.p, h_len, 8, hipMemcpyHostToDevice, s) != hipSuccess)
        return bail(fail(ctx, TM_ERR_DEVICE, "index staging"));
    tmap::MinimizerOut& mo = ctx->mins;
    if (int r = tmap::minimize_device(ctx, 2, idx->ref2.as<uint8_t>(), ctx->off.as<uint64_t>(), ctx->len.as<uint32_t>(),
                                    h_len, k, w, true, mo))
        return bail(r);
    std::vector<uint32_t> full(mo.total), kh(mo.kept), kp(mo.kept);
    uint64_t kept_off[3] = {0, 0, 0};
    bool ok = (mo.total == 0 || hipMemcpyAsync(full.data(), mo.hash.p, mo.total * 4, hipMemcpyDeviceToHost, s) == hipSuccess) &&
              (mo.kept == 0 || (hipMemcpyAsync(kh.data(), mo.khash.p, mo.kept * 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
                                hipMemcpyAsync(kp.data(), mo.kpos.p, mo.kept * 4, hipMemcpyDeviceToHost, s) == hipSuccess)) &&
              hipMemcpyAsync(kept_off, mo.kept_off.p, 24, hipMemcpyDeviceToHost, s) == hipSuccess &&
              hipStreamSynchronize(s) == hipSuccess;
    if (!ok) return bail(fail(ctx, TM_ERR_DEVICE, "index download"));
    const uint64_t ef = mo.h_entry_off[1];
    // frequency ranking per strand; both thresholds use the reverse strand's
    // unique count (the reference's GetUniqueMinimizers reads a namespace-level
    // set that the reverse Minimize call refilled last, team_mapper.cpp:431-432)
    const std::vector<std::pair<unsigned int, int>> vf = ranked(full.data(), ef);
    const std::vector<std::pair<unsigned int, int>> vr = ranked(full.data() + ef, mo.total - ef);
    const uint64_t uniq_rev = kept_off[2] - kept_off[1];
    const int thr = static_cast<int>(f * (double)uniq_rev);
    std::unordered_set<unsigned int> ban_f, ban_r;
    for (int i = 0; i < std::min(thr, (int)vf.size()); ++i) ban_f.insert(vf[i].first);
    // the reverse ban list is taken from the FORWARD ranking (team_mapper.cpp:463-465)
    for (int i = 0; i < std::min(std::min(thr, (int)vr.size()), (int)vf.size()); ++i) ban_r.insert(vf[i].first);
    if (int r = build_strand(ctx, idx->fwd, kh.data(), kp.data(), kept_off[1], ban_f)) return bail(r);
    if (int r = build_strand(ctx, idx->rev, kh.data() + kept_off[1], kp.data() + kept_off[1], kept_off[2] - kept_off[1],
                             ban_r))
        return bail(r);
    *out = idx;
    return TM_OK;
}

void tm_index_destroy(tm_index* idx) {
    if (!idx) return;
    (void)hipSetDevice(idx->ctx->device);
    for (tmap::DevBuf* b : {&idx->ref2, &idx->fwd.keys, &idx->fwd.koff, &idx->fwd.pos, &idx->rev.keys, &idx->rev.koff,
                          &idx->rev.pos})
        b->release();
    delete idx;
}

int tm_index_stats(const tm_index* idx, uint64_t* fk, uint64_t* rk, uint64_t* fp, uint64_t* rp, uint32_t* bf,
                   uint32_t* br) {
    if (!idx) return TM_ERR_ARG;
    if (fk) *fk = idx->fwd.n_keys;
    if (rk) *rk = idx->rev.n_keys;
    if (fp) *fp = idx->fwd.n_pos;
    if (rp) *rp = idx->rev.n_pos;
    if (bf) *bf = idx->fwd.banned;
    if (br) *br = idx->rev.banned;
    return TM_OK;
}

int tm_map_batch(tm_context* ctx, const tm_index* idx, uint32_t n_reads, const char* bytes, const uint64_t* off,
                 const uint32_t* len, const tm_options* opt, uint8_t* mapped, uint8_t* strand_fwd, uint32_t* q_begin,
                 uint32_t* q_end, uint32_t* t_begin, uint32_t* t_end, int32_t* score, char* arena,
                 uint64_t arena_bytes, uint64_t* cigar_off, uint32_t* cigar_len) {
    if (!ctx || !idx || !opt) return TM_ERR_ARG;
    if (opt->type != TA_GLOBAL && opt->type != TA_LOCAL && opt->type != TA_SEMI_GLOBAL)
        return fail(ctx, TM_ERR_BAD_TYPE, tm_status_string(TM_ERR_BAD_TYPE));
    if (opt->k != idx->k || opt->w != idx->w) return fail(ctx, TM_ERR_ARG, "k/w differ from the index");
    if (!n_reads) return TM_OK;
    if (!off || !len || !mapped || !strand_fwd || !q_begin || !q_end || !t_begin || !t_end || !score)
        return fail(ctx, TM_ERR_ARG, "null argument");
    if (opt->want_cigar && (!arena || !cigar_off || !cigar_len)) return fail(ctx, TM_ERR_ARG, "null cigar output");
    TM_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    uint64_t nbytes = 0;
    for (uint32_t r = 0; r < n_reads; ++r) nbytes = std::max<uint64_t>(nbytes, off[r] + len[r]);
    TM_HIP(ctx, ctx->bytes.reserve(nbytes + 1));
    TM_HIP(ctx, ctx->off.reserve(n_reads * 8ull));
    TM_HIP(ctx, ctx->len.reserve(n_reads * 4ull));
    using clk = std::chrono::steady_clock;
    auto t_last = clk::now();
    const auto t_first = t_last;
    std::fill(ctx->stage_ms, ctx->stage_ms + tmap::kStages, 0.0);
    auto stage = [&](int i) -> int {  // close stage i (the stream is drained so host time = device time)
        TM_HIP(ctx, hipStreamSynchronize(s));
        const auto t = clk::now();
        ctx->stage_ms[i] = std::chrono::duration<double, std::milli>(t - t_last).count();
        ctx->stage_ms[tmap::kStages - 1] = std::chrono::duration<double, std::milli>(t - t_first).count();
        t_last = t;
        return TM_OK;
    };
    if (nbytes) TM_HIP(ctx, hipMemcpyAsync(ctx->bytes.p, bytes, nbytes, hipMemcpyHostToDevice, s));
    TM_HIP(ctx, hipMemcpyAsync(ctx->off.p, off, n_reads * 8ull, hipMemcpyHostToDevice, s));
    TM_HIP(ctx, hipMemcpyAsync(ctx->len.p, len, n_reads * 4ull, hipMemcpyHostToDevice, s));
    if (int r = stage(0)) return r;
    // 1. read minimizers, first occurrences only (team_mapper.cpp:611-612, 713-714)
    tmap::MinimizerOut& mo = ctx->mins;
    if (int r = tmap::minimize_device(ctx, n_reads, ctx->bytes.as<uint8_t>(), ctx->off.as<uint64_t>(),
                                    ctx->len.as<uint32_t>(), len, opt->k, opt->w, true, mo))
        return r;
    if (int r = stage(1)) return r;
    // 2. seed hits on both strands
    tmap::MatchOut& mt = ctx->match;
    if (int r = tmap::match_device(ctx, n_reads, mo, idx->fwd.view(), idx->rev.view(), opt->fastq_rules, mt)) return r;
    if (int r = stage(2)) return r;
    // 3. FindLIS per (read, strand)
    const uint32_t n_lists = 2 * n_reads;
    TM_HIP(ctx, ctx->c_out.reserve(n_lists * 20ull));
    if (int r = tmap::chain_device(ctx, n_lists, mt.list_off.as<uint64_t>(), mt.tot_f + mt.tot_r, mt.hf.as<uint32_t>(),
                                 mt.hr.as<uint32_t>(), ctx->c_out.as<uint32_t>()))
        return r;
    std::vector<uint32_t> ch(5ull * n_lists);
    TM_HIP(ctx, hipMemcpyAsync(ch.data(), ctx->c_out.p, n_lists * 20ull, hipMemcpyDeviceToHost, s));
    TM_HIP(ctx, hipStreamSynchronize(s));
    if (int r = stage(3)) return r;
    // 4. windows (team_mapper.cpp:650-663)
    const uint32_t k = opt->k;
    std::vector<uint32_t> pair_read, ql, tl;
    std::vector<uint64_t> qo, to;
    for (uint32_t r = 0; r < n_reads; ++r) {
        const uint32_t* cf = &ch[5ull * r];
        const uint32_t* cr = &ch[5ull * (n_reads + r)];
        const bool fwd = cf[0] >= cr[0];
        const uint32_t* c = fwd ? cf : cr;
        mapped[r] = c[0] != 0;
        strand_fwd[r] = fwd;
        score[r] = 0;
        if (opt->want_cigar) cigar_len[r] = 0;
        if (!c[0]) {
            q_begin[r] = q_end[r] = t_begin[r] = t_end[r] = 0;
            continue;
        }
        q_begin[r] = c[1] - 1;
        q_end[r] = c[3] + k - 2;
        t_begin[r] = c[2] - 1;
        t_end[r] = c[4] + k - 2;
        pair_read.push_back(r);
        ql.push_back(q_end[r] - q_begin[r] + 1);
        tl.push_back(t_end[r] - t_begin[r] + 1);
        qo.push_back(off[r] + q_begin[r]);
        to.push_back((fwd ? 0 : idx->len) + t_begin[r]);
    }
    // 5. one alignment batch over all windows (libteam_alignment plan, device-resident)
    const uint32_t P = (uint32_t)pair_read.size();
    if (!P) return TM_OK;
    ta_plan* plan = nullptr;
    // the mapper owns the device: its code workspace may take most of the free
    // HBM (fewer, fuller chunks for long reads; the library default is half,
    // <= 64 GiB).  Memory the alignment context already holds from the last
    // batch is reused, so it counts as free.
    size_t free_b = 0, total_b = 0;
    const uint64_t budget = hipMemGetInfo(&free_b, &total_b) == hipSuccess
                                ? ((uint64_t)free_b + ta_context_held_bytes(ctx->ta)) / 100 * 85
                                : 0;
    int rc = ta_plan_create(ctx->ta, P, ql.data(), tl.data(), opt->type, opt->match, opt->mismatch, opt->gap,
                            opt->want_cigar, budget, 0, &plan);
    if (rc != TA_OK) return fail(ctx, rc == TA_ERR_BAD_TYPE ? TM_ERR_BAD_TYPE : TM_ERR_DEVICE,
                                 std::string("ta_plan_create: ") + ta_last_error(ctx->ta));
    const uint64_t slots = ta_plan_cigar_slots_bytes(plan);
    auto run = [&]() -> int {
        TM_HIP(ctx, ctx->m_qoff.reserve(P * 8ull));
        TM_HIP(ctx, ctx->m_toff.reserve(P * 8ull));
        TM_HIP(ctx, ctx->m_score.reserve(P * 4ull));
        TM_HIP(ctx, ctx->m_tb.reserve(P * 4ull));
        TM_HIP(ctx, ctx->m_cstart.reserve(P * 8ull));
        TM_HIP(ctx, ctx->m_clen.reserve(P * 4ull));
        TM_HIP(ctx, ctx->m_slots.reserve(slots + 1));
        TM_HIP(ctx, hipMemcpyAsync(ctx->m_qoff.p, qo.data(), P * 8ull, hipMemcpyHostToDevice, s));
        TM_HIP(ctx, hipMemcpyAsync(ctx->m_toff.p, to.data(), P * 8ull, hipMemcpyHostToDevice, s));
        ta_device_io io{};
        io.query_bytes = ctx->bytes.as<const char>();
        io.query_off = ctx->m_qoff.as<const uint64_t>();
        io.target_bytes = idx->ref2.as<const char>();
        io.target_off = ctx->m_toff.as<const uint64_t>();
        io.score = ctx->m_score.as<int32_t>();
        io.target_begin = ctx->m_tb.as<uint32_t>();
        io.cigar_slots = ctx->m_slots.as<char>();
        io.cigar_start = ctx->m_cstart.as<uint64_t>();
        io.cigar_len = ctx->m_clen.as<uint32_t>();
        if (int r = stage(4)) return r;
        if (int r = ta_plan_execute(plan, &io, s))
            return fail(ctx, TM_ERR_DEVICE, std::string("ta_plan_execute: ") + ta_last_error(ctx->ta) + " (" +
                                                ta_status_string(r) + ")");
        if (int r = stage(5)) return r;
        std::vector<int32_t> sc(P);
        TM_HIP(ctx, hipMemcpyAsync(sc.data(), ctx->m_score.p, P * 4ull, hipMemcpyDeviceToHost, s));
        std::vector<uint64_t> co;
        uint64_t total = 0;
        if (opt->want_cigar) {
            // pack the CIGAR slots on the device, then copy only the CIGAR bytes
            if (int r = tmap::compact_segments(ctx, P, ctx->m_slots.as<const char>(), ctx->m_cstart.as<const uint64_t>(),
                                               ctx->m_clen.as<const uint32_t>(), ctx->m_coff, ctx->m_cdst,
                                               ctx->match.cub_tmp, total))
                return r;
            if (total > arena_bytes) return fail(ctx, TM_ERR_CAPACITY, "cigar arena too small");
            co.resize(P + 1);
            TM_HIP(ctx, hipMemcpyAsync(co.data(), ctx->m_coff.p, (P + 1) * 8ull, hipMemcpyDeviceToHost, s));
            if (total) TM_HIP(ctx, hipMemcpyAsync(arena, ctx->m_cdst.p, total, hipMemcpyDeviceToHost, s));
        }
        TM_HIP(ctx, hipStreamSynchronize(s));
        if (int r = ta_plan_check(plan))
            return fail(ctx, TM_ERR_DEVICE, std::string("ta_plan_check: ") + ta_last_error(ctx->ta) + " (" +
                                                ta_status_string(r) + ")");
        for (uint32_t p = 0; p < P; ++p) {
            const uint32_t r = pair_read[p];
            score[r] = sc[p];
            if (!opt->want_cigar) continue;
            cigar_off[r] = co[p];
            cigar_len[r] = (uint32_t)(co[p + 1] - co[p]);
        }
        return TM_OK;
    };
    ctx->plan_stats[0] = P;
    ctx->plan_stats[1] = ta_plan_chunks(plan);
    ctx->plan_stats[2] = ta_plan_dual_pairs(plan);
    ctx->plan_stats[3] = ta_plan_flex_pairs(plan);
    ctx->plan_stats[4] = ta_plan_workspace_bytes(plan);
    rc = run();
    ta_plan_destroy(plan);
    if (rc == TM_OK) rc = stage(6);
    ctx->stage_cells = 0;
    for (uint32_t p = 0; p < P; ++p) ctx->stage_cells += (uint64_t)ql[p] * tl[p];
    return rc;
}

int tm_stage_times(const tm_context* ctx, double* ms, uint32_t n, uint64_t* aligned_cells) {
    if (!ctx || (n && !ms)) return TM_ERR_ARG;
    for (uint32_t i = 0; i < n && i < (uint32_t)tmap::kStages; ++i) ms[i] = ctx->stage_ms[i];
    if (aligned_cells) *aligned_cells = ctx->stage_cells;
    return TM_OK;
}

int tm_align_plan_stats(const tm_context* ctx, uint64_t out[5]) {
    if (!ctx || !out) return TM_ERR_ARG;
    for (int i = 0; i < 5; ++i) out[i] = ctx->plan_stats[i];
    return TM_OK;
}

int tm_map_files(const char* reference_path, const char* reads_path, const tm_options* opt, const char* out_path,
                 int device) {
    if (!reference_path || !reads_path || !opt || !out_path) return TM_ERR_ARG;
    tmap::FastxFile ref, reads;
    std::string err;
    if (!tmap::read_fastx(reference_path, false, ref, err) || ref.records.empty()) {
        std::fprintf(stderr, "%s\n", err.empty() ? "reference: no sequences" : err.c_str());
        return TM_ERR_INPUT;
    }
    // fragments: FASTQ first, FASTA when that fails (team_mapper.cpp:533-556)
    bool fastq = tmap::read_fastx(reads_path, true, reads, err);
    if (!fastq && !tmap::read_fastx(reads_path, false, reads, err)) {
        std::fprintf(stderr, "Given file is not in FASTA or FASTQ format! \n");
        return TM_ERR_INPUT;
    }
    tm_context* ctx = nullptr;
    if (int r = tm_context_create(device, &ctx)) return r;
    const tmap::FastxRecord& R = ref.records.front();
    tm_index* idx = nullptr;
    int rc = tm_index_create(ctx, R.name.c_str(), ref.seq.data() + R.off, R.len, opt->k, opt->w, opt->f, &idx);
    if (rc) {
        std::fprintf(stderr, "index: %s: %s\n", tm_status_string(rc), tm_last_error(ctx));
        tm_context_destroy(ctx);
        return rc;
    }
    FILE* out = std::strcmp(out_path, "-") == 0 ? stdout : std::fopen(out_path, "wb");
    if (!out) {
        tm_index_destroy(idx);
        tm_context_destroy(ctx);
        return TM_ERR_INPUT;
    }
    tm_options o = *opt;
    o.fastq_rules = fastq ? 1 : 0;
    const size_t n = reads.records.size();
    const uint64_t kBatchBases = 1ull << 30;  // reads per device batch: up to ~1 Gbase
    std::string line;
    for (size_t b = 0; b < n && rc == TM_OK;) {
        size_t e = b;
        uint64_t bases = 0;
        while (e < n && (e == b || bases + reads.records[e].len <= kBatchBases)) bases += reads.records[e++].len;
        const uint32_t nr = (uint32_t)(e - b);
        std::vector<uint64_t> off(nr);
        std::vector<uint32_t> len(nr);
        const uint64_t base = reads.records[b].off;
        uint64_t arena_bytes = 0;
        for (uint32_t i = 0; i < nr; ++i) {
            off[i] = reads.records[b + i].off - base;
            len[i] = (uint32_t)reads.records[b + i].len;
            arena_bytes += 4ull * len[i] + 2;
        }
        std::vector<uint8_t> mapped(nr), fwd(nr);
        std::vector<uint32_t> qb(nr), qe(nr), tb(nr), te(nr), cl(nr);
        std::vector<int32_t> sc(nr);
        std::vector<uint64_t> co(nr);
        std::vector<char> arena(o.want_cigar ? arena_bytes : 0);
        rc = tm_map_batch(ctx, idx, nr, reads.seq.data() + base, off.data(), len.data(), &o, mapped.data(), fwd.data(),
                          qb.data(), qe.data(), tb.data(), te.data(), sc.data(), arena.data(), arena.size(), co.data(),
                          cl.data());
        if (rc) {
            std::fprintf(stderr, "map: %s: %s\n", tm_status_string(rc), tm_last_error(ctx));
            break;
        }
        for (uint32_t i = 0; i < nr; ++i) {
            if (!mapped[i]) continue;
            const tmap::FastxRecord& q = reads.records[b + i];
            // team_mapper.cpp:686-697; reverse-strand windows reported in forward coordinates
            const uint64_t L = idx->len;
            const uint64_t ts = fwd[i] ? tb[i] : L - te[i] - 1, tend = fwd[i] ? (uint64_t)te[i] + 1 : L - tb[i];
            line.clear();
            line += q.name;
            line += '\t' + std::to_string(q.len) + '\t' + std::to_string(qb[i]) + '\t' + std::to_string(qe[i] + 1ull);
            line += fwd[i] ? "\t+\t" : "\t-\t";
            line += idx->name + '\t' + std::to_string(L) + '\t' + std::to_string(ts) + '\t' + std::to_string(tend);
            line += '\t' + std::to_string(sc[i]) + '\t' + std::to_string(qe[i] - qb[i] + 1ull) + "\t60";
            if (o.want_cigar) {
                line += "\tcg:Z:";
                line.append(arena.data() + co[i], cl[i]);
            }
            line += '\n';
            std::fwrite(line.data(), 1, line.size(), out);
        }
        b = e;
    }
    if (out != stdout) std::fclose(out);
    else std::fflush(stdout);
    tm_index_destroy(idx);
    tm_context_destroy(ctx);
    return rc;
}

}  // extern "C"
