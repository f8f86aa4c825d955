/*
 * include/team_mapper_c.h -- extern "C" ABI of the MI355X mapper stages that
 * sit either side of team::Align: minimizer sketches on the
 * GPU, the reference minimizer index, seed matching + chaining on the GPU,
 * and the batched mapper driver that feeds the alignment batch ABI
 * (team_align_c.h) and writes the reference's PAF-like lines.
 * Library: libteam_mapper.so (links libteam_alignment.so).
 *
 * Reference interfaces replaced (paths relative to /root/reference):
 *   team::KMER::Minimize              team_minimizers/team_minimizers.cpp:122-225
 *   remove_duplicates                 team_mapper.cpp:26-42
 *   reference index + frequency ban   team_mapper.cpp:406-471
 *   seed matching                     team_mapper.cpp:631-646, 718-731
 *   FindLIS (chaining)                team_mapper.cpp:283-316
 *   window -> Align -> PAF line       team_mapper.cpp:650-697, 733-789
 *   FASTA/FASTQ input (bioparser)     team_mapper.cpp:401-402, 529-556
 *
 * Plain pointers and sizes; nothing throws; every function returns a TM_*
 * status (the same numbering as TA_* in team_align_c.h).
 *
 * Product limits (the reference accepts more but hashes nonsense there):
 * 1 <= k <= 15 (2-bit codes in 30 bits, so no window can hold only the
 * UINT_MAX sentinel of GetTupleWithMinFirst), 1 <= w <= 64.
 */
#ifndef TEAM_MAPPER_C_H
#define TEAM_MAPPER_C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TM_OK 0
#define TM_ERR_BAD_TYPE 1 /* Unknown AlignmentType provided. */
#define TM_ERR_ARG 3      /* null pointer / unsupported k or w / inconsistent sizes */
#define TM_ERR_DEVICE 4   /* no usable gfx950 device or a HIP failure (tm_last_error) */
#define TM_ERR_CAPACITY 5 /* caller buffer too small */
#define TM_ERR_INPUT 6    /* unreadable file / not FASTA or FASTQ */

typedef struct tm_context tm_context; /* device + stream + grow-only scratch */
typedef struct tm_index tm_index;     /* reference (both strands) + minimizer index, in HBM */

const char* tm_status_string(int status);
const char* tm_last_error(const tm_context* ctx);
int tm_context_create(int device, tm_context** out);
void tm_context_destroy(tm_context* ctx);

/* Upper bound on the minimizers KMER::Minimize emits for one sequence of
 * length len: (w-1) leading end-minimizers + one per full window + up to
 * (w-1) trailing end-minimizers (team_minimizers.cpp:146-222). */
uint64_t tm_minimizer_bound(uint32_t len, uint32_t k, uint32_t w);

/*
 * Minimizers of n_seqs sequences (host memory in and out): for sequence s the
 * (hash, 1-based position) list KMER::Minimize returns, in its order, at
 * out_hash/out_pos[out_off[s] .. out_off[s+1]).  With dedup != 0 only the
 * first occurrence of each (hash, position) is kept -- the fragment-side
 * remove_duplicates (team_mapper.cpp:26-42).  The strand of every entry is
 * is_fwd (the KMER object's flag), so it is not returned.  cap = capacity of
 * out_hash/out_pos; sum of tm_minimizer_bound always suffices.
 */
int tm_minimize_batch(tm_context* ctx, uint32_t n_seqs, const char* bytes, const uint64_t* off, const uint32_t* len,
                      uint32_t k, uint32_t w, int dedup, uint64_t* out_off, uint32_t* out_hash, uint32_t* out_pos,
                      uint64_t cap);

/*
 * Chaining (FindLIS, team_mapper.cpp:283-316) of n_lists seed-hit lists on the
 * GPU: list l is (fpos, rpos)[off[l] .. off[l+1]) in list order.  Outputs per
 * list: chain length, and its first and last hit (the only parts the mapper
 * uses: team_mapper.cpp:650-663).  Empty list -> length 0.
 */
int tm_chain_batch(tm_context* ctx, uint32_t n_lists, const uint64_t* off, const uint32_t* fpos, const uint32_t* rpos,
                   uint32_t* chain_len, uint32_t* first_f, uint32_t* first_r, uint32_t* last_f, uint32_t* last_r);

/*
 * Reference index (team_mapper.cpp:398-471): the first record of a FASTA
 * reference and its reverse complement, their minimizers (GPU), the
 * frequency ban of the f-fraction most frequent hashes with the reference's
 * own tie order and quirks (both thresholds from the reverse strand's unique
 * count; the reverse ban list drawn from the forward ranking), and the
 * surviving (hash -> ascending positions) tables of both strands, in HBM.
 */
int tm_index_create(tm_context* ctx, const char* name, const char* seq, uint64_t len, uint32_t k, uint32_t w,
                    double f, tm_index** out);
void tm_index_destroy(tm_index* idx);
/* Forward-strand hashes / reverse-strand hashes in the index, and banned counts. */
int tm_index_stats(const tm_index* idx, uint64_t* fwd_keys, uint64_t* rev_keys, uint64_t* fwd_positions,
                   uint64_t* rev_positions, uint32_t* banned_fwd, uint32_t* banned_rev);

/* Mapping options: team_mapper.cpp:321-387 (-a -m -n -g -k -w -f -c). */
typedef struct tm_options {
    int type; /* TA_GLOBAL / TA_LOCAL / TA_SEMI_GLOBAL (default global, as the reference CLI) */
    int match, mismatch, gap;
    uint32_t k, w;
    double f;
    int want_cigar;        /* -c */
    int fastq_rules;       /* 1: reverse hits independent of forward hits (FASTQ path, :718-731);
                              0: only for hashes in the forward index (FASTA path, :631-646) */
} tm_options;

/*
 * Map n_reads reads (host SoA) against an index: per read minimizers (GPU,
 * deduplicated), seed hits on both strands, FindLIS chains (GPU), windows,
 * one batched team::Align plan (libteam_alignment), results back.  Per read:
 * mapped[r] (0 when both chains are empty: no line), strand_fwd, the query
 * window [q_begin, q_end] and target window [t_begin, t_end] in the chain's
 * strand coordinates (team_mapper.cpp:660-663), score, and when want_cigar
 * the CIGAR bytes at cigar_arena[cigar_off[r] .. + cigar_len[r]).
 * cigar_arena_bytes: capacity; the sum over reads of 2*(2*len)+2 suffices.
 */
int tm_map_batch(tm_context* ctx, const tm_index* idx, uint32_t n_reads, const char* bytes, const uint64_t* off,
                 const uint32_t* len, const tm_options* opt, uint8_t* mapped, uint8_t* strand_fwd, uint32_t* q_begin,
                 uint32_t* q_end, uint32_t* t_begin, uint32_t* t_end, int32_t* score, char* cigar_arena,
                 uint64_t cigar_arena_bytes, uint64_t* cigar_off, uint32_t* cigar_len);

/* Wall time (ms) of the last tm_map_batch on this context, per stage:
 * [0] read upload, [1] minimizers, [2] seed matching, [3] FindLIS chaining,
 * [4] windows + alignment plan (host), [5] alignment (fill + traceback),
 * [6] results to host, [7] total; and the DP cells the alignment batch
 * covered.  Stages are separated by stream synchronisations. */
int tm_stage_times(const tm_context* ctx, double* ms, uint32_t n, uint64_t* aligned_cells);

/* The alignment plan of the last tm_map_batch: out[0] pairs, [1] chunks,
 * [2] pairs on the packed int16 fills (dual + flexible), [3] pairs on the
 * flexible fill, [4] code workspace bytes (ta_plan_* of libteam_alignment). */
int tm_align_plan_stats(const tm_context* ctx, uint64_t out[5]);

/*
 * The whole mapper on files (the reference's main, team_mapper.cpp:319-796):
 * reference FASTA (first record) and reads (FASTQ, else FASTA; plain or
 * gzip), PAF-like lines written to out_path ("-" = stdout) in read order.
 */
int tm_map_files(const char* reference_path, const char* reads_path, const tm_options* opt, const char* out_path,
                 int device);

#ifdef __cplusplus
}
#endif

#endif /* TEAM_MAPPER_C_H */
