/*
 * include/team_align_c.h -- extern "C" batch ABI of the MI355X team_alignment
 * engine (libteam_alignment.so).
 *
 * This is the boundary the reference's Align() path is replaced behind.  The
 * reference exposes one C++ entry, team::Align
 * (/root/reference/team_alignment/team_alignment.hpp:14-23, implemented at
 * team_alignment.cpp:49-350), called once per read by team_mapper.cpp:666,
 * 674, 755, 763.  Each function below states which part of that interface it
 * replaces.  Plain pointers and sizes only; no C++ or torch types; nothing
 * throws.  Every function returns a TA_* status.
 *
 * Semantics per pair are exactly team::Align's:
 *   score        -- the int the reference returns
 *   target_begin -- what the reference writes to *target_begin
 *                   (0 for global/semiGlobal, end column + 1 for local)
 *   CIGAR        -- the bytes the reference assigns to *cigar: decimal run
 *                   lengths of M / I (consumes target) / D (consumes query);
 *                   an empty alignment is the 2-byte string "1\0".
 */
#ifndef TEAM_ALIGN_C_H
#define TEAM_ALIGN_C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* team::AlignmentType values (team_alignment.hpp:8-12). */
#define TA_GLOBAL 0
#define TA_LOCAL 1
#define TA_SEMI_GLOBAL 2

/* Status codes. */
#define TA_OK 0
#define TA_ERR_BAD_TYPE 1 /* reference: std::invalid_argument("Unknown AlignmentType provided.") */
#define TA_ERR_CIGAR 2    /* reference: std::invalid_argument("Unknown error in determining cigar string.") */
#define TA_ERR_ARG 3      /* null pointer / inconsistent sizes */
#define TA_ERR_DEVICE 4   /* no usable gfx950 device or a HIP runtime failure (see ta_last_error) */
#define TA_ERR_CAPACITY 5 /* caller-provided CIGAR arena too small */

typedef struct ta_context ta_context; /* device + stream + cached buffers; one per host thread */
typedef struct ta_plan ta_plan;       /* a batch's lengths, scoring and device workspace layout */

/* Message for a status code (static storage). */
const char* ta_status_string(int status);
/* Last error detail recorded on this context (e.g. the HIP error string). */
const char* ta_last_error(const ta_context* ctx);

/* Create a context on HIP device `device` (gfx950 required).  Replaces nothing
 * in the reference (which has no device state); team::Align keeps one per
 * calling thread so concurrent callers (team_mapper.cpp:596 OpenMP) are safe. */
int ta_context_create(int device, ta_context** out);
void ta_context_destroy(ta_context* ctx);
/* Free the context's cached device workspace and staging buffers (they are
 * grow-only: a large batch keeps its traceback-code workspace for the next
 * one).  Waits for the context's last execution.  The context stays usable. */
void ta_context_release(ta_context* ctx);

/* Device bytes the context holds in its grow-only traceback-code and
 * pass-boundary workspace -- the memory a plan's chunks reuse.  A caller sizing
 * ta_plan_create's workspace budget from hipMemGetInfo adds this back: the free
 * figure does not count memory the context will reuse.  (Staging and output
 * buffers are not included: a plan cannot reuse them.) */
uint64_t ta_context_held_bytes(const ta_context* ctx);

/* ---- Low-latency single pairs (the drop-in team::Align's path for calls that
 * fit).  Replaces team::Align's per-call synchronous computation
 * (team_alignment.cpp:49-56) as called by team_mapper.cpp:666-678 / 755-767:
 * a persistent kernel (one wave per slot) serves pairs posted in pinned host
 * memory, so a call costs no kernel launch and no copy.  One server per
 * (device, alignment type); its kernel starts with the first call and stops
 * after ~200 ms without calls.  Thread-safe: concurrent callers take
 * different slots. */
typedef struct ta_server ta_server;
int ta_server_create(int device, int type, uint32_t slots, ta_server** out); /* slots 1..64 */
void ta_server_destroy(ta_server* server);
/* 1 when an n x m pair with these scores runs on the server (n <= 4096,
 * m <= 16384; local mode: (n + m) * max|score| < 2^25). */
int ta_server_fits(const ta_server* server, uint32_t query_len, uint32_t target_len, int match, int mismatch,
                   int gap);
/* One pair, synchronous, team::Align's results (score, target_begin, the CIGAR
 * bytes when want_cigar).  TA_ERR_UNSERVED when the pair does not fit or no
 * slot is free: use ta_align_batch instead. */
int ta_server_align(ta_server* server, const char* query, uint32_t query_len, const char* target,
                    uint32_t target_len, int match, int mismatch, int gap, int want_cigar, int32_t* score,
                    uint32_t* target_begin, char* cigar, uint64_t cigar_capacity, uint32_t* cigar_len);
/* 1 while the server's kernel is resident. */
int ta_server_running(const ta_server* server);
/* Pause / resume (counted).  While paused, ta_server_align returns
 * TA_ERR_UNSERVED at once; ta_server_pause waits for the calls in flight and
 * stops the kernel, so that work on other streams of the device never queues
 * behind the persistent kernel on a shared hardware queue (a batch on the same
 * device pauses the server around its launches).  Pausing a server that is not
 * running only counts; the drop-in shim pauses its own servers around each
 * combined batch.  Work submitted outside the shim (ta_align_batch, plans, the
 * mapper) does not pause anything: a caller that mixes it with a live server on
 * one device pauses the server itself for the duration. */
int ta_server_pause(ta_server* server);
int ta_server_resume(ta_server* server);
/* Diagnostics: the device-side phase times (microseconds) of the last request
 * served in `slot`: [0] request + bytes into HBM, [1] fill + walk, [2] results
 * and CIGAR into the slot, [3] 0 (the release store of `done` is the fence). */
int ta_server_last_times(const ta_server* server, uint32_t slot, double* us_out4);

/* The drop-in team::Align (include/team_alignment.hpp) runs each call on:
 * the device set here (device >= 0; -1 clears the choice), else the device
 * named by the TEAM_ALIGN_DEVICE environment variable (read once), else the
 * calling thread's current HIP device (hipSetDevice) as of that thread's first
 * call (a thread keeps it: hipGetDevice per call would cost more than a small
 * pair's alignment).  TA_ERR_ARG for a device that does not exist. */
int ta_set_default_device(int device);
/* The calling thread's own choice, ahead of the three above: its drop-in calls
 * run on `device` (>= 0).  -1 drops the choice and makes the thread's next
 * call read its current HIP device again -- the call to make after a
 * hipSetDevice that should move the thread's team::Align calls with it.
 * TA_ERR_ARG for a device that does not exist. */
int ta_set_thread_device(int device);
/* The calling thread's current HIP device (0 when it has none) and the number of devices. */
int ta_current_device(void);
int ta_device_count(void);

/* Bytes of the per-pair CIGAR slot for an n x m pair: 2*(n+m)+2, an upper
 * bound on any run-length CIGAR of that pair (team_alignment.cpp:145-160). */
uint64_t ta_cigar_slot_bytes(uint32_t query_len, uint32_t target_len);

/*
 * Host-memory batch: the batched form of team::Align
 * (team_alignment.hpp:14-23), n_pairs independent calls with shared
 * type/match/mismatch/gap.  Inputs are SoA: concatenated bytes + per-pair
 * offset + length (length-delimited, not NUL-terminated, as Align takes them).
 * Outputs (host memory, n_pairs each): score[], target_begin[] (either may be
 * NULL, like Align's optional pointer), and when want_cigar != 0 the CIGARs
 * packed back to back into cigar_arena (capacity cigar_arena_bytes; at most
 * the sum of ta_cigar_slot_bytes is ever needed), pair p's bytes at
 * cigar_arena[cigar_off[p] .. cigar_off[p]+cigar_len[p]).
 * want_cigar == 0 is the reference's cigar == nullptr mode: no traceback.
 * Returns TA_ERR_BAD_TYPE for an unknown type (no pair is computed).
 * No device allocation per call once the context's grow-only buffers fit the
 * batch: per call one pinned upload of the plan arrays, offsets and (up to
 * 4 MB) sequences, the kernels, the downloads, one or two synchronisations.
 * Caller buffers may be pageable or pinned (pinned ones, e.g. allocated with
 * hipHostMalloc, transfer at full PCIe rate).
 */
int ta_align_batch(ta_context* ctx, uint32_t n_pairs, const char* query_bytes, const uint64_t* query_off,
                   const uint32_t* query_len, const char* target_bytes, const uint64_t* target_off,
                   const uint32_t* target_len, int type, int match, int mismatch, int gap, int want_cigar,
                   int32_t* score, uint32_t* target_begin, char* cigar_arena, uint64_t cigar_arena_bytes,
                   uint64_t* cigar_off, uint32_t* cigar_len);

/* ta_align_batch with plan flags (TA_PLAN_* below: kernel selection, e.g.
 * TA_PLAN_INT32_ONLY for one int32 wave per pair with its walk inside the
 * fill kernel).  Results are identical for every flag value. */
int ta_align_batch_flags(ta_context* ctx, uint32_t n_pairs, const char* query_bytes, const uint64_t* query_off,
                         const uint32_t* query_len, const char* target_bytes, const uint64_t* target_off,
                         const uint32_t* target_len, int type, int match, int mismatch, int gap, int want_cigar,
                         int32_t* score, uint32_t* target_begin, char* cigar_arena, uint64_t cigar_arena_bytes,
                         uint64_t* cigar_off, uint32_t* cigar_len, uint32_t flags);

/*
 * Device-resident batches (the mapper-side batching of SURVEY §8f and the
 * benchmark path).  A plan fixes the lengths (host arrays, copied) and the
 * scoring, lays out the device workspace (2-bit traceback pointers, pass
 * boundary rows) and chunks the batch when the pointer matrices exceed
 * workspace_budget bytes (0 = library default: half the free HBM, at most
 * 64 GiB).  flags: 0, or TA_PLAN_* below (kernel selection for tests and
 * measurements; results are identical either way).
 */
#define TA_PLAN_INT32_ONLY 1u /* no packed two-pairs-per-wave int16 kernels */
#define TA_PLAN_NO_FLEX 2u    /* no rebased couples of different shapes */
#define TA_PLAN_UNFUSED 4u    /* int32-only plans: traceback as its own kernel, not inside the fill */
#define TA_PLAN_WALK1 8u      /* local tracebacks: one pair per wave (run walk) */
#define TA_PLAN_WALK2 16u     /* local tracebacks: two pairs per wave (run walk), not one lane per pair */
#define TA_PLAN_SERIAL_PASSES 32u /* int32 fill: one wave sweeps all of a pair's passes (no pass pipelining) */
#define TA_PLAN_PASS_MAJOR 64u    /* pass-pipelined fills: tickets start-aligned (every pass 0 first), not end-aligned */
#define TA_PLAN_NO_BLK 128u       /* local plans of equal-shape couples: keep the [step][lane] code layout and the
                                     lane walks instead of the blocked layout and the band walks */
#define TA_PLAN_NO_CK 256u        /* those plans: the fill writes blocked codes walked by the band walks, never
                                     checkpoints walked by the recomputing walks (the default for large batches) */
#define TA_PLAN_CK 512u           /* those plans: checkpoints and recomputing walks at any batch size */
#define TA_PLAN_NO_FLEX_CK 1024u  /* plans with couples of different shapes: codes and the code walks, not checkpoints */
int ta_plan_create(ta_context* ctx, uint32_t n_pairs, const uint32_t* query_len_host,
                   const uint32_t* target_len_host, int type, int match, int mismatch, int gap, int want_cigar,
                   uint64_t workspace_budget, uint32_t flags, ta_plan** out);
void ta_plan_destroy(ta_plan* plan);
/* Total bytes of the device CIGAR slot arena the caller must provide. */
uint64_t ta_plan_cigar_slots_bytes(const ta_plan* plan);
/* Device workspace a plan's execution grows in its context (codes or checkpoints,
 * pass-boundary rows and the walks' event words), and the number of launch chunks. */
uint64_t ta_plan_workspace_bytes(const ta_plan* plan);
uint32_t ta_plan_chunks(const ta_plan* plan);
/* Pairs the plan runs in the packed two-pairs-per-wave int16 kernels (equal
 * shapes with scores provably within int16, or -- global / semi-global --
 * couples of different shapes in the rebased kernel); the rest use the int32
 * kernel. */
uint32_t ta_plan_dual_pairs(const ta_plan* plan);
/* Of those, the pairs in couples of different shapes / beyond int16 (ta_flex.hip). */
uint32_t ta_plan_flex_pairs(const ta_plan* plan);
/* 1 when the fill kernel walks its own pair (int32-only plans with CIGAR on). */
int ta_plan_fused(const ta_plan* plan);
/* The plan's walk (diagnostics, tests): local walk kind in bits 7:0 (64 band walks,
 * one lane per pair; 32 two pairs per wave; 16 lane walks; 0 one pair per wave),
 * bit 8 set when the codes use the blocked layout, bit 9 when the fill leaves
 * checkpoints instead and the walk recomputes codes around its path. */
int ta_plan_walk(const ta_plan* plan);
/* chunk_of_pair[p] = the chunk (0 .. ta_plan_chunks-1) whose launches align pair p
 * (caller-allocated, n_pairs entries).  Diagnostics: which chunk a checked pair ran in. */
int ta_plan_pair_chunks(const ta_plan* plan, uint32_t* chunk_of_pair);

/* Device pointers for one execution of a plan. */
typedef struct ta_device_io {
    const char* query_bytes;      /* device */
    const uint64_t* query_off;    /* device, n_pairs */
    const char* target_bytes;     /* device */
    const uint64_t* target_off;   /* device, n_pairs */
    int32_t* score;               /* device, n_pairs */
    uint32_t* target_begin;       /* device, n_pairs */
    char* cigar_slots;            /* device, ta_plan_cigar_slots_bytes(); unused when !want_cigar */
    uint64_t* cigar_start;        /* device, n_pairs: pair p's CIGAR starts at cigar_slots[cigar_start[p]] */
    uint32_t* cigar_len;          /* device, n_pairs */
} ta_device_io;

/* Enqueue the whole batch on `hip_stream` (a hipStream_t; NULL = the HIP
 * null stream, as everywhere in HIP).  Asynchronous: returns after enqueueing.
 * Plans of one context share its workspace: an execution on a different
 * stream than the context's previous one waits for that one first. */
int ta_plan_execute(ta_plan* plan, const ta_device_io* io, void* hip_stream);

/* After the plan's executions have completed (stream synchronised): TA_OK, or
 * TA_ERR_DEVICE when a kernel reported an internal failure since the last
 * check (the flexible fill's bounded pass hand-off poll gave up; see
 * ta_last_error).  Clears the flag.  ta_align_batch checks it itself. */
int ta_plan_check(ta_plan* plan);

/* Enqueue only the DP fill (scores/target_begin; traceback pointers into the
 * workspace) or only the traceback, for profiling the two kernels. */
int ta_plan_execute_fill(ta_plan* plan, const ta_device_io* io, void* hip_stream, uint32_t chunk);
int ta_plan_execute_traceback(ta_plan* plan, const ta_device_io* io, void* hip_stream, uint32_t chunk);

/* Pack n_pairs CIGARs from their slots (device: cigar_slots, cigar_start,
 * cigar_len as written by an execution) back to back into dst (device):
 * pair p's bytes go to dst[dst_off[p] ..).  Enqueued on hip_stream.  For a
 * caller that gathers CIGAR bytes between GPUs (bench.py's RCCL gather) or
 * downloads them.  The reference has no counterpart (one std::string per
 * team::Align call, team_alignment.cpp:160). */
int ta_compact_cigars(ta_context* ctx, uint32_t n_pairs, const char* cigar_slots, const uint64_t* cigar_start,
                      const uint32_t* cigar_len, const uint64_t* dst_off, char* dst, void* hip_stream);

/*
 * ---- Affine-gap extension (BASELINE config 5: "affine gaps + full CIGAR
 * traceback").  The reference has NO counterpart: team::Align is linear-gap
 * only (team_alignment.cpp:25-28, 102-116; the "Gotoh" of
 * team_alignment.hpp:11 is a label).  The semantics are defined in
 * oracle/affine_oracle.c (Gotoh E/F/H, the reference's tie order, boundaries,
 * goals, traceback and CIGAR format); a gap of length L costs
 * gap_open + L * gap_extend and a '-' byte makes its gap step free.  With
 * gap_open == 0 the results are byte-identical to team::Align with
 * gap = gap_extend (that part of parity is pinned to the reference goldens;
 * gap_open != 0 is unpinned).
 * Range: (max qlen + max tlen + 2) * max(|match|, |mismatch|,
 * |gap_open| + |gap_extend|) must be < 2^26, else TA_ERR_RANGE.
 */
#define TA_ERR_RANGE 6 /* affine scoring x lengths outside the int32-safe range */
#define TA_ERR_UNSERVED 7 /* ta_server_align: the pair is outside the server's limits, or every slot is busy */

typedef struct ta_affine_plan ta_affine_plan;

/* As ta_plan_create, with the affine scoring.  Traceback codes take 4 bits per
 * cell (source M/I/D/STOP + the E and F extension bits).  flags:
 * TA_PLAN_INT32_ONLY or 0. */
int ta_affine_plan_create(ta_context* ctx, uint32_t n_pairs, const uint32_t* query_len_host,
                          const uint32_t* target_len_host, int type, int match, int mismatch, int gap_open,
                          int gap_extend, int want_cigar, uint64_t workspace_budget, uint32_t flags,
                          ta_affine_plan** out);
void ta_affine_plan_destroy(ta_affine_plan* plan);
uint64_t ta_affine_plan_cigar_slots_bytes(const ta_affine_plan* plan);
uint64_t ta_affine_plan_workspace_bytes(const ta_affine_plan* plan);
uint32_t ta_affine_plan_chunks(const ta_affine_plan* plan);
/* Pairs the plan runs in the packed two-pairs-per-wave int16 affine fill
 * (global / semi-global couples of equal shape whose values provably fit). */
uint32_t ta_affine_plan_dual_pairs(const ta_affine_plan* plan);
int ta_affine_plan_pair_chunks(const ta_affine_plan* plan, uint32_t* chunk_of_pair);
/* Enqueue the whole batch / one chunk's fill / one chunk's traceback on hip_stream. */
int ta_affine_plan_execute(ta_affine_plan* plan, const ta_device_io* io, void* hip_stream);
int ta_affine_plan_execute_fill(ta_affine_plan* plan, const ta_device_io* io, void* hip_stream, uint32_t chunk);
int ta_affine_plan_execute_traceback(ta_affine_plan* plan, const ta_device_io* io, void* hip_stream,
                                     uint32_t chunk);
/* As ta_plan_check: TA_ERR_DEVICE when a pass hand-off poll of the packed
 * affine fill (one wave per couple and pass) gave up; clears the flag. */
int ta_affine_plan_check(ta_affine_plan* plan);

/* Host-memory batch with affine gaps: ta_align_batch with gap -> (gap_open, gap_extend). */
int ta_align_batch_affine(ta_context* ctx, uint32_t n_pairs, const char* query_bytes, const uint64_t* query_off,
                          const uint32_t* query_len, const char* target_bytes, const uint64_t* target_off,
                          const uint32_t* target_len, int type, int match, int mismatch, int gap_open,
                          int gap_extend, int want_cigar, int32_t* score, uint32_t* target_begin,
                          char* cigar_arena, uint64_t cigar_arena_bytes, uint64_t* cigar_off, uint32_t* cigar_len);

#ifdef __cplusplus
}
#endif

#endif /* TEAM_ALIGN_C_H */
