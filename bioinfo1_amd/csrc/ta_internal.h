// bioinfo1_amd/csrc/ta_internal.h -- shared layout constants and launch
// arguments between the host driver (ta_api.hip) and the kernels
// (ta_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/team_align_c.h"
#include "ta_layout.h"

namespace ta {

// 2-bit traceback code per cell, code = (D bit << 1) | I bit.  One dword per
// (pass, step, lane) holds the 16 rows of the lane's stripe as two bit
// planes: D plane in bits 31:16 (row r at bit 31 - r), I plane in bits 15:0
// (row r at bit 15 - r).  The int32 local fill stores canonical codes (M=00
// I=01 D=10 STOP=11); the other fills store the raw compares (up >
// max(diag,left), left > diag), so D wins whenever its bit is set.
enum Code : uint32_t { kCodeM = 0, kCodeI = 1, kCodeD = 2, kCodeStop = 3 };
constexpr int kDPlane = 16;  // bit offset of the D plane

struct FillArgs {
    const uint32_t* order;  // visit order (pair ids); kernel handles order[begin .. begin+count)
    uint32_t begin, count;
    const uint8_t* qbytes;
    const uint64_t* qoff;
    const uint32_t* qlen;
    const uint8_t* tbytes;
    const uint64_t* toff;
    const uint32_t* tlen;
    int match, mismatch, gap;
    uint32_t* ptrs;          // chunk workspace (2-bit codes)
    const uint64_t* ptr_off; // per pair, dwords from ptrs
    int32_t* bnd;            // chunk pass-boundary rows
    const uint64_t* bnd_off; // per pair, words from bnd
    int32_t* score;
    uint32_t* target_begin;
    uint32_t* goal_i;
    uint32_t* goal_j;
    // fused traceback (fill kernel walks its own pair right after the fill)
    int fused;
    char* slots;
    const uint64_t* slot_off;
    uint64_t* cigar_start;
    uint32_t* cigar_len;
    // dual fill: couples with a '-' query byte are handed to the int32 fill
    // through this list; that launch reads its wave count from count_dev
    uint32_t* fb_list;
    uint32_t* fb_count;
    const uint32_t* count_dev;
    // flexible fill, one wave per (couple, pass): waves take tickets in launch
    // order, so every pass a wave waits on is already held by a running wave
    const uint32_t* task_off;  // per flex couple (plan order): its first task; [w + 1] - [w] = passes
    const uint32_t* tasks;     // ticket order: couple * 64 + pass, pass-major within a chunk
    uint32_t* ticket;          // this launch's ticket counter (zeroed before the launch)
    uint32_t n_tasks;          // tasks of this launch
    uint32_t epoch;            // tag base of this launch's pass hand-off records
    uint32_t* err;             // a poll gave up (never on a correct schedule)
    void* pout;                // PassOut[2] per task (plan-global task index)
    // pipelined int32 fill (fill_pipe_kernel; task_off = per single, ticket,
    // n_tasks, err, pout = PassOut per task as above): ticket order, single << 32 | pass
    const uint64_t* tasks64;
    // multi-pass dual chunks: ticket t = level t / count of couple t % count;
    // pass = level (pass-major) or level - (chunk passes - couple passes) (end-aligned)
    uint32_t end_aligned;
    // blocked code layout (ta_layout.h blk_index): the dual fill stages 16 steps
    // in LDS and writes [block][lane][16 steps]; the int32 fill stores per step.
    // 2: the dual fill writes checkpoints instead (ta_layout.h ck_row_index; the
    // int32 fill of handed-back couples still writes blocked codes)
    uint32_t blk;
    // blk plans: per pair, 1 when its couple was handed back ('-' bytes; the
    // band walk leaves it to the fallback walk), written by the dual fill
    uint8_t* pflag;
};

// Bits of a plan's device error word (ta_plan_check, the host batches' status).
constexpr uint32_t kErrPassPoll = 1u;  // a packed fill's pass hand-off poll gave up
constexpr uint32_t kErrWalkCap = 2u;   // a band walk reached its event cap with cost left
// First event word of pair p in a band walk's workspace: its CIGAR slot's byte
// offset read as a word offset, rounded up to 4 words (16-byte stores).  Pair
// p's room is then 2 (n + m) + 2 words - the rounding >= n + m + 1 events for
// n + m >= 2 (the walk lists none for an empty pair); the workspace holds
// slots_bytes + 4 words.
__host__ __device__ inline uint64_t band_runs_off(uint64_t slot_off) { return (slot_off + 3u) & ~(uint64_t)3u; }

struct TraceArgs {
    const uint32_t* order;
    uint32_t begin, count;
    const uint32_t* qlen;
    const uint32_t* tlen;
    const uint32_t* ptrs;
    const uint64_t* ptr_off;
    const uint32_t* goal_i;
    const uint32_t* goal_j;
    char* slots;
    const uint64_t* slot_off;
    uint64_t* cigar_start;
    uint32_t* cigar_len;
    // local walks track the cost (ta_device.h WalkSeq)
    const int32_t* score;
    const uint8_t* qbytes;
    const uint64_t* qoff;
    const uint8_t* tbytes;
    const uint64_t* toff;
    int match, mismatch, gap;
    uint32_t blk;                // codes in the blocked layout (ta_layout.h blk_index); 2: checkpoints (ck_row_index)
    const uint8_t* pflag;        // band walk: pairs to leave to the fallback walk (FillArgs.pflag)
    uint32_t* runs;              // band walks: event words, pair p's at runs + band_runs_off(slot_off[p]) (format_runs_kernel)
    uint32_t* err;               // the plan's error word: band walks set kErrWalkCap
    const uint32_t* fb_order;    // band walks: the dual fill's hand-back list ('-' couples), walked after the band
    const uint32_t* fb_count;    // ... and its length (on the device)
};

struct CompactArgs {
    uint32_t n_pairs;
    const char* slots;
    const uint64_t* cigar_start;
    const uint32_t* cigar_len;
    const uint64_t* dst_off;
    char* dst;
};

// ---- the low-latency single-pair server (ta_server.cpp, serve_kernel in ta_kernels.hip)
// A persistent kernel, one wave per slot, serves team::Align calls posted in
// fine-grained pinned host memory: the host writes a request (lengths,
// scoring, sequence bytes) and bumps `seq`; the wave copies the bytes to HBM,
// fills and walks the pair (the int32 fill with its walk fused), writes the
// results and CIGAR back into the slot and sets `done = seq`.  No launch and
// no copy per call.
constexpr uint32_t kSrvQMax = 4096;       // query rows a slot takes (4 passes)
constexpr uint32_t kSrvTMax = 16384;      // target columns
constexpr uint64_t kSrvStride = 65536;    // bytes per host slot: header, query, target, CIGAR
constexpr uint64_t kSrvQOff = 128, kSrvTOff = kSrvQOff + kSrvQMax, kSrvCOff = kSrvTOff + kSrvTMax;
static_assert(kSrvCOff + 2 * (kSrvQMax + kSrvTMax) + 2 <= kSrvStride, "server slot too small");

struct ServeHdr {           // the first 128 bytes of a host slot
    uint32_t seq;            // host: number of the posted request (written last)
    uint32_t n, m;           // host: lengths
    int32_t match, mismatch, gap;
    uint32_t want_cigar;
    uint32_t pad0[9];
    uint32_t done;           // device: seq of the last finished request (written last)
    int32_t score;
    uint32_t target_begin, cigar_len, status;
    uint32_t pad1[11];       // [0..3]: the last request's phase clocks (ta_server_last_times)
};
static_assert(sizeof(ServeHdr) == kSrvQOff, "ServeHdr layout");

struct ServeCtl {            // pinned host control words shared by the slots
    uint32_t stop;           // host: the waves exit
    uint32_t heartbeat;      // host: incremented every ~1 ms while the server is wanted
    uint32_t pad[14];
};

struct ServeArgs {
    char* host;              // slot s at host + s * kSrvStride (fine-grained pinned memory)
    const ServeCtl* ctl;
    FillArgs fa;             // per-slot device arrays, pair index = slot (qlen/tlen written per request)
    uint64_t hb_timeout;     // wall-clock ticks (100 MHz) without a heartbeat before a wave exits
};

// Launchers (ta_kernels.hip).  `wide` selects the unscaled local-mode kernel
// (needed only when |scores| could reach 2^25; see run_pass SCALED).
hipError_t launch_fill(int mode, bool cigar, bool wide, const FillArgs& a, hipStream_t s);
template <int MODE, bool CIGAR>
hipError_t launch_fill_mode(bool wide, const FillArgs& a, hipStream_t s);
// group: 32 = local walks of two pairs per wave (ta_walk2.h), 16 = lane walks
// (ta_walk_lane.h), 64 = band walks (one lane per pair, ta_walk_band.h; blocked
// layout), 0 = one pair per wave
hipError_t launch_traceback(int mode, const TraceArgs& a, hipStream_t s, int group);
// Dual-pair packed int16 fill (ta_dual.hip): a.order holds 2 pair ids per wave.
hipError_t launch_dual(int mode, bool cigar, const FillArgs& a, hipStream_t s);
template <int MODE, bool CIGAR>
hipError_t launch_dual_mode(const FillArgs& a, hipStream_t s);
// the local CIGAR dual fill in the blocked code layout (ta_dual.hip, TA_DUAL_BLK)
hipError_t launch_dual_blk(const FillArgs& a, hipStream_t s);
// ... and in the checkpoint layout of any mode (TA_DUAL_BLK + TA_DUAL_CK, a translation
// unit per mode; FillArgs.blk == 2)
template <int MODE>
hipError_t launch_dual_ck(const FillArgs& a, hipStream_t s);
// The recomputing walks of checkpoint plans (ta_walk_ck.hip; TraceArgs.blk == 2), then
// the fallback walk of the handed-back pairs; format_runs_kernel follows.
hipError_t launch_walk_ck(int mode, const TraceArgs& a, hipStream_t s);
// the flexible fill with checkpoints (ta_flex.hip TA_FLEX_CK), any mode
template <int MODE>
hipError_t launch_flex_ck(const FillArgs& a, hipStream_t s);
// Flexible two-pair fill (ta_flex.hip, global / semi-global): a.order holds 2
// pair ids per wave, the larger n first; both with the same pass count and
// n mod 16; rebased int16 values, so any length fits.
hipError_t launch_flex(int mode, bool cigar, const FillArgs& a, hipStream_t s);
template <int MODE, bool CIGAR>
hipError_t launch_flex_mode(const FillArgs& a, hipStream_t s);
hipError_t launch_compact(const CompactArgs& a, hipStream_t s);
// The server of one mode (slots waves, one per block): returns once launched.
template <int MODE>
hipError_t launch_serve_mode(const ServeArgs& a, uint32_t slots, hipStream_t s);
hipError_t launch_serve(int mode, const ServeArgs& a, uint32_t slots, hipStream_t s);

}  // namespace ta
