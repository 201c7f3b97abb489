// internal.hpp — shared declarations inside liballred.so (not installed).
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "allred.h"

namespace tsa {

// ---------------- bf16 (host) ----------------
inline float bf16_to_float(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
inline uint16_t bf16_from_float_rne(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
inline uint16_t bf16_from_float_trunc(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return (uint16_t)(u >> 16);
}

// ---------------- schedule ----------------
int steps_for(int total_nodes);
// Build + validate (see allred_schedule_build in allred.h).
int build_schedule(int algo, int side, int total, allred_schedule* out, std::string* why);

// ---------------- tuning (tune.cpp; allred_tune_set / allred_tune_get) ----------------
// Kernel-form switches between bit-identical forms; defaults = the product forms.
enum class Tune {
    fused_form, lo_tree, lo_dag, lo_dag_place, lo_dag_min_tiles, mem_reduce_lds, steps_form, pipe_grid, lo_dag_reg,
    lo_dag_reg_min_tiles, check, fused_chunk_tiles, lo_tree_min_tiles, tree_bcast_lag, tree_bcast_bal, steps_groups,
    rccl_fault, multi_fault, steps_tab, steps_early, peer_fence, hier_ws_ahead, hier_ws_cols, count
};
int64_t tune(Tune key);

// ---------------- the last kernel launch of this thread (allred_last_launch, engine.cpp) ----------------
// The launchers of the kernels bench.py reports (the fused pass, the schedule form, the
// hierarchical one-launch steps) record the kernel and the grid they chose.
void note_launch(const void* func, const char* name, unsigned grid, unsigned block);

// ---------------- device launchers (kernels.hip) ----------------
// All take hipStream_t as void* and return ALLRED_OK / ALLRED_ERR_*.
int launch_bf16_add(uint16_t* dst, const uint16_t* src, size_t n, void* stream);
// dst[seg] += src[seg] for up to kMaxAddSegs segments (elements, multiples of 8), ONE launch
constexpr int kMaxAddSegs = 64;
int launch_bf16_add_segs(uint16_t* dst, const uint16_t* src, const uint64_t* off, const uint64_t* len, int nsegs,
                         void* stream);
// host_memory: the ranks live in pinned host memory (zero-copy) -> pipelined form
// launches of one persistent fused pass over `tiles` 256-element tiles (fused_chunk_tiles)
uint64_t fused_chunk_launches(uint64_t tiles);
uint64_t fused_launches(int variant, bool lo_tree, int algo, int side, size_t n, int total);
int launch_tree_fused(uint16_t* ranks, uint64_t stride, size_t n, int total, const uint8_t* order, void* stream,
                      bool host_memory = false);
// dag: the interned LO DAG of a 64-rank schedule (engine.cpp lo_dag), or null
int launch_butterfly(uint16_t* ranks, uint64_t stride, size_t n, int total, const int16_t* d_partner, int steps,
                     const uint8_t* dag, void* stream);
// fused LO of a non-rank-uniform Swing schedule as its build-time DAG in registers
// (k_lo_dag_reg); ALLRED_ERR_UNSUPPORTED when no DAG was generated for (algo, side,
// total) or n is not a multiple of 256
int launch_lo_dag_reg(uint16_t* ranks, uint64_t stride, size_t n, int algo, int side, int total, void* stream);
int launch_tree_reduce(const uint16_t* ranks, uint64_t stride, size_t n, int total,
                       const uint8_t* order, uint16_t* out, void* stream);
int launch_broadcast(uint16_t* ranks, uint64_t stride, size_t n, int total, const uint16_t* src,
                     void* stream);
int launch_rs_step(uint16_t* ranks, uint64_t stride, int total, const int16_t* d_partner,
                   const int16_t* d_blocks, int blocks_per_rank, size_t block_elems, void* stream);
int launch_ag_step(uint16_t* ranks, uint64_t stride, int total, const int16_t* d_partner,
                   const int16_t* d_blocks, int blocks_per_rank, size_t block_elems, void* stream);
int launch_lo_step(const uint16_t* src, uint64_t src_stride, uint16_t* dst, uint64_t dst_stride,
                   int total, const int16_t* d_partner, size_t n, void* stream);
int launch_copy_ranks(const uint16_t* src, uint64_t src_stride, uint16_t* dst, uint64_t dst_stride,
                      int total, size_t n, void* stream);
// mem_2D; acc16: the reference's bf16 accumulation (every add rounded), else fp32 rounded once
int launch_mem_reduce(const uint16_t* ranks, uint64_t stride, size_t n, int total, uint16_t* dst, bool acc16,
                      void* stream);
int launch_mem_fused(uint16_t* ranks, uint64_t stride, size_t n, int total, bool acc16, void* stream);
// dst = rows[0] + rows[1] + ... + rows[nrows-1] in that order (fp32 rounded once, or
// bf16 per add): mem_2D's owner-first sum once the owner's copy is row 0
int launch_rows_sum(const uint16_t* rows, uint64_t stride, size_t n, int nrows, uint16_t* dst, bool acc16,
                    void* stream);
// allred_run with args->gpus > 0 (multi.cpp): the plan over G GPUs, one host thread each,
// on the backend ALLRED_TRANSPORT / ALLRED_SHARE_GPU select
int run_multi_gpu(const allred_args* a, int verbose, allred_report* report);
// run_multi_gpu: a flag every RCCL wait of `c` polls (another GPU's thread failed -> abort)
void comm_set_cancel(allred_comm* c, const std::atomic<int>* cancel);
// the checks allred_dist_allreduce applies to a desc (and its schedule)
int dist_check_desc(const allred_dist_desc* d, allred_schedule* s);
// bucket i+1's tree (-> cur_partial) and bucket i's broadcast (prev_result -> prev's rows) in one
// pass (k_tree_bcast_x; 64 ranks, whole tiles) or the two launches (same bits)
int launch_tree_bcast_x(uint16_t* cur, uint16_t* prev, uint64_t stride, size_t n, int total, const uint8_t* order,
                        uint16_t* cur_partial, const uint16_t* prev_result, void* stream);
// the mem_2D validation of one rank's result and the per-rank profile zones (engine.cpp)
int write_profile_log(const char* path, int N, int side, const uint64_t* start, const uint64_t* end);
// the schedule form as one persistent launch (k_bo_steps / k_lo_steps).  BO: d_tab = per block
// the phase table of engine.cpp bo_steps_table; LO: d_pairs = per step N/2 (r, p) pairs.
// stamps: null, or bo/lo_steps_units() x (2S + 1) / (S + 1) words (s_memrealtime)
constexpr int kBoPipeTabBytes = 256;   // the schedule form's BO program bytes per block (4N - 4 <= 252)
// d_pipe_tab: the pipelined form's table (engine.cpp bo_steps_pipe_table / lo_steps_pipe_table), or null;
// d_reg_tab: k_steps_reg's program (bo_steps_reg_table: N x 256 bytes, then the step-0 pairs), or null
int launch_bo_steps(uint16_t* ranks, uint64_t stride, int total, int steps, const uint8_t* d_tab,
                    const uint8_t* d_pipe_tab, const uint8_t* d_reg_tab, size_t block_elems, uint64_t* stamps,
                    void* stream);
uint64_t bo_steps_units(size_t block_elems, int total);
int launch_lo_steps(uint16_t* ranks, uint64_t stride, int total, int steps, const uint8_t* d_pairs,
                    const uint8_t* d_pipe_tab, size_t n, uint64_t* stamps, void* stream);
uint64_t lo_steps_units(size_t n);

// peer flag area (uint32 words): [0, 64) the multi-kernel barrier, then the
// one-kernel form's [2 phases][kPeerFusedMaxGroups][64 ranks] slots, then the
// scheduled (Swing / RecDub) form's progress slots [kPeerSchedMaxGroups][64 ranks]
constexpr uint32_t kPeerFusedFlagOff = 64;
constexpr uint32_t kPeerFusedMaxGroups = 128;
constexpr uint32_t kPeerSchedFlagOff = kPeerFusedFlagOff + 2 * kPeerFusedMaxGroups * 64;
constexpr uint32_t kPeerSchedMaxGroups = 256;
// the push form's data-arrived slots [kPeerSchedMaxGroups][64 ranks] behind the progress slots
constexpr uint32_t kPeerSchedPushOff = kPeerSchedFlagOff + kPeerSchedMaxGroups * 64;
constexpr size_t kPeerFlagBytes = 4 * ((size_t)kPeerSchedPushOff + kPeerSchedMaxGroups * 64);

// One rank's BO / LO program over peer-mapped windows (dist.cpp builds it from
// the same schedule + link-spreading channels as the RCCL program).
constexpr int kPeerMaxChannels = 7;
constexpr int kPeerMaxSteps = 6;
struct PeerProg {
    int S = 0, C = 1, N = 1, lo = 0;
    int fence = 0;   // tune peer_fence (set by the launchers): release / acquire fences around every flag
    int peer[kPeerMaxChannels][kPeerMaxSteps] = {};       // real rank, [channel][step]
    uint64_t recv[kPeerMaxChannels][kPeerMaxSteps] = {};  // block masks in the channel's labels
    uint64_t send[kPeerMaxChannels][kPeerMaxSteps] = {};
    uint64_t base[kPeerMaxChannels] = {}, len[kPeerMaxChannels] = {};  // channel slice, 16-byte vectors
};
int peer_prog(const allred_dist_desc* d, int rank, PeerProg* out);
// device copy of tree_order[0] of a (algo, side, total) schedule (cached per device)
int local_tree_order(int algo, int side, int total, const uint8_t** out);

int launch_peer_allreduce(uint16_t* const* wins, uint32_t* const* flags, int nranks, int me, uint16_t* bucket,
                          size_t n, uint32_t epoch, uint32_t* status, void* stream);
// full barrier of the peer set (flag region [0, 64))
int launch_peer_barrier(uint32_t* const* flags, int nranks, int me, uint32_t epoch, uint32_t* status, void* stream);
// the scheduled form: one launch; flag values base_epoch + 1 .. base_epoch + 2S + 1
int launch_peer_sched(uint16_t* const* wins, uint32_t* const* flags, int me, uint16_t* bucket, const PeerProg& prog,
                      uint64_t half_vec, uint32_t base_epoch, uint32_t* status, unsigned max_groups,
                      void* stream);
// the same BO program with every exchange a PUSH (k_peer_sched_push): the sender writes its blocks
// into the receiver's staging window (reduce-scatter) or main window (all-gather); stages[q] = GPU
// q's staging window (max_elems), same offsets as the windows
int launch_peer_sched_push(uint16_t* const* wins, uint16_t* const* stages, uint32_t* const* flags, int me,
                           uint16_t* bucket, const PeerProg& prog, uint32_t base_epoch, uint32_t* status,
                           unsigned max_groups, void* stream);
// the hierarchical forms' hand-off words: a tile's 512 bytes as 3 x 32 8-byte words (6 data
// bytes + a 16-bit epoch each), kHSlot words per tile slot (peer_kernels.hip h_pack)
constexpr int kHSlot = 96;
// hierarchical one-kernel form (64 local ranks, k_hier_ws): tree -> mem_2D across GPUs -> broadcast
// with LL (push) hand-offs: ll[q] = GPU q's LL area for this parity, [inbox box_words words][result
// box box_words words]; nranks <= 8; epoch grows by 1 per call
int launch_hier_ws(uint16_t* ranks, uint64_t stride, const uint8_t* order, uint64_t* const* ll, int nranks, int me,
                   size_t n, uint64_t box_words, uint32_t epoch, uint32_t* status, unsigned max_grid,
                   void* stream);
// the same step two buckets deep (k_hier_x2): starts `cur`, sums the owned tiles of the bucket
// the previous launch started (llm non-null: its parity's LL areas), writes `old` (started two
// launches ago; llo: its parity); the flush launch (cur null) also writes that middle bucket
// `fin` from its results
int launch_hier_x2(uint16_t* cur, uint16_t* old, uint16_t* fin, uint64_t stride, const uint8_t* order,
                   uint64_t* const* llc, uint64_t* const* llm, uint64_t* const* llo, int nranks, int me, size_t n,
                   uint64_t box_words, uint32_t ecur, uint32_t emid, uint32_t eold, uint32_t* status,
                   unsigned max_grid, void* stream);
// allred_mem_2D across GPUs with LL pushes (k_peer_mem_ll): area_words >= 8 * (n / 8 rounded up to 32)
int launch_peer_mem_ll(uint64_t* const* ll, int nranks, int me, uint16_t* bucket, size_t n, uint64_t area_words,
                       uint32_t epoch, uint32_t* status, unsigned max_groups, void* stream);
// the one-channel LO program with LL pushes (k_peer_lo_ll): ll[q] = GPU q's LL area of this
// parity (area_words 8-byte words >= steps * n / 2)
int launch_peer_lo_ll(uint64_t* const* ll, int nranks, int me, uint16_t* bucket, const PeerProg& prog, size_t n,
                      uint64_t area_words, uint32_t epoch, uint32_t* status, void* stream);
// one launch; epoch must grow by >= 1 per call
int launch_peer_oneshot(uint16_t* const* wins, uint32_t* const* flags, int nranks, int me, uint16_t* bucket,
                        size_t n, uint32_t epoch, uint32_t* status, void* stream);

int hip_status(int hip_err);  // maps hipError_t -> ALLRED_*

}  // namespace tsa
