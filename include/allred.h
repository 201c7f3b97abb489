/*
 * allred.h — C-ABI of the MI355X allreduce engine (liballred.so).
 *
 * Drop-in boundary for the reference EngineerCharlie/TenstorrentAllreduce.
 * Plain pointers and sizes only; every entry point names the reference
 * interface it replaces (file:line under the reference tree).  All functions
 * return ALLRED_OK (0) or a negative ALLRED_ERR_* code unless documented
 * otherwise; the reference itself has no error codes (bad configurations hang
 * the Wormhole) — here they are rejected up front.
 *
 * Host-only entry points (schedule, data generation, validation) never touch
 * the GPU.  Device entry points take a hipStream_t as `void* stream`
 * (NULL = the default stream) and enqueue asynchronously.
 */
#ifndef ALLRED_H
#define ALLRED_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 7 (round 6): the one-deep peer pipeline (allred_peer_allreduce_pipelined, k_hier_x) and
 * k_hier_ll are retired, allred_peer_set_hier_ll takes 0 (launch form) / 1 (k_hier_ws, the
 * default), the tune keys hier_x2_tail / hier_x_lag / hier_x_chunked / hier_x_rearly /
 * hier_x_latepoll are gone (k_hier_x2 runs its measured product form only), and
 * allred_last_launch is new.  ABI 6 (round 5): the hierarchical forms' hand-off area holds
 * 6 data bytes + a 16-bit epoch per word — peers of different ABIs must not connect. */
#define ALLRED_ABI_VERSION 7

/* ---- status codes ---------------------------------------------------- */
#define ALLRED_OK 0
#define ALLRED_ERR_ARG (-1)          /* bad argument / size / alignment       */
#define ALLRED_ERR_SCHEDULE (-2)     /* grid is not a valid allreduce schedule */
#define ALLRED_ERR_HIP (-3)          /* HIP runtime failure                   */
#define ALLRED_ERR_RCCL (-4)         /* RCCL failure                          */
#define ALLRED_ERR_NOMEM (-5)
#define ALLRED_ERR_UNSUPPORTED (-6)
#define ALLRED_ERR_TRANSPORT (-7)    /* host exchange callback failed         */

/* ---- enums --------------------------------------------------------------*/
/* argv[1] "is swing version?" (allred_helper.cpp:205-208) */
#define ALLRED_RECDUB 0
#define ALLRED_SWING 1
/* the 1D schedules of the reference's prototypes (side_length ignored) */
#define ALLRED_RECDUB_1D 2  /* scratch_work/recdub_multicore_1D/recdub_multicore_1D.cpp:165-175 */
#define ALLRED_SWING_1D 3   /* scratch_work/all_red_swing_1D/all_red_swing_1D.cpp:32-36 */
/* which reference program: allred_BO_2D with arg 8 = 1 / = 0, allred_mem_2D */
#define ALLRED_BO 0
#define ALLRED_LO 1
#define ALLRED_MEM 2
/* execution form of a virtual-rank plan */
#define ALLRED_EXEC_STEPS 0  /* the reference's step program, step by step (partner exchange + add per step) */
#define ALLRED_EXEC_FUSED 1  /* one HBM pass for the whole allreduce, same arithmetic, same bits */
/* mem_2D accumulation (allred_mem_2D/kernels/compute_kernel.cpp:44-67) */
#define ALLRED_ACC_FP32 0    /* fp32 sum, rounded to bf16 once (default) */
#define ALLRED_ACC_BF16 1    /* the reference's bf16 dest register (fp32_dest_acc_en = false,
                                allred_helper.cpp:331-335): every add rounded to bf16 */

#define ALLRED_MAX_NODES 64
#define ALLRED_MAX_STEPS 6

const char* allred_status_string(int status);
int allred_abi_version(void);

/* ======================================================================
 * Schedule — replaces allred_helper.hpp:24-30 / allred_helper.cpp:122-191
 * and allred_BO_2D.cpp:4-5 / :217-270 (same arguments; the C++ reference
 * signatures are kept in include/allred_helper.hpp).
 * ==================================================================== */
int allred_highest_power_of_two(int value);                          /* allred_helper.cpp:122 */
uint32_t allred_get_step_directions(int node_x, int node_y);         /* allred_helper.cpp:136 */
int allred_get_comm_partner_swing_2d(int node, int step, int horizontal_step,
                                     int side_length, int total_nodes);   /* allred_helper.cpp:166 */
int allred_get_comm_partner_recdub_2d(int node, int recdub_step, int horizontal_step,
                                      int message_pass_depth, uint32_t* step_directions,
                                      int side_length);                   /* allred_helper.cpp:145 */
void allred_get_swing_block_comm_indexes(int node, int step, uint32_t* blocks /*[2]*/,
                                         int horizontal_step, int side_length,
                                         int total_nodes);                /* allred_BO_2D.cpp:220 */
void allred_get_recdub_block_comm_indexes(int node, int step, uint32_t* blocks /*[2]*/,
                                          int horizontal_step, int side_length, int total_nodes,
                                          int message_pass_depth,
                                          uint32_t* step_directions);     /* allred_BO_2D.cpp:242 */
/* NUM_TILES normalisation, allred_helper.cpp:224-234 */
int allred_normalize_tiles(int tiles, int total_nodes, int large_buffer);
/* 1D partners of the reference's 8-core prototypes */
int allred_get_comm_partner_swing_1d(int node, int step, int num_nodes);          /* all_red_swing_1D.cpp:32 */
int allred_get_comm_partner_recdub_1d(int node, int step, uint32_t* step_directions); /* recdub_multicore_1D.cpp:165 */

/* Whole per-rank schedule, as the per-core loop of allred_BO_2D.cpp:75-212
 * builds it into runtime args: partners (args 14+2i), send masks (22+2s+2i),
 * recv masks (22+4s+2i / compute args 6+2i), direction bits (arg 11).
 * Grids: side in {1,2,4,8}, total a power of two <= 64 (side*side for the
 * reference's square grids; (2,2), (2,4), (4,8) for 2/4/8 GPUs).  algo may
 * also be ALLRED_RECDUB_1D / ALLRED_SWING_1D (any power-of-two total; the
 * block masks then come from the same "reachable at later steps" rule).
 * Also validates the schedule (partners in range and symmetric, send ==
 * partner's recv, reduce-scatter leaves block r at rank r, every rank's
 * contributor sets disjoint at each merge) and derives tree_order[x]: the
 * leaf order of the reduction tree rank x evaluates, leaves(x, k) =
 * leaves(x, k-1) ++ leaves(partner_{k-1}(x), k-1); level k adds adjacent
 * groups of 2^k leaves.  LO gives rank x the value of tree x; BO gives block
 * b the value of tree b (reduced at its owner, then all-gathered).  For
 * RecDub all trees coincide; for Swing they differ (in bf16 rounding only). */
typedef struct {
    int32_t algo, side, total, steps;
    int32_t partner[ALLRED_MAX_NODES][ALLRED_MAX_STEPS];
    uint64_t send[ALLRED_MAX_NODES][ALLRED_MAX_STEPS];
    uint64_t recv[ALLRED_MAX_NODES][ALLRED_MAX_STEPS];
    uint32_t dirs[ALLRED_MAX_NODES];
    uint8_t tree_order[ALLRED_MAX_NODES][ALLRED_MAX_NODES];
} allred_schedule;
int allred_schedule_build(int algo, int side_length, int total_nodes, allred_schedule* out);
/* The fused LO pass's DAG of distinct sums (64 ranks; no reference
 * counterpart — the per-core butterfly of allred_BO_2D/kernels/
 * dataflow_kernel.cpp:19-29 evaluated once per distinct value).  Writes the
 * layout k_butterfly_lds64_pipe reads (kernels.hip) into out[cap]; returns
 * the bytes written, 0 when the schedule has no DAG form (not 64 ranks, a
 * step with more than 32 distinct sums), or a negative status.
 * *read_conflicts = extra LDS bank cycles of its reads per column group and
 * tile (0 once placed; allred_tune_set("lo_dag_place", 0) keeps first-appearance order). */
int allred_lo_dag(int algo, int side_length, int total_nodes, uint8_t* out, size_t cap, int* read_conflicts);
/* The schedule form's step program as k_steps_reg reads it (kernels.hip):
 * the per-core RS / AG loops of allred_BO_2D/kernels/dataflow_kernel.cpp:152-267
 * (variant ALLRED_BO: total x 256 bytes, one block per 256) or the LO exchange
 * steps of allred_LOO_2D/kernels/dataflow_kernel.cpp:127-175 (ALLRED_LO:
 * 2 (total/2) S + total bytes), restated on a strip's pair rows (BO: the
 * kernel recasts step 0 per block for its register-staged loads).  Returns the
 * bytes written into out[cap], 0 when the schedule has no such program, or a
 * negative status.  For inspection and CPU checks (tests/test_steps_program.py).
 * variant ALLRED_BO | ALLRED_STEPS_REG: the program k_steps_reg actually loads
 * for BO (engine.cpp bo_steps_reg_table): per block 256 bytes with step 0 recast
 * as byte u = row of step-0 pair u | 0x80 when its higher rank holds, then the
 * (total/2) pairs' (lower, higher) ranks — total x 256 + total bytes. */
#define ALLRED_STEPS_REG 0x100
int allred_steps_program(int algo, int variant, int side_length, int total_nodes, uint8_t* out, size_t cap);

/* ======================================================================
 * Host data — tt-metal bfloat16 helpers the reference calls
 * (allred_helper.cpp:277-285) and validate_result_vector (:18-120).
 * ==================================================================== */
/* create_random_vector_of_bfloat16(num_bytes, rand_max, seed): std::mt19937 +
 * uniform_real_distribution<float>(0, rand_max); two bf16 per uint32, low
 * half first.  round_mode 0 = truncating bfloat16(float) (default), 1 = RNE. */
void allred_random_bf16_vector(size_t num_bytes, int rand_max, int seed, int round_mode, uint32_t* out);
void allred_constant_bf16_vector(size_t num_bytes, float value, uint32_t* out);
/* validate_result_vector: expected = bf16((a+b) * (total_nodes/2)); prints the
 * reference's messages ("All values match!" ...) when verbose != 0.
 * Returns the number of elements with |actual - expected| > error.          */
long allred_validate_result_vector(const uint32_t* result_vec, const uint32_t* src_vec_0,
                                   const uint32_t* src_vec_1, size_t num_els, float error,
                                   uint32_t total_nodes, int verbose, float* max_error);

/* ======================================================================
 * Device compute (HIP, gfx950)
 * ==================================================================== */
/* dst[i] = bf16_rne(float(dst[i]) + float(src[i])), i < n.  Replaces the
 * per-tile add_tiles + pack_tile<true> of allred_BO_2D/kernels/compute_kernel.cpp:53-60. */
int allred_bf16_add(uint16_t* dst, const uint16_t* src, size_t n, void* stream);
/* Same over the blocks named by a 64-bit mask (block b = [b*block_elems, (b+1)*block_elems)),
 * the BO compute loop of compute_kernel.cpp:35-67 for one step. */
int allred_bf16_add_masked(uint16_t* dst, const uint16_t* src, uint64_t block_mask,
                           size_t block_elems, void* stream);

/* Reduce `total` virtual ranks (rank r at ranks + r*rank_stride) into `out`
 * with the reduction tree of rank 0 of the (algo, side, total) schedule (one
 * HBM pass; the hierarchical first stage), and the matching broadcast of one
 * vector back to every rank (the all-gather's data movement). n % 8 == 0. */
int allred_tree_reduce(const uint16_t* ranks, uint64_t rank_stride, size_t n, int algo, int side_length,
                       int total_nodes, uint16_t* out, void* stream);
int allred_broadcast(uint16_t* ranks, uint64_t rank_stride, size_t n, int total_nodes, const uint16_t* src,
                     void* stream);

/* ======================================================================
 * Virtual-rank plan: `total` ranks resident in ONE GPU's HBM, rank r at
 * ranks + r * rank_stride (elements).  Replaces the 64-core Tensix program
 * (allred_BO_2D/kernels, allred_LOO_2D/kernels, allred_mem_2D/kernels).
 * Every rank ends with the allreduced vector, in place.
 * ==================================================================== */
typedef struct allred_plan allred_plan;
typedef struct {
    int32_t algo;          /* ALLRED_SWING / ALLRED_RECDUB                      */
    int32_t variant;       /* ALLRED_BO / ALLRED_LO / ALLRED_MEM                */
    int32_t exec;          /* ALLRED_EXEC_STEPS / ALLRED_EXEC_FUSED             */
    int32_t side_length;   /* 1, 2, 4, 8                                        */
    int32_t total_nodes;   /* 0 = side*side                                     */
    int32_t device;        /* HIP device ordinal (-1 = current)                 */
    uint64_t elems_per_rank; /* bf16 elements; BO/MEM need a multiple of 8*total, LO of 8 */
    int32_t mem_accum;     /* MEM only: ALLRED_ACC_FP32 (default) / ALLRED_ACC_BF16 */
} allred_plan_desc;
int allred_plan_create(const allred_plan_desc* desc, allred_plan** out);
/* HBM layout helper: the rank stride (elements) this engine lays virtual ranks
 * out with — elems rounded up to 64, plus a 128-byte skew so the P rank rows
 * of a tile do not start on the same HBM channel (655,360-byte rows are
 * 5 * 2^17 apart: +5.6 % on the fused pass). */
uint64_t allred_preferred_rank_stride(uint64_t elems_per_rank);
int allred_plan_destroy(allred_plan* plan);
size_t allred_plan_workspace_bytes(const allred_plan* plan);
/* workspace: device memory of allred_plan_workspace_bytes() (may be NULL when 0) */
int allred_plan_execute(allred_plan* plan, uint16_t* ranks, uint64_t rank_stride,
                        void* workspace, void* stream);
/* number of kernel launches one execute enqueues (for per-launch accounting) */
int allred_plan_launches(const allred_plan* plan);
/* Device-side profiling of the schedule form (the reference's DeviceZoneScopedN
 * "ALL_RED_LOOP", allred_BO_2D/kernels/dataflow_kernel.cpp:147, dumped by
 * DumpDeviceProfileResults, allred_helper.hpp:88).  stamp_words: the uint64
 * words of device memory execute_profiled writes (0: this plan's form has no
 * stamps — only ALLRED_EXEC_STEPS BO / LO do).  rank_zones: from the stamps
 * copied to the host, each rank's zone start / end (s_memrealtime, 100 MHz):
 * start = its first load, end = the end of the step of its last store. */
uint64_t allred_plan_stamp_words(const allred_plan* plan);
int allred_plan_execute_profiled(allred_plan* plan, uint16_t* ranks, uint64_t rank_stride, void* workspace,
                                 uint64_t* device_stamps, void* stream);
int allred_plan_rank_zones(const allred_plan* plan, const uint64_t* host_stamps, uint64_t* zone_start /*[total]*/,
                           uint64_t* zone_end /*[total]*/);

/* ======================================================================
 * Tuning: the one entry point for switching between kernel forms that give
 * bit-identical results (A/B measurements).  The defaults are the measured
 * product forms; nothing needs setting.  Initial values may come from
 * ALLRED_TUNE="key=value,key=value" (read once at load).  Keys:
 *   fused_form        0 auto | 1 register tree | 2 one tile per workgroup | 3 persistent pipe
 *   lo_tree           1: fused LO of rank-uniform schedules through the BO tree pass
 *   lo_dag            1: fused 64-rank LO as the DAG of distinct sums (0 = per-rank butterfly)
 *   lo_dag_place      1: bank-conflict-free DAG placement (0 = first-appearance order)
 *   lo_dag_min_tiles  256: smallest bucket (256-element tiles) for the DAG pass
 *   mem_reduce_lds    1: mem_2D schedule-form reduce staged through LDS
 *   steps_form        schedule form: 0 one pipelined launch (units staged into LDS two ahead, the step
 *                     program among LDS rows, stores one unit late) | 1 one launch per step (rank
 *                     copies in the buckets) | 2 one launch with every unit resident at once
 *   pipe_grid         0: auto grid of the persistent passes
 *   lo_dag_reg        1: fused LO of the non-rank-uniform Swing schedules (32 / 64 ranks) as the
 *                     build-time DAG of distinct sums in registers (0 = the LDS DAG pass above)
 *   lo_dag_reg_min_tiles  64: smallest bucket (256-element tiles per rank, 32 kB) for lo_dag_reg
 *   check             0; 1: check mode of the N > 1 step programs (allred_dist_allreduce and its
 *                     host twin): each rank's program is verified once against its partners'
 *                     (what a partner sends at step k is exactly what this rank receives; the
 *                     received runs of a step are disjoint, inside the bucket) — ALLRED_ERR_SCHEDULE
 *                     if not — and every receive region is filled with 0xFFFF (a bf16 NaN) before
 *                     its step, so an element the transport never delivered surfaces as NaN in the
 *                     result instead of stale data.  Same result bits on a correct run.  (The
 *                     reference has no invariant or race checking)
 *   fused_chunk_tiles 1280: the persistent fused 64-rank passes run a bucket of T 256-element
 *                     tiles as max(1, round(T / 1280)) launches over consecutive tile ranges
 *                     (0 = one launch); allred_plan_launches counts them
 *   lo_tree_min_tiles 64: a 64-rank rank-uniform LO plan (every RecDub schedule) takes the BO tree
 *                     pass from this many 256-element tiles per rank, the register butterfly below
 *   tree_bcast_lag    1: k_tree_bcast_x (allred_dist_allreduce_pipelined) stores the previous
 *                     bucket's rows of a tile one iteration after the tile's tree (0: in the same one)
 *   tree_bcast_bal    0; 1: k_tree_bcast_x spreads the result-tile loads and partial stores over
 *                     its four waves (8 columns each) instead of wave 0
 *   steps_groups      0: workgroups per CU of the schedule form k_steps_reg — 0 auto (BO 3; LO 4,
 *                     or 3 where 4 would leave every wave exactly one strip), 3, 4 or 5 (1 and 2:
 *                     ALLRED_ERR_ARG)
 *   steps_tab         1: k_steps_reg (BO) stages only the programs of its own units' blocks (when fewer
 *                     than P); 0: every block's program (P x 256 bytes) per workgroup (round 3)
 *   steps_early       1: k_steps_reg issues the first strip's loads before it stages its programs when
 *                     its grid is full (units >= workgroups), else after; 2: always before; 0: always
 *                     after (round 3)
 *   peer_fence        0; 1: the flag protocols of the peer windows (k_peer_oneshot, k_peer_sched,
 *                     k_peer_sched_push) put a system-scope release fence before every flag store
 *                     and an acquire fence after every flag wait.  Same bits; the default relies on
 *                     the ordering argument of DESIGN.md §5 (uncached hand-off memory, s_waitcnt
 *                     before the workgroup barrier that precedes a flag).  The LL kernels have no
 *                     separate flag (each word carries its epoch) and take no fence.  Every rank
 *                     must use the same setting
 *   hier_ws_ahead     1: k_hier_ws's reducing waves load one tile ahead; 2: two (measured slower,
 *                     +0.3-0.5 us at W = 1)
 *   hier_ws_cols      16: 16-byte columns of a tile per k_hier_ws reducing wave — 8 (quarters: 8
 *                     waves per workgroup), 16 (halves: 4 waves) or 32 (whole tiles: 2 waves); other
 *                     values ALLRED_ERR_ARG
 *   multi_fault       0; fault injection (tests only): 1..32: GPU value - 1 of allred_run_multi fails its
 *                     timed allreduce while its peers are in theirs (every thread must return);
 *                     33..64: GPU value - 33 fails its warm-up (every thread skips the timed region)
 *   rccl_fault        0; fault injection of the bounded RCCL waits (tests only), a bit mask: 1 init,
 *                     2 every group end, 4 every allred_comm_wait stays pending as if a peer never
 *                     arrived, so the deadline / ncclCommAbort path runs (ALLRED_ERR_TRANSPORT)
 * Plans read the keys when they are created (lo_*, steps_form) or launched.
 * ALLRED_ERR_ARG: unknown key or value out of range.  No reference
 * counterpart (the reference picks its kernel directory by string,
 * allred_BO_2D.cpp:203-211). */
int allred_tune_set(const char* key, int64_t value);
int allred_tune_get(const char* key, int64_t* value);

/* The last kernel launch of the calling thread among the ones the bench
 * reports (the fused BO pass k_tree_lds_lag, the schedule form k_steps_reg,
 * the hierarchical one-launch steps k_hier_ws / k_hier_x2): the kernel, the
 * grid its launcher chose, and — queried at this call — its static LDS,
 * VGPRs, resident workgroups per CU (hipOccupancyMaxActiveBlocksPerMultiprocessor)
 * and the device's CU count.  ALLRED_ERR_ARG when this thread launched none of
 * them.  No reference counterpart (the reference fixes its core grid,
 * allred_BO_2D.cpp:26). */
typedef struct {
    char kernel[64];
    uint32_t grid;
    uint32_t block;
    uint32_t lds_bytes;
    int32_t regs;
    int32_t resident_per_cu;
    int32_t cus;
    int32_t device;
    int32_t reserved;
} allred_launch_info;
int allred_last_launch(allred_launch_info* out);

/* ======================================================================
 * Reference program surface: AllredConfig (allred_helper.hpp:47-97) +
 * the mains of allred_BO_2D.cpp:7-215 / allred_LO_2D.cpp:9-106 /
 * allred_mem_2D.cpp:4-165, with the same 8 positional arguments.
 * ==================================================================== */
typedef struct {
    int32_t variant;         /* ALLRED_BO (bo flag decides BO vs LO), ALLRED_LO (legacy binary), ALLRED_MEM */
    int32_t swing;           /* argv[1] == 1                                     */
    int32_t run_kernel;      /* argv[2] == 1                                     */
    int32_t side_length;     /* highest_power_of_two(argv[3])                    */
    int32_t seed;            /* argv[4]: < 0 -> all ones                          */
    int32_t tiles;           /* argv[5] (raw, >= 1)                              */
    int32_t error;           /* argv[6]                                          */
    int32_t print_core;      /* argv[7]                                          */
    int32_t bandwidth_optimal; /* argv[8]                                        */
    int32_t total_nodes;     /* extension (ALLRED_NODES env / argv[9]); 0 = side^2 */
    int32_t exec;            /* extension (ALLRED_EXEC env): fused (default) / steps */
    int32_t round_mode;      /* extension (ALLRED_BF16_ROUND env): 0 trunc, 1 rne */
    int32_t num_tiles;       /* derived: normalised NUM_TILES                    */
    int32_t device;          /* HIP device ordinal, -1 = current (ALLRED_DEVICE env); the
                                reference's CreateDevice(0) / IDevice*, allred_BO_2D.cpp:8 */
    int32_t mem_accum;       /* extension (ALLRED_MEM_ACC=bf16): ALLRED_ACC_FP32 / ALLRED_ACC_BF16 */
    int32_t gpus;            /* extension (argv[10] or ALLRED_GPUS): 0 = every rank a virtual rank on
                                `device` (the default); G >= 1 = the ranks spread over GPUs
                                device .. device + G - 1, one host thread and one RCCL rank per GPU */
} allred_args;
/* Parses argv exactly like AllredConfig's ctor (std::stoi semantics: leading
 * integer, junk -> ALLRED_ERR_ARG where the reference would throw).          */
int allred_args_parse(int argc, const char* const* argv, int variant, allred_args* out);

typedef struct {
    int64_t mismatches;      /* validate_result_vector count, -1 if not run      */
    float max_error;
    double device_seconds;   /* hipEvent time of the device-resident allreduce */
    double e2e_seconds;      /* pinned H2D + allreduce + D2H                     */
    uint64_t bytes_per_rank;
    int32_t total_nodes;
    int32_t launches;
} allred_report;
/* Generate inputs, H2D, run (if run_kernel), D2H of print_core, validate
 * (printing like the reference when verbose), report timing, on args->device.
 * args->gpus = G >= 1 (ALLRED_GPUS / argv[10]): the same program on G GPUs of
 * this node in ONE process, one host thread per GPU, one RCCL communicator per
 * GPU (ncclCommInitAll).  The total_nodes ranks are split into G groups of
 * L = total / G consecutive ranks, group g on GPU device + g (G a power of two
 * dividing total, G <= the visible GPUs; else ALLRED_ERR_ARG before any HIP
 * call).  L == 1: the reference's own (side, total) schedule runs across the
 * GPUs (allred_dist_allreduce: Swing / RecDub BO or LO, or mem_2D's
 * one-shot exchange); L > 1: each GPU reduces its L ranks with the (side, L)
 * sub-grid's tree (or (2,2)/(2,4)/(4,8)/... when the rows do not form one),
 * the GPUs allreduce the partials on the (2,2)/(2,4)/(4,8) grid, and every
 * rank gets the result (mem_2D: L == 1 or G == 1 only, else
 * ALLRED_ERR_UNSUPPORTED).  Every GPU's first rank is validated as well as
 * print_core (ALLRED_CHECK_ALL: every rank); device_seconds / e2e_seconds are
 * the slowest GPU's.  The reference is single-chip (allred_BO_2D.cpp:7-29,
 * allred_helper.cpp:205-220): this is its argv across the GPUs of one node.
 * ALLRED_PROFILE_LOG=<path> also writes every rank's ALL_RED_LOOP zone in the
 * layout of tt-metal's profile_log_device.csv (the reference's
 * TT_METAL_DEVICE_PROFILER=1 run, python/timing_taker.py:60-65).            */
int allred_run(const allred_args* args, int verbose, allred_report* report);

/* ======================================================================
 * Multi-GPU: one process per GPU, RCCL point-to-point over xGMI.
 * The grid (side_length, total_nodes) maps GPUs onto the reference's own
 * 2D schedule: 2 GPUs (2,2), 4 GPUs (2,4), 8 GPUs (4,8).
 * ==================================================================== */
#define ALLRED_UNIQUE_ID_BYTES 128
typedef struct allred_comm allred_comm;
int allred_comm_get_unique_id(uint8_t* id /*[128]*/);
int allred_comm_init(const uint8_t* id, int nranks, int rank, int device, allred_comm** out);
/* ndev communicators in ONE process (ncclCommInitAll), rank i on devices[i]:
 * one host thread per communicator afterwards (each thread its own stream).
 * The reference's CreateDevice(0) (allred_BO_2D.cpp:8) for the GPUs of a node. */
int allred_comm_init_all(int ndev, const int* devices, allred_comm** out /*[ndev]*/);
int allred_comm_destroy(allred_comm* comm);

typedef struct {
    int32_t algo;           /* ALLRED_SWING / ALLRED_RECDUB                     */
    int32_t variant;        /* ALLRED_BO, ALLRED_LO, or ALLRED_MEM (local_ranks == 1: the
                               mem_2D one-shot exchange, allred_mem_2D.cpp:4-165 — every
                               rank's copy of block b to rank b, summed there in mem_2D
                               order, then gathered; all links at once)      */
    int32_t side_length;    /* GPU grid                                         */
    int32_t total_nodes;    /* == nranks                                        */
    uint64_t elems;         /* bf16 elements per GPU bucket (multiple of 8*total for BO) */
    /* hierarchical extension: the bucket holds local_ranks virtual ranks
     * (stride `elems`), reduced on-GPU first with the local_side grid. 1 = flat. */
    int32_t local_ranks;
    int32_t local_side;
    int32_t local_algo;
    int32_t channels;       /* link-spreading channels: 0 = auto (all 2^S-1 links for
                               buckets >= 1 MiB on XOR grids), 1 = the plain schedule */
    int32_t mem_accum;      /* ALLRED_MEM only: ALLRED_ACC_FP32 (default) / ALLRED_ACC_BF16 */
} allred_dist_desc;
/* Scratch device bytes the call needs (recv staging + hierarchical partial). */
size_t allred_dist_workspace_bytes(const allred_dist_desc* desc);
int allred_dist_allreduce(allred_comm* comm, const allred_dist_desc* desc, uint16_t* buf,
                          void* workspace, void* stream);

/* The hierarchical step (local_ranks > 1, BO / LO) PIPELINED across consecutive
 * buckets: the call with `cur` reduces cur's local ranks to its partial (the
 * local tree), FUSED with writing the previous call's bucket's rows from its
 * allreduced partial (one HBM pass, k_tree_bcast_x, reads and writes of the two
 * buckets overlapping), then runs the RCCL program on cur's partial; cur ==
 * NULL (flush) writes the last pending bucket's rows.  K buckets = K + 1 calls:
 * b0, b1, ..., b_{K-1}, NULL.  A bucket's rows are final, in stream order,
 * after the next call (or the flush): keep it alive until then.  workspace:
 * 2 * allred_dist_workspace_bytes(desc) bytes (two parities), the same on every
 * call of a sequence; every call of a sequence has the same elems and
 * local_ranks (else ALLRED_ERR_ARG).  Same result bits as allred_dist_allreduce
 * per bucket.  The reference runs one vector per program: no counterpart. */
int allred_dist_allreduce_pipelined(allred_comm* comm, const allred_dist_desc* desc, uint16_t* cur, void* workspace,
                                    void* stream);
/* The two local phases of the pipelined step as one call: cur's tree (local
 * rank 0's, as allred_tree_reduce) into cur_out, and prev_src to every one of
 * prev's `total` rank rows (as allred_broadcast). */
int allred_tree_broadcast_pipelined(uint16_t* cur, uint16_t* prev, uint64_t rank_stride, size_t n, int algo,
                                    int side_length, int total_nodes, uint16_t* cur_out, const uint16_t* prev_src,
                                    void* stream);

/* The per-rank program allred_dist_allreduce (and its host twin) runs for
 * `desc`: steps = exchange steps (one RCCL group each), add_launches = add
 * kernels it enqueues over all steps (one per reduce-scatter / LO step,
 * whatever the channel count), segments = send + receive segments.  Programs
 * are built once per (desc, rank) and cached. */
int allred_dist_program_stats(const allred_dist_desc* desc, int rank, int* steps, int* add_launches, int* segments);

/* Host-memory twin of allred_dist_allreduce for CPU tests and loopback
 * checks: the same per-rank step program, exchanges done by a callback.     */
typedef struct {
    void* ptr;
    uint64_t bytes;
} allred_seg;
/* Exchange with `peer`: send every send segment, receive every recv segment
 * (in list order on both sides).  Return 0 on success. */
typedef int (*allred_exchange_fn)(void* ctx, int peer, int nsend, const allred_seg* send,
                                  int nrecv, const allred_seg* recv);
int allred_dist_allreduce_host(const allred_dist_desc* desc, int rank, uint16_t* buf,
                               uint16_t* scratch, allred_exchange_fn exchange, void* ctx);

/* ---- bounded RCCL (a bad configuration returns an error
 * instead of hanging; the reference hangs, allred_helper.hpp:84-96) -------
 * Communicators are created non-blocking (ncclConfig_t.blocking = 0): init
 * and every ncclGroupEnd are polled (ncclCommGetAsyncError) against a
 * deadline; allred_comm_wait polls the stream the same way.  Past the
 * deadline the communicator is aborted (ncclCommAbort: its kernels leave
 * their waits) and the call returns ALLRED_ERR_TRANSPORT; every later call
 * on that communicator returns ALLRED_ERR_TRANSPORT too (destroy it).
 * timeout_ms: 0 = the default, ALLRED_RCCL_TIMEOUT_MS or 4000 ms for
 * operations (init: at least 60 s — a node's first RCCL init takes seconds). */
int allred_comm_set_timeout(allred_comm* comm, int timeout_ms);
/* Waits until `stream` has drained (hipStreamQuery) or the deadline passed
 * (-> ncclCommAbort, ALLRED_ERR_TRANSPORT); an asynchronous RCCL error ->
 * ALLRED_ERR_RCCL.  Replaces hipStreamSynchronize after RCCL work. */
int allred_comm_wait(allred_comm* comm, void* stream);
/* 1 once the communicator was aborted, else 0. */
int allred_comm_aborted(const allred_comm* comm);

/* ======================================================================
 * allred_run across GPUs (args->gpus = G >= 1) in two parts.
 * (1) The PLAN — pure host computation, no HIP call: how the reference's
 *     (side, total) ranks (allred_BO_2D.cpp:7-29, allred_helper.cpp:205-220)
 *     split over G GPUs and which exchange every GPU runs.
 * (2) An EXCHANGE BACKEND executing it, one host thread per GPU:
 *   ALLRED_TRANSPORT_RCCL  one RCCL rank per GPU (allred_comm_init_all +
 *                          allred_dist_allreduce), the default;
 *   ALLRED_TRANSPORT_PEER  peer windows of the G threads mapped into each other
 *                          in-process (allred_peer_connect_all) and
 *                          allred_peer_dist_allreduce; with share_device every
 *                          group runs on ONE GPU (a rehearsal of the G-GPU
 *                          orchestration on hardware: threads, barriers, per-GPU
 *                          H2D / D2H slices, validation);
 *   ALLRED_TRANSPORT_HOST  the host twin: G threads on host memory running
 *                          allred_dist_allreduce_host with an in-memory exchange;
 *                          no HIP call at all (CPU tests of the orchestration;
 *                          only ever selected explicitly).
 * allred_run picks them from ALLRED_TRANSPORT=rccl|peer|host and
 * ALLRED_SHARE_GPU=1.
 * ==================================================================== */
#define ALLRED_MULTI_FLAT 0   /* L = 1: the reference's own (side, total) schedule across the GPUs */
#define ALLRED_MULTI_HIER 1   /* L > 1: each GPU's L ranks -> its sub-grid's tree, the partials
                                 allreduced on the (2,2)/(2,4)/(4,8)... GPU grid, the result written
                                 to every rank: a hierarchical COMPOSITION — on arbitrary data its
                                 bits differ from the flat one-GPU plan of the same argv; on the
                                 reference's own inputs both are exactly RNE(a+b)*N/2 */
#define ALLRED_MULTI_LOCAL 2  /* G = 1, mem_2D: the fused mem_2D pass over every rank, no exchange */
#define ALLRED_TRANSPORT_RCCL 0
#define ALLRED_TRANSPORT_PEER 1
#define ALLRED_TRANSPORT_HOST 2
typedef struct {
    int32_t gpus;             /* G                                                   */
    int32_t local_ranks;      /* L = total / G: ranks g*L .. g*L + L - 1 live on GPU g */
    int32_t total_nodes;
    int32_t variant;          /* ALLRED_BO / ALLRED_LO / ALLRED_MEM, as executed      */
    int32_t mode;             /* ALLRED_MULTI_*                                      */
    int32_t print_core;       /* validated with the reference's printed report        */
    uint64_t elems;           /* bf16 elements per rank                              */
    uint64_t validated_mask;  /* bit r: rank r goes through validate_result_vector    */
    allred_dist_desc desc;    /* the exchange every GPU runs (FLAT / HIER)            */
} allred_multi_plan;
/* check_all != 0: every rank validated (ALLRED_CHECK_ALL), else print_core and
 * every GPU's first rank.  ALLRED_ERR_ARG / _SCHEDULE / _UNSUPPORTED exactly
 * where allred_run refuses the split (before any HIP call). */
int allred_multi_plan_build(const allred_args* args, int check_all, allred_multi_plan* out);
typedef struct {
    int32_t transport;        /* ALLRED_TRANSPORT_*                                  */
    int32_t share_device;     /* 1: every group on args->device (PEER / HOST only)     */
    int32_t timeout_ms;       /* RCCL deadline (0 = default); HOST: exchange deadline */
    int32_t reserved;
} allred_multi_opts;
/* allred_run's multi-GPU form with an explicit backend.  in_all: NULL (the
 * reference's generated inputs, validated as allred_run does), or total * elems
 * bf16 rank-major inputs of the caller's own (arbitrary data: validation is
 * skipped, report->mismatches = -1).  out_all: NULL, or total * elems bf16
 * receiving every rank's result (rank-major) for checks. */
int allred_run_multi(const allred_args* args, const allred_multi_opts* opts, int verbose, allred_report* report,
                     const uint16_t* in_all, uint16_t* out_all);

/* ======================================================================
 * Peer-mapped one-shot allreduce across GPUs: the shared-memory variant
 * (allred_mem_2D.cpp:4-165) with every GPU's window IPC-mapped into every
 * peer (one process per GPU).  Result semantics = allred_mem_2D: block b is
 * owner b's copy + every other rank's copy in rank order, fp32, one rounding.
 *   create -> handle (256 bytes, exchange with every rank) -> connect(all
 *   handles in rank order) -> allreduce ... -> destroy.
 * Barriers spin with a bound; allred_peer_status() reports bit 0 = timeout,
 * and the WIN/FLAGS_CACHED bits when uncached (fine-grained) device memory
 * was unavailable and ordinary hipMalloc memory had to be used instead.
 * A timed-out call has produced wrong bytes: callers must check the status
 * (allred_peer_status after the stream, or allred_peer_check) before using
 * results; the first timeout makes every later wait of that launch give up.
 * ==================================================================== */
#define ALLRED_PEER_HANDLE_BYTES 256
/* largest IPC-exported window: a peer's hipIpcOpenMemHandle of a ~2 GiB
 * allocation never returned on the MI355X boxes (profiles/r01_peer_open_probe_2gib_hang.txt),
 * so allred_peer_create rejects max_elems * 2 > 1 GiB (ALLRED_ERR_ARG) */
#define ALLRED_PEER_MAX_WINDOW_BYTES (1ull << 30)
#define ALLRED_PEER_TIMEOUT 0x1u
#define ALLRED_PEER_WIN_CACHED 0x100u
#define ALLRED_PEER_FLAGS_CACHED 0x200u
typedef struct allred_peer allred_peer;
int allred_peer_create(int nranks, int rank, int device, uint64_t max_elems, allred_peer** out);
int allred_peer_handle(allred_peer* peer, uint8_t* handle /*[ALLRED_PEER_HANDLE_BYTES]*/);
int allred_peer_connect(allred_peer* peer, const uint8_t* all_handles /*[nranks * ALLRED_PEER_HANDLE_BYTES]*/);
/* The peers of ONE process (peers[q] = rank q, one host thread per rank
 * afterwards): every window mapped into every peer directly, no IPC (peer
 * access enabled between distinct devices).  Replaces handle + connect when
 * the ranks are threads (allred_run across GPUs, ALLRED_TRANSPORT_PEER). */
int allred_peer_connect_all(int nranks, allred_peer* const* peers);
/* elems % (8 * nranks) == 0, elems <= max_elems.  local_ranks > 1: `buf`
 * holds local_ranks virtual ranks (stride elems) reduced on-GPU first
 * (tree of local rank 0) into `workspace` (elems * 2 bytes), then broadcast. */
int allred_peer_allreduce(allred_peer* peer, uint16_t* buf, uint64_t elems, int local_ranks, int local_side,
                          int local_algo, void* workspace, void* stream);
/* The hierarchical step of allred_peer_allreduce (64 local ranks per GPU, the
 * same result bits) PIPELINED across consecutive buckets, two deep
 * (k_hier_x2): the call with cur starts it
 * (tree, partials pushed to the owners), sums the owned tiles of the bucket
 * the previous call started and writes the rank rows of the bucket started
 * two calls earlier; cur == NULL (flush) finishes every pending bucket in one
 * launch.  K buckets = K + 1 calls: b0, b1, ..., b_{K-1}, NULL.  A bucket's
 * rows are final, in stream order, after the call that started the bucket
 * two calls later (or the flush); keep it alive until then.  Every poll of a
 * launch waits for pushes of the previous launch on the other GPUs, so a GPU
 * up to one launch late stalls nobody.  While buckets are pending, the other
 * peer allreduce calls return ALLRED_ERR_ARG; so does another bucket size
 * mid-sequence or a flush with nothing pending.  ALLRED_ERR_UNSUPPORTED:
 * local_ranks != 64, more than 8 GPUs, flags not uncached, or a bucket beyond
 * the hand-off area (elems > min(max_elems, 4 Mi)).  Any grid cap
 * (allred_peer_set_max_groups) works: a workgroup runs any number of tiles, its
 * results staged in LDS 8 tiles at a time.  (The one-deep form of rounds 3-5,
 * k_hier_x, is retired: 15.1-15.3 us at W = 1 against this form's 15.0.)
 * No reference counterpart (the reference runs one vector per program). */
int allred_peer_allreduce_pipelined2(allred_peer* peer, uint16_t* cur, uint64_t elems, int local_ranks,
                                     int local_side, int local_algo, void* stream);
/* Buckets of at most `bytes` (default 4 MiB) run as one kernel (per-workgroup
 * flags, no kernel boundaries); larger ones as copy / barrier / reduce-scatter /
 * barrier / all-gather launches.  Same result bits either way.  Every rank
 * must use the same setting. */
int allred_peer_set_oneshot_max(allred_peer* peer, uint64_t bytes);
/* enable = 1 (the default): with local_ranks == 64 and nranks <= 8,
 * allred_peer_allreduce runs the hierarchical step as ONE kernel, k_hier_ws,
 * with LL hand-offs (each cross-GPU transfer a push of self-validating 8-byte
 * data+epoch words into the consumer's own memory; no flags, no remote reads)
 * and reducing and writing waves in every workgroup, so each CU reads and
 * writes at once, for buckets of up to min(max_elems, 4 Mi) elements that are
 * a multiple of 256 x nranks (others run the launch form).  0 = the launch
 * form (tree, the mem_2D exchange, broadcast as launches).  Same result bits
 * either way (allred_mem_2D semantics over the per-GPU trees); other values
 * ALLRED_ERR_ARG.  Every rank must use the same setting.  Replaces nothing in
 * the reference (its mem_2D phases sync through semaphores,
 * allred_mem_2D/kernels/dataflow_kernel.cpp:201-230).  (Retired forms and
 * their numbers at W = 1, profiles/README.md: k_hier_ll — the three phases in
 * sequence, 16.2 us vs k_hier_ws's 14.5-14.6 — in round 6; the per-tile flag
 * form, 19.9 us, and the pipelined LL form, 17.8 us, in round 5; the
 * specialised-wave form of round 1, 27-38 us.)  ABI 7: 2 is no longer a value. */
int allred_peer_set_hier_ll(allred_peer* peer, int enable);
/* Caps the grid of the hierarchical one-kernel forms, k_peer_mem_ll and the
 * scheduled form (allred_peer_dist_allreduce) at `groups` workgroups (0 =
 * default: 512 for the hierarchical forms, two per CU, 256 for the scheduled
 * form; the whole grid resident on a GPU of its own).
 * Their workgroups wait for each other across processes, so when several
 * processes share one GPU (rehearsals) the sum of their grids must fit at once:
 * groups <= 512 / processes.  Same result bits at any cap. */
int allred_peer_set_max_groups(allred_peer* peer, uint32_t groups);
/* allred_peer_dist_allreduce runs one-channel LO buckets of at most `bytes`
 * (default 256 KiB; 0 = never) with LL hand-offs (k_peer_lo_ll: each step
 * pushes data+epoch words into the partner's memory and polls its own — one
 * one-way xGMI trip per step instead of a flag and a remote read).  Same
 * result bits.  Every rank must use the same setting.  Replaces the semaphore
 * handshake + NoC write of allred_LOO_2D/kernels/dataflow_kernel.cpp:127-175. */
int allred_peer_set_lo_ll_max(allred_peer* peer, uint64_t bytes);
/* allred_peer_allreduce (mem_2D) runs buckets of at most `bytes` (default
 * 256 KiB; 0 = never) with LL hand-offs (k_peer_mem_ll: block copies pushed to
 * their owners, owners push the sums; two one-way xGMI trips, no flags, no
 * remote reads), larger ones as before.  Same result bits.  Every rank must
 * use the same setting. */
int allred_peer_set_mem_ll_max(allred_peer* peer, uint64_t bytes);
/* allred_peer_dist_allreduce runs BO buckets of at least `min_bytes` (default
 * 0 = never) in the PUSH form (k_peer_sched_push): each exchange is written by
 * the sender into the receiver's staging window (reduce-scatter) or main window
 * (all-gather) and announced with a flag, instead of read by the receiver
 * over xGMI — posted writes, no read round trips.  Same program, same adds,
 * same result bits.  Every rank must use the same setting.  Replaces the NoC
 * writes of allred_BO_2D/kernels/dataflow_kernel.cpp:152-267 (the reference's
 * sender also writes into the receiver's L1). */
int allred_peer_set_sched_push(allred_peer* peer, uint64_t min_bytes);
/* The allred_dist_allreduce program (same desc, same result bits: Swing /
 * RecDub BO or LO, link-spreading channels, hierarchical local ranks) with
 * RCCL replaced by direct reads of the partners' IPC-mapped windows: one
 * kernel, each step waits only for its partner (allred_BO_2D
 * dataflow_kernel.cpp:152-267 semaphore handshakes, over xGMI).
 * desc->variant ALLRED_MEM runs allred_peer_allreduce (fp32 accumulation only: mem_accum
 * ALLRED_ACC_BF16 -> ALLRED_ERR_UNSUPPORTED; RCCL runs it).  desc->total_nodes
 * must equal nranks; elems <= max_elems (BO) or max_elems / 2 (LO);
 * workspace: allred_dist_workspace_bytes(desc) bytes when local_ranks > 1. */
int allred_peer_dist_allreduce(allred_peer* peer, const allred_dist_desc* desc, uint16_t* buf, void* workspace,
                               void* stream);
int allred_peer_status(allred_peer* peer, uint32_t* status);
/* Synchronises `stream` and returns ALLRED_ERR_TRANSPORT if any call so far
 * timed out (ALLRED_PEER_TIMEOUT), else ALLRED_OK. */
int allred_peer_check(allred_peer* peer, void* stream);
/* Clears the status word (ALLRED_PEER_TIMEOUT is sticky: once set, every later bounded
 * wait of this peer gives up at once) through the null stream, and nothing else.  Call
 * with no kernel of this peer in flight (after allred_peer_check).  The call counter
 * keeps advancing, so the next call's LL words and flags carry epochs no timed-out call
 * wrote.  Returns ALLRED_ERR_ARG while a pipelined sequence (allred_peer_allreduce_pipelined2)
 * is pending: finish it first.  ABI 5. */
int allred_peer_clear_status(allred_peer* peer);
int allred_peer_destroy(allred_peer* peer);

#ifdef __cplusplus
}
#endif
#endif /* ALLRED_H */
