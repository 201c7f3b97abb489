// kernels.hip — CDNA4 (gfx950) kernels of the virtual-rank engine (P ranks
// resident in one GPU's HBM) and the bf16 tile add of the multi-GPU paths.
//
// Every kernel is HBM-bound bf16 streaming work (device.hpp): 16-byte
// (8 x bf16) accesses per lane, fp32 add, v_cvt_pk_bf16_f32 back to bf16.
// No MFMA: a pointwise add is not a contraction.
//
// Replaces the Tensix compute kernels of the reference:
//   add_tiles + pack_tile<true>      allred_BO_2D/kernels/compute_kernel.cpp:53-60
//   LO_2D add loop                   allred_LO_2D/kernels/compute_kernel.cpp:50-62
//   mem_2D dest-reuse accumulate     allred_mem_2D/kernels/compute_kernel.cpp:43-72
// and the NoC block moves of the dataflow kernels (RS / AG loops,
// allred_BO_2D/kernels/dataflow_kernel.cpp:152-267) for ranks resident in
// one GPU's HBM, where a "send" is a load of the partner's bytes.
// Kernel selection is fixed (the measured product forms);
// allred_tune_set (tune.cpp) switches between bit-identical forms for A/B.
#include <utility>

#include "device.hpp"

namespace tsa {
namespace {

// LO DAGs of the non-rank-uniform Swing schedules (generated at build time
// from the schedule by csrc/gen_lo_dag.cpp): struct LoDag<i> + TSA_LO_DAGS(X)
#include "lo_dag_gen.inc"

// ---------------------------------------------------------------------------
// dst += src over n_vec 16-byte vectors: one vector per lane (grid covers the
// whole range; the loop only runs past 2^31 threads).  Many short-lived waves
// stream HBM better than a capped grid-stride loop (6.4 vs 5.0 TB/s at 256 MiB).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_add(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                uint64_t n_vec) {
    for (uint64_t i = gtid(); i < n_vec; i += gthreads()) st_nt(dst + i, add8(ld_nt(dst + i), ld_nt(src + i)));
}

__global__ void k_add_scalar(uint16_t* __restrict__ dst, const uint16_t* __restrict__ src, uint64_t n) {
    for (uint64_t i = gtid(); i < n; i += gthreads()) {
        float s = __uint_as_float((uint32_t)dst[i] << 16) + __uint_as_float((uint32_t)src[i] << 16);
        dst[i] = (uint16_t)(pack_rne(s, 0.0f) & 0xffffu);
    }
}

// ---------------------------------------------------------------------------
// dst[seg] += src[seg] for a list of segments (offsets / lengths in 16-byte
// vectors), grid.y = segment: the BO compute loop of compute_kernel.cpp:35-67
// for one step — every received block run of every link-spreading channel of
// an RCCL step (dist.cpp) in ONE launch, or the blocks of one 64-bit mask.
// ---------------------------------------------------------------------------
struct SegList {
    uint64_t off[kMaxAddSegs];
    uint64_t len[kMaxAddSegs];
};

__global__ __launch_bounds__(kBlock) void k_add_segs(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                     SegList segs) {
    const uint64_t off = segs.off[blockIdx.y], len = segs.len[blockIdx.y];
    for (uint64_t v = gtid(); v < len; v += gthreads())
        st_nt(dst + off + v, add8(ld_nt(dst + off + v), ld_nt(src + off + v)));
}

// ---------------------------------------------------------------------------
// BO allreduce of P ranks in one pass.  Block b of the result is what the
// reference's reduce-scatter computes at b's owner: a binary tree whose leaf
// order is order[b] (allred_schedule.tree_order, row stride 64) and whose
// level-k nodes add adjacent groups of 2^k leaves, each add rounded to bf16.
// The all-gather then copies it to every rank, so the pass stores it to all.
// block_vec == 0 selects row 0 for the whole vector (hierarchical partials).
//
// Lane layout (P = 64): lane = g * CH + c.  The 8 lanes of chunk column c
// each load 8 leaves (ranks order[b][8g .. 8g+7]) of the same 16-byte chunk,
// reduce them locally (tree levels 0-2), then combine across lanes with
// xor-shuffles (levels 3-5).  Every lane then holds the result and stores it
// to its own 8 ranks.  Each rank's chunk is read and written by one lane only,
// so the pass is safe in place.  (Shapes the LDS forms below do not take.)
// ---------------------------------------------------------------------------
template <int P, bool WRITE_ALL>
__global__ __launch_bounds__(kBlock) void k_tree(uint16_t* __restrict__ ranks, uint64_t stride, uint64_t n_vec,
                                                 const uint8_t* __restrict__ order, uint64_t block_vec,
                                                 uint16_t* __restrict__ out) {
    constexpr int LEAVES = P >= 8 ? 8 : P;  // leaves per lane
    constexpr int LANES = P / LEAVES;        // lanes per chunk
    constexpr int CH = 64 / LANES;           // chunks per wave
    const int lane = threadIdx.x & 63;
    const int g = lane / CH;
    const int c = lane % CH;
    uint4* rows[LEAVES];
    uint64_t cur = ~0ull;
    const uint64_t wave = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const uint64_t waves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t base = wave * CH; base < n_vec; base += waves * CH) {
        const uint64_t v = base + c;
        const bool ok = v < n_vec;
        const uint64_t b = (block_vec && ok) ? v / block_vec : 0;
        if (b != cur) {  // wave-uniform whenever block_vec % CH == 0
            cur = b;
#pragma unroll
            for (int i = 0; i < LEAVES; ++i)
                rows[i] = reinterpret_cast<uint4*>(ranks + (uint64_t)order[b * ALLRED_MAX_NODES + g * LEAVES + i] * stride);
        }
        uint4 x[LEAVES];
#pragma unroll
        for (int i = 0; i < LEAVES; ++i) x[i] = ok ? ld_nt(rows[i] + v) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int w = 1; w < LEAVES; w *= 2)
#pragma unroll
            for (int i = 0; i < LEAVES; i += 2 * w) x[i] = add8(x[i], x[i + w]);
        uint4 acc = x[0];
#pragma unroll
        for (int m = CH; m < 64; m *= 2) acc = add8(acc, shfl_xor4(acc, m));
        if (ok) {
            if (WRITE_ALL) {
#pragma unroll
                for (int i = 0; i < LEAVES; ++i) st_nt(rows[i] + v, acc);
            } else if (g == 0) {
                reinterpret_cast<uint4*>(out)[v] = acc;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// The same BO pass staged through LDS (the shipped form for P >= 8): one
// workgroup = one tile of 256 elements (512 B) of all P ranks.  HBM -> LDS by
// global_load_lds, 1 KiB contiguous per wave-instruction (two ranks' rows);
// the LDS tile turns the rank-major HBM layout into the per-column leaf reads
// of the tree; the result row leaves with 1 KiB contiguous wave-stores.
// Wave w stages ranks [P/4 w, P/4 (w+1)) and reduces tree positions
// [P/4 w, P/4 (w+1)) of every column (lane = h * 32 + column: h picks the
// half, levels below P/8 in registers, one xor-32 shuffle); the four wave
// partials meet in LDS rows 0-3 (free once every wave has read its leaves).
// 16.0 us vs 17.3 us for k_tree at 64 x 640 kB (= a 42+42 MB copy's time).
// ---------------------------------------------------------------------------
template <int P, bool WRITE_ALL>
__global__ __launch_bounds__(kBlock) void k_tree_lds(uint16_t* __restrict__ ranks, uint64_t stride,
                                                     const uint8_t* __restrict__ order, uint64_t block_vec,
                                                     uint16_t* __restrict__ out) {
    constexpr int TV = 32;          // 16-byte vectors per rank row of a tile
    constexpr int RPW = P / 4;      // ranks staged (and tree leaves reduced) per wave
    constexpr int LPL = RPW / 2;    // leaves per lane
    __shared__ __attribute__((aligned(16))) uint4 tile[P * TV];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane & 31, h = lane >> 5;
    const uint64_t v0 = (uint64_t)blockIdx.x * TV;
#pragma unroll
    for (int k = 0; k < RPW / 2; ++k) {
        const int r = RPW * w + 2 * k + h;
        const uint4* src = reinterpret_cast<const uint4*>(ranks + (uint64_t)r * stride) + v0 + c;
        __builtin_amdgcn_global_load_lds((global_u32*)src, (lds_u32*)&tile[(RPW * w + 2 * k) * TV], 16, 0, 2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint8_t* ord = order + (block_vec ? v0 / block_vec : 0) * ALLRED_MAX_NODES + RPW * w + LPL * h;
    uint4 x[LPL];
#pragma unroll
    for (int i = 0; i < LPL; ++i) x[i] = tile[(int)ord[i] * TV + c];
#pragma unroll
    for (int s = 1; s < LPL; s *= 2)
#pragma unroll
        for (int i = 0; i < LPL; i += 2 * s) x[i] = add8(x[i], x[i + s]);
    const uint4 part = add8(x[0], shfl_xor4(x[0], 32));
    __syncthreads();
    if (h == 0) tile[w * TV + c] = part;
    __syncthreads();
    const uint4 res = add8(add8(tile[0 * TV + c], tile[1 * TV + c]), add8(tile[2 * TV + c], tile[3 * TV + c]));
    if (!WRITE_ALL) {  // hierarchical partial: one row out
        if (w == 0 && h == 0) st_nt(reinterpret_cast<uint4*>(out) + v0 + c, res);
        return;
    }
#pragma unroll
    for (int k = 0; k < RPW / 2; ++k) {
        const int r = RPW * w + 2 * k + h;
        st_nt(reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + v0 + c, res);
    }
}

// ---------------------------------------------------------------------------
// k_tree_lds on a persistent grid with two LDS tile buffers: tile j+1's loads
// are issued before tile j is reduced and stored, and the wait before tile j
// is an exact vmcnt that leaves tile j-1's stores in flight.  Used on pinned
// HOST buckets (zero-copy end to end: both PCIe directions run at once), for
// 8 / 16 / 32-rank buckets on HBM, and (WRITE_ALL = false) for the
// hierarchical partial: the tree of every tile goes to `out` (one row; wave 0
// keeps its one partial store in flight, the other waves wait for their loads
// alone).  Tiles of a workgroup are blockIdx.x + j * G, so the workgroups in
// flight together read adjacent 512-byte segments of every rank row (a
// contiguous run per workgroup measured 18.8 vs 15.6 us: DRAM page locality
// across workgroups is what counts).
// ---------------------------------------------------------------------------
template <int P, bool WRITE_ALL = true>
__global__ __launch_bounds__(kBlock) void k_tree_lds_pipe(uint16_t* __restrict__ ranks, uint64_t stride,
                                                          const uint8_t* __restrict__ order, uint64_t block_vec,
                                                          uint64_t ntiles, uint16_t* __restrict__ out) {
    constexpr int TV = 32, RPI = 2, RPW = P / 4, OPS = RPW / RPI, LPL = OPS;
    static_assert(OPS >= 1, "P >= 8");
    __shared__ __attribute__((aligned(16))) uint4 buf[2][P * TV];
    __shared__ __attribute__((aligned(16))) uint4 part[4 * TV];
    __shared__ __attribute__((aligned(16))) uint8_t ord_lds[P * ALLRED_MAX_NODES];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane % TV, q = lane / TV;
    const uint32_t wbase = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&buf[0][0] + (uint32_t)(RPW * w * TV * 16));
    auto issue = [&](uint64_t t, int b) {
#pragma unroll
        for (int k = 0; k < OPS; ++k) {
            const int r = RPW * w + RPI * k + q;
            const uint4* src = reinterpret_cast<const uint4*>(ranks + (uint64_t)r * stride) + t * TV + c;
            lds_dma16(src, wbase + (uint32_t)(b * P * TV * 16 + RPI * k * TV * 16));
        }
    };
    const uint64_t G = gridDim.x;
    const int mine = blockIdx.x < ntiles ? (int)((ntiles - 1 - blockIdx.x) / G + 1) : 0;
    // the order rows of all P blocks, once, then the first tile's loads
    for (int i = threadIdx.x; i < P * ALLRED_MAX_NODES / 16; i += kBlock)
        reinterpret_cast<uint4*>(ord_lds)[i] = reinterpret_cast<const uint4*>(order)[i];
    __syncthreads();
    if (mine > 0) issue(blockIdx.x, 0);
    for (int j = 0; j < mine; ++j) {
        if (WRITE_ALL) wait_tile<OPS, 1>(j < 1 ? j : 1);
        else if (j > 0 && w == 0) wait_vm<1>();   // tile j-1's partial store may stay in flight
        else wait_vm<0>();
        lds_barrier();
        if (j + 1 < mine) issue(blockIdx.x + (uint64_t)(j + 1) * G, (j + 1) & 1);
        const uint4* tile = buf[j & 1];
        const uint64_t v0 = (blockIdx.x + (uint64_t)j * G) * TV;
        const uint8_t* ord = ord_lds + (block_vec ? v0 / block_vec : 0) * ALLRED_MAX_NODES + RPW * w + LPL * q;
        uint4 x[LPL];
#pragma unroll
        for (int i = 0; i < LPL; ++i) x[i] = tile[(int)ord[i] * TV + c];
#pragma unroll
        for (int s = 1; s < LPL; s *= 2)
#pragma unroll
            for (int i = 0; i < LPL; i += 2 * s) x[i] = add8(x[i], x[i + s]);
        const uint4 pw = add8(x[0], shfl_xor4(x[0], 32));   // tree level across the two lane halves
        if (q == 0) part[w * TV + c] = pw;
        lds_barrier();
        const uint4 res = add8(add8(part[0 * TV + c], part[1 * TV + c]), add8(part[2 * TV + c], part[3 * TV + c]));
        if (!WRITE_ALL) {
            if (w == 0 && q == 0) st_nt(reinterpret_cast<uint4*>(out) + v0 + c, res);
            continue;
        }
#pragma unroll
        for (int k = 0; k < OPS; ++k) {
            const int r = RPW * w + RPI * k + q;
            st_nt(reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + v0 + c, res);
        }
    }
}

// ---------------------------------------------------------------------------
// k_tree_lds_lag: the fused BO pass (the bench kernel at config 2; same tree,
// same bits as k_tree_lds) on a persistent grid of two workgroups per CU with
// every tile's stores one iteration late.  Iteration j: wait for tile j's
// loads (one exact vmcnt), reduce it out of LDS, then issue tile j+2's loads
// into its buffer (early release) interleaved op by op with the stores of
// tile j-1's result, kept in registers from the previous iteration.  A tile's
// stores thus always queue behind the next tile's loads and a wave never
// waits for a store before a load.  Issue order per wave: L0 L1 | L2 | L3 S0 |
// L4 S1 | ..., so after tile j's loads come tile j+1's loads and the stores of
// tiles j-2 and j-3.  The 4 KiB tree order table's load goes out first, then
// the first two tiles' loads, and only the table's load is waited for before
// it is staged into LDS.  Measured arms (the table first, an LDS-counter
// barrier, 2 / 8 waves, 1 KiB rows, other interleave orders) and their
// numbers: DESIGN.md §4, tools/ubench/fused_ab.hip.
// ---------------------------------------------------------------------------
template <int P>
__global__ __launch_bounds__(kBlock) void k_tree_lds_lag(uint16_t* __restrict__ ranks, uint64_t stride,
                                                         const uint8_t* __restrict__ order, uint64_t block_vec,
                                                         uint64_t t0, uint64_t ntiles) {
    constexpr int NW = 4, TV = 32, RPI = 2, RPW = P / NW, OPS = RPW / RPI, LPL = OPS;
    static_assert(OPS >= 1 && 3 * OPS <= 63, "vmcnt is 6 bits");
    __shared__ __attribute__((aligned(16))) uint4 buf[2][P * TV];
    __shared__ __attribute__((aligned(16))) uint4 part[2][NW * TV];
    __shared__ __attribute__((aligned(16))) uint8_t ord_lds[P * ALLRED_MAX_NODES];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane % TV, q = lane / TV;
    const uint32_t wbase = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&buf[0][0] + (uint32_t)(RPW * w * TV * 16));
    auto row = [&](int k) { return ranks + (uint64_t)(RPW * w + RPI * k + q) * stride; };
    auto issue = [&](uint64_t t, int b) {
#pragma unroll
        for (int k = 0; k < OPS; ++k)
            lds_dma16(reinterpret_cast<const uint4*>(row(k)) + t * TV + c,
                      wbase + (uint32_t)(b * P * TV * 16 + RPI * k * TV * 16));
    };
    const uint64_t G = gridDim.x;
    const int mine = blockIdx.x < ntiles ? (int)((ntiles - 1 - blockIdx.x) / G + 1) : 0;
    auto tile_of = [&](int j) { return t0 + blockIdx.x + (uint64_t)j * G; };   // tiles t0 .. t0 + ntiles - 1
    // the 4 KiB order table (16 bytes per thread) is loaded ahead of the first two tiles
    // and waited for exactly, so tile 0's tree waits for tile 0 only, not for tile 1 too
    // (a compiler-issued load would be followed by vmcnt(0): it cannot see the LDS-DMA ops)
    static_assert(P * ALLRED_MAX_NODES == 16 * 64 * NW, "one 16-byte load per thread");
    u32x4 ov;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(ov) : "v"(reinterpret_cast<const uint4*>(order) + threadIdx.x) : "memory");
    if (mine > 0) issue(tile_of(0), 0);
    if (mine > 1) issue(tile_of(1), 1);
    if (mine > 1) wait_vm<2 * OPS>(); else if (mine > 0) wait_vm<OPS>(); else wait_vm<0>();
    asm volatile("" : "+v"(ov));   // no use of ov may move above the wait
    reinterpret_cast<u32x4*>(ord_lds)[threadIdx.x] = ov;
    lds_barrier();
    uint4 prev = make_uint4(0, 0, 0, 0);
    for (int j = 0; j < mine; ++j) {
        // after L(j): the last op of S(j-3) (interleaved with L(j)), L(j+1), S(j-2)
        wait_any((j >= 3 ? 1 : 0) + (j + 1 < mine ? OPS : 0) + (j >= 2 ? OPS : 0));
        lds_barrier();   // every wave's rows of tile j are in LDS
        const uint4* tile = buf[j & 1];
        const uint64_t t = tile_of(j), v0 = t * TV;
        const uint8_t* ord = ord_lds + (block_vec ? v0 / block_vec : 0) * ALLRED_MAX_NODES + RPW * w + LPL * q;
        uint4 x[LPL];
#pragma unroll
        for (int i = 0; i < LPL; ++i) x[i] = tile[(int)ord[i] * TV + c];
#pragma unroll
        for (int s = 1; s < LPL; s *= 2)
#pragma unroll
            for (int i = 0; i < LPL; i += 2 * s) x[i] = add8(x[i], x[i + s]);
        const uint4 pw = add8(x[0], shfl_xor4(x[0], 32));   // tree level across the two lane halves
        if (q == 0) part[j & 1][w * TV + c] = pw;
        lds_barrier();   // every wave has read tile j out of buf[j & 1]; the partials are in
        {   // tile j+2's loads and tile j-1's stores, interleaved op by op
            const uint64_t tl = tile_of(j + 2), ts = tile_of(j - 1);
            const uint32_t bl = wbase + (uint32_t)((j & 1) * P * TV * 16);
#pragma unroll
            for (int k = 0; k < OPS; ++k) {
                if (j + 2 < mine)
                    lds_dma16(reinterpret_cast<const uint4*>(row(k)) + tl * TV + c, bl + (uint32_t)(RPI * k * TV * 16));
                if (j >= 1) st_nt(reinterpret_cast<uint4*>(row(k)) + ts * TV + c, prev);
            }
        }
        const uint4* pp = part[j & 1];
        prev = add8(add8(pp[0 * TV + c], pp[1 * TV + c]), add8(pp[2 * TV + c], pp[3 * TV + c]));
    }
    if (mine > 0) {
#pragma unroll
        for (int k = 0; k < OPS; ++k) st_nt(reinterpret_cast<uint4*>(row(k)) + tile_of(mine - 1) * TV + c, prev);
    }
}

// ---------------------------------------------------------------------------
// k_tree_bcast_x: the two HBM phases of the hierarchical step of CONSECUTIVE
// buckets in one pass (allred_dist_allreduce_pipelined: tree -> RCCL program ->
// broadcast per bucket, the broadcast of bucket i and the tree of bucket i+1
// fused).  Tile j: bucket i+1's 64 rank rows are reduced with the tree of rank 0
// of the local grid into its partial (one row out, same tree and bits as
// k_tree_lds_pipe<64, false>), and bucket i's allreduced partial tile is
// written to bucket i's 64 rank rows (k_broadcast's data movement).  Reads and
// writes of the two buckets overlap as in the fused one-bucket pass, where one
// bucket's tree then broadcast run as a read-only launch, then a write-only one.
// Schedule (k_tree_lds_lag's, stores not lagged: their data does not depend on
// the tree): iteration j waits for tile j's loads (bucket i+1's rows by LDS-DMA,
// and — wave 0 — bucket i's result tile by LDS-DMA into a small slot), reduces
// tile j, writes its partial (wave 0), then issues tile j+2's loads interleaved
// op by op with the 64 row stores of bucket i's tile j.  Per-wave exact vmcnt:
// wave 0 issues the result loads and the partial stores, the others do not.
// ---------------------------------------------------------------------------
// LAG 0: bucket i's tile j rows stored in iteration j; 1: in iteration j + 1.
// BAL: every wave stages 8 columns of the result tile and stores 8 columns of the
// partial (equal memory queues); else wave 0 does both for all 32 columns.
template <int LAG, bool BAL>
__global__ __launch_bounds__(kBlock) void k_tree_bcast_x(uint16_t* __restrict__ cur, uint16_t* __restrict__ prev,
                                                         uint64_t stride, const uint8_t* __restrict__ order,
                                                         uint16_t* __restrict__ cur_partial,
                                                         const uint16_t* __restrict__ prev_result, uint64_t t0,
                                                         uint64_t ntiles) {
    constexpr int P = 64, NW = 4, TV = 32, RPI = 2, RPW = P / NW, OPS = RPW / RPI, LPL = OPS;
    static_assert(2 * OPS + 3 <= 63, "vmcnt is 6 bits");
    static_assert(LAG == 0 || LAG == 1, "lag of the row stores: 0 or 1 iteration");
    __shared__ __attribute__((aligned(16))) uint4 buf[2][P * TV];
    __shared__ __attribute__((aligned(16))) uint4 part[2][NW * TV];
    __shared__ __attribute__((aligned(16))) uint4 res_lds[2][64];   // bucket i's result tile (wave 0: two copies)
    __shared__ __attribute__((aligned(16))) uint8_t ord_lds[ALLRED_MAX_NODES];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane % TV, q = lane / TV;
    const bool w0 = w == 0;
    const bool hasr = BAL || w0;   // this wave issues result loads and partial stores
    const uint32_t wbase = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&buf[0][0] + (uint32_t)(RPW * w * TV * 16));
    const uint32_t rbase = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&res_lds[0][0]);
    auto crow = [&](int k) { return cur + (uint64_t)(RPW * w + RPI * k + q) * stride; };
    auto prow = [&](int k) { return prev + (uint64_t)(RPW * w + RPI * k + q) * stride; };
    const uint64_t G = gridDim.x;
    const int mine = blockIdx.x < ntiles ? (int)((ntiles - 1 - blockIdx.x) / G + 1) : 0;
    auto tile_of = [&](int j) { return t0 + blockIdx.x + (uint64_t)j * G; };
    const uint32_t rbase_w = __builtin_amdgcn_readfirstlane(rbase + (uint32_t)(w * 128));   // BAL: this wave's 8 columns
    auto issue_res = [&](uint64_t t, int slot) {   // bucket i's result tile t into res_lds[slot]
        if (BAL) {
            if (lane < 8)
                lds_dma16(reinterpret_cast<const uint4*>(prev_result) + t * TV + 8 * w + lane,
                          rbase_w + (uint32_t)(slot * 1024));
        } else if (w0) {
            lds_dma16(reinterpret_cast<const uint4*>(prev_result) + t * TV + c, rbase + (uint32_t)(slot * 1024));
        }
    };
    auto issue_loads = [&](int j) {   // tile j of bucket i+1 into buf[j & 1]; wave 0: bucket i's result tile j
        const uint64_t t = tile_of(j);
#pragma unroll
        for (int k = 0; k < OPS; ++k)
            lds_dma16(reinterpret_cast<const uint4*>(crow(k)) + t * TV + c,
                      wbase + (uint32_t)((j & 1) * P * TV * 16 + RPI * k * TV * 16));
        issue_res(t, j & 1);
    };
    const int own = hasr ? 1 : 0;   // the extra ops per tile: the result load (and the partial store)
    // the 64-byte tree order of local rank 0 (one byte per lane of wave 0), ahead of the first tiles' loads
    uint32_t ob = 0;
    if (w0) ob = order_byte_load(order, lane);
    if (mine > 0) issue_loads(0);
    if (mine > 1) issue_loads(1);
    if (w0) {
        wait_any((mine > 0 ? OPS + 1 : 0) + (mine > 1 ? OPS + 1 : 0));
        asm volatile("" : "+v"(ob));   // no use of ob may move above the wait
        ord_lds[lane] = (uint8_t)ob;
    }
    lds_barrier();
    uint4 pres = make_uint4(0, 0, 0, 0);   // LAG 1: bucket i's result of the previous tile
    for (int j = 0; j < mine; ++j) {
        // ops issued after tile j's last load (its DMAs, then wave 0's result load): j = 0 ->
        // tile 1's loads; j = 1 -> iteration 0; j >= 2 -> the last row store interleaved behind
        // tile j's last DMA (a store of tile j-2-LAG: non-zero waves only, wave 0's result load
        // comes after it) and iteration j-1: partial (wave 0), tile j+1's loads, row stores
        const int next = j + 1 < mine ? OPS + own : 0;
        if (j == 0) wait_any(next);
        else wait_any((j >= 2 + LAG && !hasr ? 1 : 0) + own + next + (j - 1 >= LAG ? OPS : 0));
        lds_barrier();   // every wave's rows of tile j and wave 0's result tile are in LDS
        const uint4* tile = buf[j & 1];
        const uint64_t t = tile_of(j), v0 = t * TV;
        const uint4 pnew = res_lds[j & 1][c];   // bucket i's result, read before the slot is reloaded
        const uint8_t* ord = ord_lds + RPW * w + LPL * q;
        uint4 x[LPL];
#pragma unroll
        for (int i = 0; i < LPL; ++i) x[i] = tile[(int)ord[i] * TV + c];
#pragma unroll
        for (int s = 1; s < LPL; s *= 2)
#pragma unroll
            for (int i = 0; i < LPL; i += 2 * s) x[i] = add8(x[i], x[i + s]);
        const uint4 pw = add8(x[0], shfl_xor4(x[0], 32));   // tree level across the two lane halves
        if (q == 0) part[j & 1][w * TV + c] = pw;
        lds_barrier();   // tile j and result slot j & 1 are read by every wave; the partials are in
        if (hasr) {
            const uint4* pp = part[j & 1];
            const uint4 r = add8(add8(pp[0 * TV + c], pp[1 * TV + c]), add8(pp[2 * TV + c], pp[3 * TV + c]));
            if (q == 0 && (!BAL || (c >> 3) == w)) st_nt(reinterpret_cast<uint4*>(cur_partial) + v0 + c, r);
        }
        {   // tile j+2's loads and bucket i's row stores (tile j - LAG), interleaved op by op
            const uint64_t tl = tile_of(j + 2), ts = tile_of(j - LAG);
            const uint4 sv = LAG ? pres : pnew;
            const uint32_t bl = wbase + (uint32_t)((j & 1) * P * TV * 16);
#pragma unroll
            for (int k = 0; k < OPS; ++k) {
                if (j + 2 < mine)
                    lds_dma16(reinterpret_cast<const uint4*>(crow(k)) + tl * TV + c, bl + (uint32_t)(RPI * k * TV * 16));
                if (j >= LAG) st_nt(reinterpret_cast<uint4*>(prow(k)) + ts * TV + c, sv);
            }
            if (j + 2 < mine) issue_res(tl, j & 1);
        }
        pres = pnew;
    }
    if (LAG && mine > 0) {
#pragma unroll
        for (int k = 0; k < OPS; ++k) st_nt(reinterpret_cast<uint4*>(prow(k)) + tile_of(mine - 1) * TV + c, pres);
    }
}

// ---------------------------------------------------------------------------
// LO allreduce of P ranks in one pass: the butterfly itself.  Rank x keeps
// its own tree (for Swing the P results differ in bf16 rounding, exactly as
// the reference's per-core LO results do).  Lane (q, x) = q * P + x holds
// rank x's chunk; step k adds the value of lane q * P + partner_k(x),
// fetched with ds_bpermute, and rounds to bf16.  U consecutive chunks per
// lane keep each rank's 128-byte lines in flight together.
// ---------------------------------------------------------------------------
template <int P, int U>
__global__ __launch_bounds__(kBlock) void k_butterfly(uint16_t* __restrict__ ranks, uint64_t stride, uint64_t n_vec,
                                                      const int16_t* __restrict__ partner, int steps) {
    constexpr int Q = 64 / P;  // rank groups per wave
                               // U: chunks per lane per iteration (1 for small buckets: latency)
    const int lane = threadIdx.x & 63;
    const int x = lane % P;
    const int q = lane / P;
    int src[ALLRED_MAX_STEPS];
#pragma unroll
    for (int k = 0; k < ALLRED_MAX_STEPS; ++k) src[k] = k < steps ? (q * P + partner[k * P + x]) * 4 : lane * 4;
    uint4* row = reinterpret_cast<uint4*>(ranks + (uint64_t)x * stride);
    const uint64_t wave = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const uint64_t waves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t base = wave * (Q * U); base < n_vec; base += waves * (Q * U)) {
        uint4 val[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t v = base + (uint64_t)q * U + u;
            val[u] = v < n_vec ? row[v] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < ALLRED_MAX_STEPS; ++k) {
            if (k >= steps) break;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                uint4 o;
                o.x = (uint32_t)__builtin_amdgcn_ds_bpermute(src[k], (int)val[u].x);
                o.y = (uint32_t)__builtin_amdgcn_ds_bpermute(src[k], (int)val[u].y);
                o.z = (uint32_t)__builtin_amdgcn_ds_bpermute(src[k], (int)val[u].z);
                o.w = (uint32_t)__builtin_amdgcn_ds_bpermute(src[k], (int)val[u].w);
                val[u] = add8(val[u], o);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t v = base + (uint64_t)q * U + u;
            if (v < n_vec) row[v] = val[u];
        }
    }
}

// ---------------------------------------------------------------------------
// LO pass for 64 ranks staged through LDS: a tile of 256 elements of all 64
// ranks comes in with global_load_lds (1 KiB contiguous per wave-instruction),
// each lane x then holds rank x's columns (transposed LDS reads), runs the
// butterfly across lanes with ds_bpermute, writes back, and the rows leave
// with 1 KiB contiguous stores.  Row x's column c lives in 16-byte slot
// c ^ (x & 31) (swizzle applied on the global side, so global_load_lds's
// linear destination stays legal) — the 64 lanes' transposed reads of one
// column are then bank-conflict free.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_butterfly_lds64(uint16_t* __restrict__ ranks, uint64_t stride,
                                                            const int16_t* __restrict__ partner, int steps) {
    constexpr int TV = 32;
    __shared__ __attribute__((aligned(16))) uint4 tile[64 * TV];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int h = lane >> 5, l32 = lane & 31;
    const uint64_t v0 = (uint64_t)blockIdx.x * TV;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int r = 16 * w + 2 * k + h;
        const uint4* src = reinterpret_cast<const uint4*>(ranks + (uint64_t)r * stride) + v0 + (l32 ^ (r & 31));
        __builtin_amdgcn_global_load_lds((global_u32*)src, (lds_u32*)&tile[(16 * w + 2 * k) * TV], 16, 0, 2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // lane = rank x; wave w owns columns 8w .. 8w+7
    const int x = lane;
    uint4 val[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) val[j] = tile[x * TV + ((8 * w + j) ^ (x & 31))];
    for (int k = 0; k < steps; ++k) {
        const int src = (int)partner[k * 64 + x] * 4;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint4 o;
            o.x = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)val[j].x);
            o.y = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)val[j].y);
            o.z = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)val[j].z);
            o.w = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)val[j].w);
            val[j] = add8(val[j], o);
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[x * TV + ((8 * w + j) ^ (x & 31))] = val[j];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int r = 16 * w + 2 * k + h;
        st_nt(reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + v0 + (l32 ^ (r & 31)),
              tile[(16 * w + 2 * k + h) * TV + l32]);
    }
}

// ---------------------------------------------------------------------------
// k_butterfly_lds64 on a persistent grid with two LDS tiles: tile j+1's
// LDS-DMA loads are in flight while tile j runs its butterfly and leaves;
// the only vmcnt wait lets tile j-1's stores stay outstanding (see
// k_tree_lds_pipe).
// ---------------------------------------------------------------------------
// EX = 0: the butterfly in registers (ds_bpermute, 4 per 16-byte vector per
// step, one add per rank and step).  It is bound by its adds, not by the
// exchange: exchanging through the LDS tile, or by DPP / v_permlane16/32_swap
// on the XOR steps, ran as fast or slower; one add per partner pair 19.3 us
// (profiles/r01_lo_exchange_arms.txt; those arms were removed).
// EX = 4 (dag != nullptr, the default): each step adds only the DISTINCT sums.  Ranks whose
// step-k values come from the same pair of step-(k-1) values hold the same
// bits, so the host interns them (engine.cpp lo_dag): step k has d_k distinct
// nodes (Swing 8x8: 32, 16, 16, 16, 8, 4 — 92 adds per column instead of the
// butterfly's 384); its inputs are rows of step k-1 (the leaves at step 0).
// Lane group g = lane >> 3 takes the nodes in slots g, g + 8, g + 16, g + 24
// in column 8w + (lane & 7); the host chooses each node's slot and tile row
// so that every operand read (ds_read_b128, four 16-lane bank groups) is
// bank-conflict free (engine.cpp lo_dag_place; Swing 8x8: 92 extra LDS cycles
// per column group and tile with row = slot = first appearance, 0 placed).  A
// step issues all its reads before its writes, so overwriting rows of step
// k-1 is safe in wave order.  Rank r's result is row fin[r], stored to rank
// r's bucket.  dag: the lane-group form of allred_lo_dag's table
// (engine.cpp lo_dag_lanes).
template <int EX>   // 0 or 4
__global__ __launch_bounds__(kBlock) void k_butterfly_lds64_pipe(uint16_t* __restrict__ ranks, uint64_t stride,
                                                                 const int16_t* __restrict__ partner, int steps,
                                                                 uint64_t ntiles, const uint8_t* __restrict__ dag) {
    constexpr int TV = 32, OPS = 8;
    __shared__ __attribute__((aligned(16))) uint4 buf[2][64 * TV];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int h = lane >> 5, l32 = lane & 31;
    const int x = lane;
    const uint32_t wbase = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&buf[0][0] + (uint32_t)(16 * w * TV * 16));
    auto issue = [&](uint64_t t, int b) {
#pragma unroll
        for (int k = 0; k < OPS; ++k) {
            const int r = 16 * w + 2 * k + h;
            const uint4* src = reinterpret_cast<const uint4*>(ranks + (uint64_t)r * stride) + t * TV + (l32 ^ (r & 31));
            lds_dma16(src, wbase + (uint32_t)(b * 64 * TV * 16 + 2 * k * TV * 16));
        }
    };
    const uint64_t G = gridDim.x;
    const int mine = blockIdx.x < ntiles ? (int)((ntiles - 1 - blockIdx.x) / G + 1) : 0;
    // partner table first, then the first tile's loads (the other order
    // measured slower: 24.0-24.3 vs 23.6-23.9 us at 640 kB)
    int src_lane[ALLRED_MAX_STEPS];
#pragma unroll
    for (int k = 0; k < ALLRED_MAX_STEPS; ++k) src_lane[k] = k < steps ? (int)partner[k * 64 + x] * 4 : 0;
    // EX = 4: this lane's node of each step and item as a | b << 8 | dest << 16
    // (input rows, output row; -1: empty slot) and the final rows, from the
    // lane-group form of the table (engine.cpp lo_dag_lanes): six 16-byte loads
    int nab[ALLRED_MAX_STEPS][4], fin[OPS];
    if constexpr (EX == 4) {
        const uint4* tab = reinterpret_cast<const uint4*>(dag) + (lane >> 3) * 6;
#pragma unroll
        for (int k = 0; k < ALLRED_MAX_STEPS; ++k) {
            const uint4 t = tab[k];
            nab[k][0] = (int)t.x, nab[k][1] = (int)t.y, nab[k][2] = (int)t.z, nab[k][3] = (int)t.w;
        }
        const uint4 fv = reinterpret_cast<const uint4*>(dag + 768)[w];   // ranks 16w .. 16w+15
        const uint32_t fw[4] = {fv.x, fv.y, fv.z, fv.w};
#pragma unroll
        for (int k = 0; k < OPS; ++k) fin[k] = (int)(fw[k >> 1] >> (8 * (2 * (k & 1) + h))) & 255;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (mine > 0) issue(blockIdx.x, 0);
    for (int j = 0; j < mine; ++j) {
        wait_tile<OPS, 1>(j < 1 ? j : 1);
        lds_barrier();
        if (j + 1 < mine) issue(blockIdx.x + (uint64_t)(j + 1) * G, (j + 1) & 1);
        uint4* tile = buf[j & 1];
        const uint64_t v0 = (blockIdx.x + (uint64_t)j * G) * TV;
        if constexpr (EX == 0) {
            uint4 val[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) val[i] = tile[x * TV + ((8 * w + i) ^ (x & 31))];
#pragma unroll
            for (int k = 0; k < ALLRED_MAX_STEPS; ++k) {
                if (k >= steps) break;
                const int sl = src_lane[k];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    uint4 o;
                    o.x = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)val[i].x);
                    o.y = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)val[i].y);
                    o.z = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)val[i].z);
                    o.w = (uint32_t)__builtin_amdgcn_ds_bpermute(sl, (int)val[i].w);
                    val[i] = add8(val[i], o);
                }
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) tile[x * TV + ((8 * w + i) ^ (x & 31))] = val[i];  // own columns only
        } else {
            const int c = 8 * w + (lane & 7);
#pragma unroll
            for (int k = 0; k < ALLRED_MAX_STEPS; ++k) {
                if (k >= steps) break;
                uint4 A[4], B[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (nab[k][i] >= 0) {
                        const int a = nab[k][i] & 255, b = (nab[k][i] >> 8) & 255;
                        A[i] = tile[a * TV + (c ^ (a & 31))];
                        B[i] = tile[b * TV + (c ^ (b & 31))];
                    }
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (nab[k][i] >= 0) {
                        const int q = nab[k][i] >> 16;
                        tile[q * TV + (c ^ (q & 31))] = add8(A[i], B[i]);
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        lds_barrier();
#pragma unroll
        for (int k = 0; k < OPS; ++k) {
            const int r = 16 * w + 2 * k + h;
            const int fr = EX == 4 ? fin[k] : r;  // LDS row holding rank r's result
            st_nt(reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + v0 + (l32 ^ (fr & 31)), tile[fr * TV + l32]);
        }
    }
}

// ---------------------------------------------------------------------------
// k_lo_dag_reg<D>: fused LO of a Swing schedule whose ranks do not share one
// tree (Swing 8x8: the per-rank results take 4 distinct values per element),
// as the DAG of its distinct sums evaluated in REGISTERS.  D is the schedule's
// DAG generated at build time (csrc/gen_lo_dag.cpp -> build/lo_dag_gen.inc,
// engine.cpp lo_dag_build's interning): node P + i = RNE(v[a[i]] + v[b[i]]),
// the leaves are the P rank rows.  Thread t of the workgroup owns element t of
// the 256-element tile: it reads its P leaves out of the LDS tile (each wave
// reads 128 contiguous bytes per rank row), evaluates the N nodes with two
// VALU ops each (v_add_f32, v_cvt_pk_bf16_f32 with a zero low half: the
// rounded value stays an fp32 with zero low bits, ready for the next add),
// and writes the F distinct finals into F LDS rows.  Rank r's row then leaves
// from final row fin[r].  No LDS round trip or wave barrier between DAG steps
// (k_butterfly_lds64_pipe<4> writes and re-reads every node through LDS).
// The pipeline is k_tree_lds_lag's: two workgroups per CU, two tiles of LDS,
// tile j+2's LDS-DMA loads interleaved with tile j-1's stores.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float rne_bf16(float s) { return __uint_as_float(pack_rne(0.0f, s)); }

template <class D, int... I>
__device__ __forceinline__ void lo_dag_eval(float* v, std::integer_sequence<int, I...>) {
    ((v[D::P + I] = rne_bf16(v[D::a[I]] + v[D::b[I]])), ...);
}

template <class D>
__global__ __launch_bounds__(kBlock) void k_lo_dag_reg(uint16_t* __restrict__ ranks, uint64_t stride,
                                                       uint64_t t0, uint64_t ntiles) {
    constexpr int P = D::P, F = D::F, NW = 4, TV = 32, RPI = 2, RPW = P / NW, OPS = RPW / RPI;
    static_assert(OPS >= 1 && 3 * OPS <= 63, "vmcnt is 6 bits");
    static_assert(NW * 64 == 256 && TV * 8 == 256, "one element of the 256-element tile per thread");
    __shared__ __attribute__((aligned(16))) uint4 buf[2][P * TV];
    __shared__ __attribute__((aligned(16))) uint4 fin[2][F * TV];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane % TV, q = lane / TV;
    const uint32_t wbase = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&buf[0][0] + (uint32_t)(RPW * w * TV * 16));
    auto row = [&](int k) { return ranks + (uint64_t)(RPW * w + RPI * k + q) * stride; };
    // final row of each rank row this lane stores (rank RPW*w + RPI*k + q)
    int fsel[OPS];
#pragma unroll
    for (int k = 0; k < OPS; ++k) {
        int f = 0;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww)
#pragma unroll
            for (int qq = 0; qq < RPI; ++qq)
                if (w == ww && q == qq) f = D::fin[RPW * ww + RPI * k + qq];
        fsel[k] = f;
    }
    const uint64_t G = gridDim.x;
    const int mine = blockIdx.x < ntiles ? (int)((ntiles - 1 - blockIdx.x) / G + 1) : 0;
    auto tile_of = [&](int j) { return t0 + blockIdx.x + (uint64_t)j * G; };
    auto issue = [&](uint64_t t, int b) {
#pragma unroll
        for (int k = 0; k < OPS; ++k)
            lds_dma16(reinterpret_cast<const uint4*>(row(k)) + t * TV + c,
                      wbase + (uint32_t)(b * P * TV * 16 + RPI * k * TV * 16));
    };
    if (mine > 0) issue(tile_of(0), 0);
    if (mine > 1) issue(tile_of(1), 1);
    for (int j = 0; j < mine; ++j) {
        // after L(j): the last op of S(j-3) (interleaved with L(j)), L(j+1), S(j-2)
        wait_any((j >= 3 ? 1 : 0) + (j + 1 < mine ? OPS : 0) + (j >= 2 ? OPS : 0));
        lds_barrier();   // tile j is in LDS; fin[(j-1) & 1] is complete
        {
            const uint16_t* t16 = reinterpret_cast<const uint16_t*>(buf[j & 1]) + threadIdx.x;
            float v[P + D::N];
#pragma unroll
            for (int r = 0; r < P; ++r) v[r] = __uint_as_float((uint32_t)t16[r * 256] << 16);
            lo_dag_eval<D>(v, std::make_integer_sequence<int, D::N>{});
            uint16_t* f16 = reinterpret_cast<uint16_t*>(fin[j & 1]) + threadIdx.x;
#pragma unroll
            for (int f = 0; f < F; ++f) f16[f * 256] = (uint16_t)(__float_as_uint(v[D::fnode[f]]) >> 16);
        }
        lds_barrier();   // every wave has read tile j out of buf[j & 1]; fin[j & 1] is complete
        if (j >= 1 || j + 2 < mine) {   // tile j+2's loads and tile j-1's stores, interleaved op by op
            const uint64_t tl = tile_of(j + 2), ts = tile_of(j - 1);
            const uint32_t bl = wbase + (uint32_t)((j & 1) * P * TV * 16);
            const uint4* fp = fin[(j + 1) & 1];
            uint4 sv[OPS];
#pragma unroll
            for (int k = 0; k < OPS; ++k) sv[k] = fp[fsel[k] * TV + c];
#pragma unroll
            for (int k = 0; k < OPS; ++k) {
                if (j + 2 < mine)
                    lds_dma16(reinterpret_cast<const uint4*>(row(k)) + tl * TV + c, bl + (uint32_t)(RPI * k * TV * 16));
                if (j >= 1) st_nt(reinterpret_cast<uint4*>(row(k)) + ts * TV + c, sv[k]);
            }
        }
    }
    if (mine > 0) {
        const uint4* fp = fin[(mine - 1) & 1];
#pragma unroll
        for (int k = 0; k < OPS; ++k)
            st_nt(reinterpret_cast<uint4*>(row(k)) + tile_of(mine - 1) * TV + c, fp[fsel[k] * TV + c]);
    }
}

// ---------------------------------------------------------------------------
// mem_2D one-pass through LDS: tile of 256 elements of all P ranks (32 KiB at
// P = 64); thread t owns dword t of the tile row and accumulates the P copies
// in the reference order (owner's block first, then ranks 0..P-1) — in fp32,
// rounded once, or (ACC16) in bf16 rounded after every add — and the result
// row is stored to every rank (1 KiB per wave-instruction).  128 threads.
// ---------------------------------------------------------------------------
template <int P, bool ACC16 = false>
__global__ __launch_bounds__(128) void k_mem_lds(uint16_t* __restrict__ ranks, uint64_t stride, uint64_t block_vec,
                                                 uint16_t* __restrict__ out = nullptr) {   // out: reduce only (schedule form)
    constexpr int TV = 32;                      // 16-byte vectors per rank row
    constexpr int RPW = P / 2;                  // rank rows staged per wave
    __shared__ __attribute__((aligned(16))) uint4 tile[P * TV];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int h = lane >> 5, l32 = lane & 31;
    const uint64_t v0 = (uint64_t)blockIdx.x * TV;
#pragma unroll
    for (int k = 0; k < RPW / 2; ++k) {
        const int r = RPW * w + 2 * k + h;
        const uint4* src = reinterpret_cast<const uint4*>(ranks + (uint64_t)r * stride) + v0 + l32;
        __builtin_amdgcn_global_load_lds((global_u32*)src, (lds_u32*)&tile[(RPW * w + 2 * k) * TV], 16, 0, 2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int own = (int)(v0 / block_vec);
    uint32_t* t32 = reinterpret_cast<uint32_t*>(tile);
    const int d = threadIdx.x;                   // dword column 0..127
    uint32_t y = t32[own * TV * 4 + d];
    float a0 = lo_f(y), a1 = hi_f(y);
    t32[own * TV * 4 + d] = 0x80008000u;         // owner seeds the sum; -0.0 adds nothing (k_mem_lds_lag)
#pragma unroll
    for (int r = 0; r < P; ++r) {
        y = t32[r * TV * 4 + d];
        a0 = acc_add<ACC16>(a0, lo_f(y));
        a1 = acc_add<ACC16>(a1, hi_f(y));
    }
    if (out) {   // the schedule form's reduce: the block's sum goes to `out` (k_broadcast reads it back)
        reinterpret_cast<uint32_t*>(out + v0 * 8)[d] = pack_rne(a0, a1);
        return;
    }
    __syncthreads();
    reinterpret_cast<uint32_t*>(tile)[d] = pack_rne(a0, a1);
    __syncthreads();
    const uint4 res = tile[l32];
#pragma unroll 4
    for (int k = 0; k < RPW / 2; ++k) {
        const int r = RPW * w + 2 * k + h;
        st_nt(reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + v0 + l32, res);
    }
}

// ---------------------------------------------------------------------------
// k_mem_lds_lag: the fused mem_2D pass of k_mem_lds (same bits: per element
// owner first, then every other rank ascending, fp32 or ACC16) as a
// persistent double-buffered pipeline with the k_tree_lds_lag schedule, 64
// ranks: one thread per element of a 256-element tile, results through a
// small LDS row, each tile's 64 row stores one iteration late, behind tile
// j+2's loads.
// ---------------------------------------------------------------------------
template <bool ACC16 = false>
__global__ __launch_bounds__(kBlock) void k_mem_lds_lag(uint16_t* __restrict__ ranks, uint64_t stride,
                                                        uint64_t block_vec, uint64_t t0, uint64_t ntiles) {
    constexpr int P = 64, TV = 32, RPW = 16, OPS = 8;
    __shared__ __attribute__((aligned(16))) uint4 buf[2][P * TV];
    __shared__ __attribute__((aligned(16))) uint4 resb[2][TV];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane & 31, h = lane >> 5;
    const uint32_t wbase = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&buf[0][0] + (uint32_t)(RPW * w * TV * 16));
    auto issue = [&](uint64_t t, int b) {
#pragma unroll
        for (int k = 0; k < OPS; ++k) {
            const int r = RPW * w + 2 * k + h;
            const uint4* src = reinterpret_cast<const uint4*>(ranks + (uint64_t)r * stride) + t * TV + c;
            lds_dma16(src, wbase + (uint32_t)(b * P * TV * 16 + 2 * k * TV * 16));
        }
    };
    auto store = [&](uint64_t t, uint4 res) {
#pragma unroll
        for (int k = 0; k < OPS; ++k) {
            const int r = RPW * w + 2 * k + h;
            st_nt(reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + t * TV + c, res);
        }
    };
    const uint64_t G = gridDim.x;
    const int mine = blockIdx.x < ntiles ? (int)((ntiles - 1 - blockIdx.x) / G + 1) : 0;
    auto tile_of = [&](int j) { return t0 + blockIdx.x + (uint64_t)j * G; };
    if (mine > 0) issue(tile_of(0), 0);
    if (mine > 1) issue(tile_of(1), 1);
    uint4 prev = make_uint4(0, 0, 0, 0);
    const int e = threadIdx.x;   // element of the tile (0..255)
    for (int j = 0; j < mine; ++j) {
        // after L(j): the last op of S(j-3) (interleaved with L(j)), L(j+1), S(j-2)
        wait_any((j >= 3 ? 1 : 0) + (j + 1 < mine ? OPS : 0) + (j >= 2 ? OPS : 0));
        lds_barrier();
        const uint64_t t = tile_of(j);
        const int own = (int)(t * TV / block_vec);
        uint16_t* t16 = reinterpret_cast<uint16_t*>(buf[j & 1]);
        // the owner's element seeds the sum and is replaced by -0.0 (x + -0.0 == x
        // for every x, -0.0 included), so the 64-rank loop has no branch and its
        // LDS reads issue back to back (with `if (r == own) continue` every read
        // waited for the previous add: 16.0-16.5 us at 640 kB)
        float a = __uint_as_float((uint32_t)t16[own * TV * 8 + e] << 16);
        t16[own * TV * 8 + e] = 0x8000;
#pragma unroll
        for (int r = 0; r < P; ++r) a = acc_add<ACC16>(a, __uint_as_float((uint32_t)t16[r * TV * 8 + e] << 16));
        // one rounding (exact under ACC16); pairs of threads pack their two elements
        const float b = __shfl_xor(a, 1);
        if ((e & 1) == 0) reinterpret_cast<uint32_t*>(resb[j & 1])[e >> 1] = pack_rne(a, b);
        lds_barrier();   // the tile is read out of buf[j & 1]; resb[j & 1] is complete
        const uint4 res = resb[j & 1][c];
        {   // tile j+2's loads and tile j-1's stores interleaved op by op (as k_tree_lds_lag)
            const uint64_t tl = tile_of(j + 2), ts = tile_of(j - 1);
            const uint32_t bl = wbase + (uint32_t)((j & 1) * P * TV * 16);
#pragma unroll
            for (int k = 0; k < OPS; ++k) {
                const int r = RPW * w + 2 * k + h;
                if (j + 2 < mine)
                    lds_dma16(reinterpret_cast<const uint4*>(ranks + (uint64_t)r * stride) + tl * TV + c,
                              bl + (uint32_t)(2 * k * TV * 16));
                if (j >= 1) st_nt(reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + ts * TV + c, prev);
            }
        }
        prev = res;
    }
    if (mine > 0) store(tile_of(mine - 1), prev);
}


// ranks[r] = src for every r (all-gather of a reduced vector)
// grid.y picks a group of up to 8 ranks, so even a 640 kB vector fills the chip
__global__ __launch_bounds__(kBlock) void k_broadcast(uint16_t* __restrict__ ranks, uint64_t stride, int total,
                                                      const uint4* __restrict__ src, uint64_t n_vec) {
    const int r0 = blockIdx.y * 8;
    const int r1 = r0 + 8 < total ? r0 + 8 : total;
    for (uint64_t v = gtid(); v < n_vec; v += gthreads()) {
        const uint4 x = src[v];
        for (int r = r0; r < r1; ++r) st_nt(reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + v, x);
    }
}

// ---------------------------------------------------------------------------
// mem_2D: block b (owner rank b) summed over every rank's copy, starting
// from the owner's own block, then ranks 0..N-1 in order, in fp32 rounded once
// or (ACC16) in bf16 rounded after every add, the Tensix dest register with
// fp32_dest_acc_en = false (allred_mem_2D/kernels/compute_kernel.cpp:43-72
// with the own-block seed; allred_helper.cpp:331-335).  WRITE_ALL:
// store to every rank (fused one-shot form); else store to `out` (the shared
// dst buffer, allred_mem_2D dataflow :169-174).
// ---------------------------------------------------------------------------
template <bool WRITE_ALL, int B = 8, bool ACC16 = false>   // B ranks' loads in flight per thread before their adds
__global__ __launch_bounds__(kBlock) void k_mem(uint16_t* __restrict__ ranks, uint64_t stride, int total,
                                                uint64_t n_vec, uint64_t block_vec, uint16_t* __restrict__ out) {
    for (uint64_t v = gtid(); v < n_vec; v += gthreads()) {
        const int own = (int)(v / block_vec);
        const uint4 s = reinterpret_cast<const uint4*>(ranks + (uint64_t)own * stride)[v];
        float a[8] = {lo_f(s.x), hi_f(s.x), lo_f(s.y), hi_f(s.y), lo_f(s.z), hi_f(s.z), lo_f(s.w), hi_f(s.w)};
        // B ranks' loads in flight before their adds (in rank order: the sum's
        // order does not change); the owner's slot and ranks past `total`
        // contribute -0.0 (x + -0.0 == x for every x)
        for (int r0 = 0; r0 < total; r0 += B) {
            uint4 y[B];
#pragma unroll
            for (int i = 0; i < B; ++i) {
                const int r = r0 + i;
                y[i] = (r < total && r != own) ? reinterpret_cast<const uint4*>(ranks + (uint64_t)r * stride)[v]
                                               : make_uint4(0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u);
            }
#pragma unroll
            for (int i = 0; i < B; ++i) {
                const float v[8] = {lo_f(y[i].x), hi_f(y[i].x), lo_f(y[i].y), hi_f(y[i].y),
                                    lo_f(y[i].z), hi_f(y[i].z), lo_f(y[i].w), hi_f(y[i].w)};
#pragma unroll
                for (int e = 0; e < 8; ++e) a[e] = acc_add<ACC16>(a[e], v[e]);
            }
        }
        uint4 o;
        o.x = pack_rne(a[0], a[1]);
        o.y = pack_rne(a[2], a[3]);
        o.z = pack_rne(a[4], a[5]);
        o.w = pack_rne(a[6], a[7]);
        if (WRITE_ALL) {
            for (int r = 0; r < total; ++r) reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride)[v] = o;
        } else {
            reinterpret_cast<uint4*>(out)[v] = o;
        }
    }
}

// ---------------------------------------------------------------------------
// Schedule form (ALLRED_EXEC_STEPS): the reference's per-core step program,
// executed step by step:
//   BO  S reduce-scatter steps, then the S all-gather steps in reverse
//       (allred_BO_2D/kernels/dataflow_kernel.cpp:152-267, compute_kernel.cpp:35-67):
//       RS step k: rank r adds partner p_k(r)'s copy of every block b in
//       recv_k(r); AG step k: rank r copies p_k(r)'s blocks send_k(r).
//   LO  S full-vector exchange + add steps (shouldSendBlock with
//       bandwidth_optimal = 0, dataflow_kernel.cpp:19-29): r and p_k(r) both
//       become old_r + old_p (one fp32 add, commutative, one rounding).
// Step k of block b only touches block b's bytes (LO: column v only column
// v), so the program splits into independent units — (block, column slice)
// for BO, a column slice of the whole vector for LO — that run every step
// with one workgroup barrier per step: ONE persistent launch, no grid-wide
// synchronisation, no partner handshake across workgroups.  Between steps a
// unit's rank copies live in LDS, the Tensix L1 of the reference: loaded from
// the buckets once (DRAM -> L1, dataflow_kernel.cpp:126-130), every step
// reads the partner's copy and writes its own (the NoC write + add_tiles into
// the local CB), and each rank's result is written back once (L1 -> DRAM,
// :271-280).  BO keeps only the live copies: RS step 0 reads both operands
// from the buckets into the N/2 rows of its holders (their partners' copies
// are never read again), steps 1 .. 2S-2 run among those rows, and AG step 0
// writes its receivers' copies straight to their buckets, beside the
// holders' own results: 16 KiB of LDS per 512-byte unit, the whole of
// config 2 resident at once (64 rows: 32 KiB, one unit per CU could not
// start until another had finished: 30.4 us).  Measured forms that read the
// partner's copy back from the buckets instead (one launch 40.4 us, one
// launch per step 67.8 us; steps_form 1 keeps the latter): DESIGN.md §4.
//   tab (BO, per block, bytes): phase 0: (r, p) x N/2 ranks — holder r adds
//     partner p into LDS row i; phases 1 .. 2S-2: (row of r, row of p) x the
//     step's count; phase 2S-1: (r, row of p) x N/2 — receiver r's bucket
//     gets row p — then the N/2 holders' ranks (their rows' results).
//   pairs (LO): per step, N/2 (r, p) pairs with r < p, uint8.
//   stamps (optional, profiling): per unit, s_memrealtime (100 MHz) at its
//     start and at the end of every phase; the host derives each rank's
//     ALL_RED_LOOP zone (DeviceZoneScopedN, dataflow_kernel.cpp:147) from
//     them (allred_plan_rank_zones).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void stamp(uint64_t* stamps, uint64_t at) {
    if (stamps && threadIdx.x == 0) stamps[at] = __builtin_amdgcn_s_memrealtime();
}

// the unit's N rows (rank r's columns [v0, v0 + width)) bucket <-> LDS rows of SV vectors
template <bool LOAD, int SV, int T>
__device__ __forceinline__ void unit_rows(uint16_t* __restrict__ ranks, uint64_t stride, int N, uint64_t v0, int width,
                                          uint4* tile) {
    const int items = N * width;
    for (int i0 = threadIdx.x; i0 < items; i0 += 8 * T) {
        uint4 x[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int i = i0 + t * T;
            if (i < items) {
                const int r = i / width, v = i - r * width;
                uint4* g = reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + v0 + v;
                if (LOAD) x[t] = ld_nt(g);
                else st_nt(g, tile[r * SV + v]);
            }
        }
        if (LOAD) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int i = i0 + t * T;
                if (i < items) {
                    const int r = i / width, v = i - r * width;
                    tile[r * SV + v] = x[t];
                }
            }
        }
    }
}

constexpr int kStepSV = 32;   // BO unit row: 32 x 16 B = 512 B, the fused passes' tile width

__global__ __launch_bounds__(kBlock) void k_bo_steps(uint16_t* __restrict__ ranks, uint64_t stride,
                                                     const uint8_t* __restrict__ tab, int N, int S, uint64_t bv,
                                                     uint64_t slices, uint64_t units, uint64_t* __restrict__ stamps) {
    constexpr int SV = kStepSV, T = kBlock;
    __shared__ __attribute__((aligned(16))) uint4 tile[ALLRED_MAX_NODES / 2 * SV];
    const int H = N / 2;
    const int L = 2 * 2 * (N - 1) + H;   // tab bytes per block
    const int P = 2 * S + 1;             // stamps per unit
    auto grow = [&](int r) { return reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride); };
    for (uint64_t u = blockIdx.x; u < units; u += gridDim.x) {
        const uint64_t b = u / slices, j = u % slices;
        const uint64_t v0 = b * bv + j * SV;
        const int width = (int)(bv - j * SV < (uint64_t)SV ? bv - j * SV : (uint64_t)SV);
        const uint8_t* tb = tab + b * (uint64_t)L;
        stamp(stamps, u * P);
        // RS step 0: holder r (row i) = r's copy + partner's copy, both from the buckets
        for (int i0 = threadIdx.x; i0 < H * width; i0 += 4 * T) {
            uint4 x[4], y[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int i = i0 + t * T;
                if (i < H * width) {
                    const int row = i / width, v = i - row * width;
                    x[t] = ld_nt(grow(tb[2 * row]) + v0 + v);
                    y[t] = ld_nt(grow(tb[2 * row + 1]) + v0 + v);
                }
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int i = i0 + t * T;
                if (i < H * width) {
                    const int row = i / width, v = i - row * width;
                    tile[row * SV + v] = add8(x[t], y[t]);
                }
            }
        }
        __syncthreads();
        stamp(stamps, u * P + 1);
        // RS steps 1 .. S-1 and AG steps S-1 .. 1 among the holder rows.  A step's
        // writers never read each other's rows (its pairs are disjoint), so
        // reading and writing row by row within the step is safe.
        const uint8_t* e = tb + 2 * H;
        for (int q = 1; q < 2 * S - 1; ++q) {
            const bool rs = q < S;
            const int k = rs ? q : 2 * S - 1 - q;
            const int cnt = N >> (k + 1);
            for (int i = threadIdx.x; i < cnt * width; i += T) {
                const int x = i / width, v = i - x * width;
                const int a = e[2 * x] * SV + v, c = e[2 * x + 1] * SV + v;
                tile[a] = rs ? add8(tile[a], tile[c]) : tile[c];
            }
            e += 2 * cnt;
            lds_barrier();
            stamp(stamps, u * P + 1 + q);
        }
        // AG step 0: receivers' buckets get their partners' rows; the holders' results leave too
        const uint8_t* fin = e + 2 * H;   // the holders' ranks, row order
        for (int i = threadIdx.x; i < 2 * H * width; i += T) {
            const int x = i / width, v = i - x * width;
            if (x < H) st_nt(grow(e[2 * x]) + v0 + v, tile[e[2 * x + 1] * SV + v]);
            else st_nt(grow(fin[x - H]) + v0 + v, tile[(x - H) * SV + v]);
        }
        __syncthreads();   // the rows are read out before the next unit overwrites them
        stamp(stamps, u * P + 2 * S);
    }
}

// LO: after step k the two ranks of every step-k pair hold the same value
// (old_r + old_p: one add, commutative), so a unit keeps one LDS row per pair
// — N/2 rows, 16 KiB at 512-byte rows: every unit of a 640 kB bucket resident
// at once (one row per rank, 32 KiB, left one unit per CU waiting: 28.6 us).
// Step 0 adds the pair's two bucket rows into row i; step k (1 .. S-2) reads
// the rows of its pairs' step-(k-1) pairs into registers, barrier, writes its
// own rows; the last step stores each pair's sum straight to both buckets.
//   pairs: per step, N/2 (r, p) ranks, r < p; then per step >= 1 the N/2
//   (row of r, row of p) in the previous step's rows.
__global__ __launch_bounds__(kBlock) void k_lo_steps(uint16_t* __restrict__ ranks, uint64_t stride,
                                                     const uint8_t* __restrict__ pairs, int N, int S, uint64_t n_vec,
                                                     uint64_t units, uint64_t* __restrict__ stamps) {
    constexpr int SV = kStepSV, T = kBlock, IPT = ALLRED_MAX_NODES / 2 * SV / T;
    __shared__ __attribute__((aligned(16))) uint4 tile[ALLRED_MAX_NODES / 2 * SV];
    const int H = N / 2;
    const uint8_t* rows = pairs + 2 * H * S;   // [step >= 1][H] (row of r, row of p)
    auto grow = [&](int r) { return reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride); };
    for (uint64_t u = blockIdx.x; u < units; u += gridDim.x) {
        const uint64_t v0 = u * SV;
        const int width = (int)(n_vec - v0 < (uint64_t)SV ? n_vec - v0 : (uint64_t)SV);
        const int items = H * width;
        stamp(stamps, u * (S + 1));
        for (int k = 0; k < S; ++k) {
            const uint8_t* pk = pairs + 2 * H * k;
            const uint8_t* rk = rows + 2 * H * (k - 1);
            uint4 val[IPT];
#pragma unroll
            for (int t = 0; t < IPT; ++t) {
                const int i = threadIdx.x + t * T;
                if (i < items) {
                    const int x = i / width, v = i - x * width;
                    if (k == 0) val[t] = add8(ld_nt(grow(pk[2 * x]) + v0 + v), ld_nt(grow(pk[2 * x + 1]) + v0 + v));
                    else val[t] = add8(tile[rk[2 * x] * SV + v], tile[rk[2 * x + 1] * SV + v]);
                }
            }
            if (k > 0) lds_barrier();   // every read of the step-(k-1) rows is done
#pragma unroll
            for (int t = 0; t < IPT; ++t) {
                const int i = threadIdx.x + t * T;
                if (i < items) {
                    const int x = i / width, v = i - x * width;
                    if (k == S - 1) {   // the last step's sums leave for both ranks' buckets
                        st_nt(grow(pk[2 * x]) + v0 + v, val[t]);
                        st_nt(grow(pk[2 * x + 1]) + v0 + v, val[t]);
                    } else {
                        tile[x * SV + v] = val[t];
                    }
                }
            }
            if (k == S - 1) __syncthreads();   // (the rows are free for the next unit)
            else lds_barrier();
            stamp(stamps, u * (S + 1) + 1 + k);
        }
    }
}

// The schedule form's programs (engine.cpp), read by k_steps_reg:
//   BO (bo_steps_pipe_table, 256 bytes per block): (r, p) x P/2 of RS step 0 ->
//     row i; (row a, row c) pairs of RS 1..S-1 and AG S-1..1 (RS: a += c, AG:
//     a = c); then P bytes: the row holding rank r's result after AG step 0
//     (holders: their own row, receivers: their step-0 partner's).
//   LO (lo_steps_pipe_table): per step P/2 (r, p) ranks (step 0) / (row of r,
//     row of p) (steps >= 1) -> row i = pair i; then P bytes: rank r's pair at
//     the last step.
// S = log2(P) (every 2D and 1D schedule of P ranks), so the step loops unroll.
// ---------------------------------------------------------------------------
constexpr int kBoPipeTab = kBoPipeTabBytes;

template <int P>
constexpr int log2_of() { return P <= 1 ? 0 : 1 + log2_of<P / 2>(); }

// k_steps_reg<P, BO, MINW>: the schedule form (every RS / AG step of BO, every
// exchange step of LO, in order, one persistent launch).  A wave's work item
// is a STRIP: 8 columns (128 bytes) of one 512-byte unit in all P rank rows.
// Step 0 happens in registers as the rows arrive: lane (pair u, column) loads
// both ranks of its step-0 pairs straight into VGPRs and adds them; only the
// H pair rows go to LDS (4 KiB per wave), where the later phases run as the
// tables' row moves (RS a += c, AG a = c; LO: pair x = row x, kept in a
// register, + its other operand); then the result rows are read out and
// stored.  One register set per lane: strip j+1's loads go out right after
// strip j's step 0 (its registers are free then) and land behind strip j's
// step chain (99 VGPRs at 64 ranks, four waves per SIMD).  No barrier after
// the programs are staged.  The round-2 form (k_steps_pipe) staged a whole
// unit's rank rows in LDS by LDS-DMA and ran the step program there: the step
// chain (ten dependent LDS phases for BO, ≈2.4 us per strip) then held the
// unit's buffer, so a CU had only about ten strips in flight (17.4 / 18.3 us
// BO / LO at config 2, no better with every wave its own LDS pipeline or
// deeper LDS prefetch: profiles/r03_steps_wave_ab.txt; both removed).
//   BO: the step-0 pairs are the same for every block, only which rank holds
//   (keeps the sum, adds first) and the holder's row differ: tab =
//   bo_steps_reg_table (engine.cpp), per block 256 bytes — byte u = row of
//   pair u | 0x80 when its higher rank holds, then the pipe table's phases and
//   result rows — in LDS for the workgroup; pairs: H x (lower rank, higher rank).
//   LO: there are no blocks; tab = lo_steps_pipe_table (its step-0 (r, p) give
//   the loads), in LDS; pairs unused.
// MINW: waves per SIMD the compiler must allow = workgroups per CU (3, 4, 5).
template <int P, bool BO, int MINW>
__global__ __launch_bounds__(256, MINW) void k_steps_reg(uint16_t* __restrict__ ranks, uint64_t stride,
                                                         const uint8_t* __restrict__ tab,
                                                         const uint8_t* __restrict__ pairs, uint64_t bv,
                                                         uint64_t slices, uint64_t units, uint64_t* __restrict__ stamps,
                                                         int flags) {
    constexpr int NW = 4, TV = 32, CW = 8, Q = TV / CW, RPO = 64 / CW, OPS = P / RPO, H = P / 2, S = log2_of<P>();
    constexpr int IPW = (H * CW + 63) / 64;   // step-0 items (pair, column) per lane
    constexpr int NPH = BO ? 2 * S - 2 : S - 1;
    constexpr int STAMPS = BO ? 2 * S + 1 : S + 1;
    constexpr int MPH = BO ? (P / 4 * CW + 63) / 64 : IPW;
    // the program(s) in LDS: BO every block's (P x 256 bytes), LO the one step program (2H S + P <= 448 bytes)
    constexpr int LOTAB = 2 * H * S + P;
    __shared__ __attribute__((aligned(16))) uint8_t tabs[BO ? P : 1][BO ? kBoPipeTab : (LOTAB + 15) / 16 * 16];
    __shared__ __attribute__((aligned(16))) uint4 work[NW][H * CW];   // per wave: the strip's pair rows
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int cl = lane % CW, rl = lane / CW;
    auto cnt_of = [](int ph) {
        if (!BO) return H;
        const int k = ph < S ? ph : 2 * S - 1 - ph;
        return P >> (k + 1);
    };
    auto off_of = [&](int ph) {
        int o = 2 * H;
        for (int x = 1; x < ph; ++x) o += 2 * cnt_of(x);
        return o;
    };
    uint32_t pra[IPW], prb[IPW];   // this lane's step-0 pairs: first / second rank
    if constexpr (!BO)   // LO: the one step program (<= 448 bytes) staged first, as in round 3
        for (int i = threadIdx.x; i < LOTAB; i += NW * 64) tabs[0][i] = tab[i];
    if constexpr (BO) {
#pragma unroll
        for (int t = 0; t < IPW; ++t) {
            const int i = lane + 64 * t, u = i < H * CW ? i / CW : 0;
            pra[t] = pairs[2 * u];
            prb[t] = pairs[2 * u + 1];
        }
    } else {
        const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tab);
#pragma unroll
        for (int t = 0; t < IPW; ++t) {
            const int i = lane + 64 * t;
            const uint32_t e = i < H * CW ? t16[i / CW] : 0;
            pra[t] = e & 255;
            prb[t] = e >> 8;
        }
    }
    const uint64_t GW = (uint64_t)gridDim.x * NW, gw = (uint64_t)blockIdx.x * NW + w, strips = units * Q;
    const int mine = gw < strips ? (int)((strips - 1 - gw) / GW + 1) : 0;
    auto strip_of = [&](int j) { return gw + (uint64_t)j * GW; };
    auto col0 = [&](uint64_t s) {
        const uint64_t u = s / Q;
        return (BO ? (u / slices) * bv + (u % slices) * TV : u * TV) + (s % Q) * CW;
    };
    auto grow = [&](uint32_t r) { return reinterpret_cast<const uint4*>(ranks + (uint64_t)r * stride); };
    auto load = [&](int j, uint4 (&A)[IPW], uint4 (&B)[IPW]) {   // both ranks of every pair item of strip j
        const uint64_t c0 = col0(strip_of(j)) + cl;
#pragma unroll
        for (int t = 0; t < IPW; ++t)
            if (lane + 64 * t < H * CW) {
                A[t] = ld_nt(grow(pra[t]) + c0);
                B[t] = ld_nt(grow(prb[t]) + c0);
            }
    };
    uint4 A[IPW], B[IPW];
    // flags bit 1 (tune steps_early): the first strip's loads go out before the programs are staged
    const bool early = (flags & 2) != 0;
    if (early && mine > 0) load(0, A, B);
    // BO flags bit 0 (tune steps_tab): the workgroup's units are blockIdx + j * grid (its four waves
    // take the unit's four strips), so only their J blocks' programs are staged, tabs[j] for unit j,
    // when J < P (config 2: 1-2 programs, 256-512 bytes, instead of all P blocks' 16 KiB)
    const int J = blockIdx.x < units ? (int)((units - 1 - blockIdx.x) / gridDim.x + 1) : 0;
    const bool perj = BO && (flags & 1) && J < P;
    if constexpr (BO) {
        if (perj) {
            for (int i = threadIdx.x; i < J * (kBoPipeTab / 16); i += NW * 64) {
                const int jj = i / (kBoPipeTab / 16), k = i % (kBoPipeTab / 16);
                const uint64_t blk = (blockIdx.x + (uint64_t)jj * gridDim.x) / slices;
                reinterpret_cast<uint4*>(&tabs[jj][0])[k] = reinterpret_cast<const uint4*>(tab + blk * kBoPipeTab)[k];
            }
        } else {
            for (int i = threadIdx.x; i < P * kBoPipeTab / 16; i += NW * 64)
                reinterpret_cast<uint4*>(&tabs[0][0])[i] = reinterpret_cast<const uint4*>(tab)[i];
        }
    }
    __syncthreads();   // the program(s) in LDS (the only barrier)
    uint4* tile = work[w];
    // strip j: step 0 from A / B (registers), then strip j+1's loads into the same registers (free once
    // step 0 has written the pair rows), the later phases among the pair rows, result rows stored
    auto body = [&](int j) {
        const uint64_t s = strip_of(j);
        const bool st_on = stamps && s % Q == 0 && lane == 0;
        if (st_on) stamps[(s / Q) * STAMPS] = __builtin_amdgcn_s_memrealtime();
        const uint8_t* tb = tabs[BO ? (perj ? j : (s / Q) / slices) : 0];
        const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tb);
        uint4 val[BO ? 1 : IPW];   // LO: this lane's pair rows after the latest step
#pragma unroll
        for (int t = 0; t < IPW; ++t)
            if (lane + 64 * t < H * CW) {
                if constexpr (BO) {
                    const uint32_t e = tb[(lane + 64 * t) / CW];   // row | 0x80: the higher rank holds
                    tile[(e & 127) * CW + cl] = (e & 128) ? add8(B[t], A[t]) : add8(A[t], B[t]);
                } else {
                    val[t] = add8(A[t], B[t]);
                    tile[((lane + 64 * t) / CW) * CW + cl] = val[t];
                }
            }
        if (st_on) stamps[(s / Q) * STAMPS + 1] = __builtin_amdgcn_s_memrealtime();
        if (j + 1 < mine) load(j + 1, A, B);   // in flight behind this strip's step chain and stores
#pragma unroll
        for (int ph = 1; ph <= NPH; ++ph) {
            if constexpr (BO) {   // RS 1 .. S-1 (a += c), AG S-1 .. 1 (a = c); a step's pairs are disjoint
                const bool rs = ph < S;
#pragma unroll
                for (int m = 0; m < MPH; ++m)
                    if (lane + 64 * m < cnt_of(ph) * CW) {
                        const uint32_t pr = t16[off_of(ph) / 2 + (lane + 64 * m) / CW];
                        const int a = (pr & 255) * CW + cl, cc = (pr >> 8) * CW + cl;
                        tile[a] = rs ? add8(tile[a], tile[cc]) : tile[cc];
                    }
            } else {   // exchange step ph: pair x = row x (kept in val) + the row of its other rank
                uint4 oth[IPW];
#pragma unroll
                for (int m = 0; m < IPW; ++m)
                    if (lane + 64 * m < H * CW) oth[m] = tile[(t16[off_of(ph) / 2 + (lane + 64 * m) / CW] >> 8) * CW + cl];
#pragma unroll
                for (int m = 0; m < IPW; ++m)
                    if (lane + 64 * m < H * CW) {
                        val[m] = add8(val[m], oth[m]);
                        tile[((lane + 64 * m) / CW) * CW + cl] = val[m];
                    }
            }
            if (st_on) stamps[(s / Q) * STAMPS + 1 + ph] = __builtin_amdgcn_s_memrealtime();
        }
        const uint64_t cs = col0(s) + cl;
#pragma unroll
        for (int k = 0; k < OPS; ++k) {   // rank RPO k + rl's value is row fin
            st_nt(reinterpret_cast<uint4*>(ranks + (uint64_t)(RPO * k + rl) * stride) + cs,
                  tile[(int)tb[off_of(NPH + 1) + RPO * k + rl] * CW + cl]);
        }
        if (BO && st_on) stamps[(s / Q) * STAMPS + 2 * S] = __builtin_amdgcn_s_memrealtime();
    };
    if (!early && mine > 0) load(0, A, B);
    for (int j = 0; j < mine; ++j) body(j);
}

// One launch per step (allred_tune_set("steps_form", 1), the round-1 form, A/B):
// one wave per (rank, block), U vectors' loads in flight per lane.
//   RS: ranks[r][b] += ranks[p][b] for b in recv_mask_k(r)   (in place: the
//       pair's recv masks are disjoint, so nobody reads what another writes)
//   AG: ranks[r][b]  = ranks[p][b] for b in send_mask_k(r) (= recv_mask_k(p))
template <bool ADD, int U>
__global__ __launch_bounds__(64) void k_step_w(uint16_t* __restrict__ ranks, uint64_t stride,
                                               const int16_t* __restrict__ partner,
                                               const int16_t* __restrict__ blocks, int blocks_per_rank,
                                               uint64_t block_vec) {
    const int t = blockIdx.x;
    const int r = t / blocks_per_rank;
    const int p = partner[r];
    const uint64_t off = (uint64_t)blocks[t] * block_vec;
    uint4* L = reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + off;
    const uint4* R = reinterpret_cast<const uint4*>(ranks + (uint64_t)p * stride) + off;
    for (uint64_t v0 = threadIdx.x; v0 < block_vec; v0 += 64 * U) {
        uint4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t v = v0 + 64 * u;
            if (v < block_vec) {
                b[u] = ld_nt(R + v);
                if (ADD) a[u] = ld_nt(L + v);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t v = v0 + 64 * u;
            if (v < block_vec) st_nt(L + v, ADD ? add8(a[u], b[u]) : b[u]);
        }
    }
}

// LO step of the per-step form (full vector): dst[r] = src[r] + src[p(r)], ping-pong buffers
__global__ __launch_bounds__(kBlock) void k_lo_step(const uint16_t* __restrict__ src, uint64_t src_stride,
                                                    uint16_t* __restrict__ dst, uint64_t dst_stride,
                                                    const int16_t* __restrict__ partner, uint64_t n_vec) {
    const int r = blockIdx.y;
    const int p = partner[r];
    const uint4* A = reinterpret_cast<const uint4*>(src + (uint64_t)r * src_stride);
    const uint4* B = reinterpret_cast<const uint4*>(src + (uint64_t)p * src_stride);
    uint4* D = reinterpret_cast<uint4*>(dst + (uint64_t)r * dst_stride);
    for (uint64_t v = gtid(); v < n_vec; v += gthreads()) st_nt(D + v, add8(ld_nt(A + v), ld_nt(B + v)));
}

__global__ __launch_bounds__(kBlock) void k_copy_ranks(const uint16_t* __restrict__ src, uint64_t src_stride,
                                                       uint16_t* __restrict__ dst, uint64_t dst_stride,
                                                       uint64_t n_vec) {
    const uint4* A = reinterpret_cast<const uint4*>(src + (uint64_t)blockIdx.y * src_stride);
    uint4* D = reinterpret_cast<uint4*>(dst + (uint64_t)blockIdx.y * dst_stride);
    for (uint64_t v = gtid(); v < n_vec; v += gthreads()) st_nt(D + v, ld_nt(A + v));
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
int last_error() { return hip_status((int)hipGetLastError()); }

// fused_form (tune.cpp): 0 auto, 1 register tree, 2 one tile per workgroup, 3 persistent
inline int64_t fused_form() { return tune(Tune::fused_form); }

template <bool WRITE_ALL>
int tree_dispatch(uint16_t* ranks, uint64_t stride, uint64_t n_vec, int total, const uint8_t* order,
                  uint64_t block_vec, uint16_t* out, hipStream_t st) {
    const int64_t form = fused_form();
    // hierarchical partial of 64 ranks, >= 1024 tiles: the persistent
    // double-buffered form (2 workgroups per CU), as the fused pass.  (The
    // early-release / two-tiles-ahead forms measured slower on this read-only
    // stream: 10.4 / 9.9 vs 9.6 us, profiles/r01_partial_ab.txt.)
    if (!WRITE_ALL && total == 64 && n_vec % 32 == 0 && block_vec == 0 && form != 1 && form != 2 &&
        (n_vec / 32 >= 1024 || form == 3)) {
        const uint64_t tiles = n_vec / 32;
        hipLaunchKernelGGL((k_tree_lds_pipe<64, false>), dim3((unsigned)(tiles < 512 ? tiles : 512)), dim3(kBlock), 0,
                           st, ranks, stride, order, (uint64_t)0, tiles, out);
        return last_error();
    }
    // LDS-staged form: whole 32-vector tiles inside one block (any tile when block_vec == 0)
    if (total >= 8 && n_vec % 32 == 0 && (block_vec == 0 || block_vec % 32 == 0) && (block_vec || !WRITE_ALL) &&
        form != 1) {
        const dim3 grid((unsigned)(n_vec / 32)), blk(kBlock);
        switch (total) {
            case 8: hipLaunchKernelGGL((k_tree_lds<8, WRITE_ALL>), grid, blk, 0, st, ranks, stride, order, block_vec, out); break;
            case 16: hipLaunchKernelGGL((k_tree_lds<16, WRITE_ALL>), grid, blk, 0, st, ranks, stride, order, block_vec, out); break;
            case 32: hipLaunchKernelGGL((k_tree_lds<32, WRITE_ALL>), grid, blk, 0, st, ranks, stride, order, block_vec, out); break;
            case 64: hipLaunchKernelGGL((k_tree_lds<64, WRITE_ALL>), grid, blk, 0, st, ranks, stride, order, block_vec, out); break;
            default: return ALLRED_ERR_UNSUPPORTED;
        }
        return last_error();
    }
    const int lanes = total >= 8 ? total / 8 : 1;
    const uint64_t chunk_groups = (n_vec + (64 / lanes) - 1) / (64 / lanes);  // one per wave
    uint64_t blocks = (chunk_groups + 3) / 4;
    if (blocks < 1) blocks = 1;
    if (blocks > 256 * 16) blocks = 256 * 16;
    const dim3 grid((unsigned)blocks), blk(kBlock);
    switch (total) {
        case 1: hipLaunchKernelGGL((k_tree<1, WRITE_ALL>), grid, blk, 0, st, ranks, stride, n_vec, order, block_vec, out); break;
        case 2: hipLaunchKernelGGL((k_tree<2, WRITE_ALL>), grid, blk, 0, st, ranks, stride, n_vec, order, block_vec, out); break;
        case 4: hipLaunchKernelGGL((k_tree<4, WRITE_ALL>), grid, blk, 0, st, ranks, stride, n_vec, order, block_vec, out); break;
        case 8: hipLaunchKernelGGL((k_tree<8, WRITE_ALL>), grid, blk, 0, st, ranks, stride, n_vec, order, block_vec, out); break;
        case 16: hipLaunchKernelGGL((k_tree<16, WRITE_ALL>), grid, blk, 0, st, ranks, stride, n_vec, order, block_vec, out); break;
        case 32: hipLaunchKernelGGL((k_tree<32, WRITE_ALL>), grid, blk, 0, st, ranks, stride, n_vec, order, block_vec, out); break;
        case 64: hipLaunchKernelGGL((k_tree<64, WRITE_ALL>), grid, blk, 0, st, ranks, stride, n_vec, order, block_vec, out); break;
        default: return ALLRED_ERR_UNSUPPORTED;
    }
    return last_error();
}

unsigned persistent_grid(uint64_t tiles, uint64_t dflt) {
    const int64_t g = tune(Tune::pipe_grid);
    const uint64_t cap = g > 0 ? (uint64_t)g : dflt;
    return (unsigned)(tiles < cap ? tiles : cap);
}

// the schedule form with register-staged strips (k_steps_reg): 8..64 ranks; false if the shape has no instance.
// per_cu: four-wave workgroups per CU (3, 4 or 5; 5 x 32 KiB of LDS at 64 ranks fills the CU's 160 KiB)
bool launch_steps_reg(bool bo, int per_cu, uint16_t* ranks, uint64_t stride, int total, const uint8_t* tab,
                      const uint8_t* pairs, uint64_t bv, uint64_t slices, uint64_t units, uint64_t* stamps,
                      hipStream_t st) {
    const dim3 grid(persistent_grid(units, 256 * (uint64_t)per_cu));
    // early first-strip loads (tune steps_early: 0 never, 1 auto, 2 always): auto when the grid is full
    // (units >= its workgroups), where they win 0.8 us at config 2; with fewer units every wave has
    // one strip and the program staging behind that burst costs 0.3-0.8 us (profiles/r04_steps_small_ab.txt)
    const int64_t early = tune(Tune::steps_early);
    const bool early_on = early == 2 || (early == 1 && units >= 256 * (uint64_t)per_cu);
    const int flags = (tune(Tune::steps_tab) ? 1 : 0) | (early_on ? 2 : 0);
#define TSA_SR(PP, BOV, MW) do { \
        hipLaunchKernelGGL((k_steps_reg<PP, BOV, MW>), grid, dim3(256), 0, st, ranks, stride, tab, pairs, bv, slices, \
                           units, stamps, flags); \
        note_launch(reinterpret_cast<const void*>(&k_steps_reg<PP, BOV, MW>), "k_steps_reg<" #PP ", " #BOV ", " #MW ">", \
                    grid.x, 256); \
    } while (0)
#define TSA_SRB(PP, BOV) do { if (per_cu >= 5) TSA_SR(PP, BOV, 5); else if (per_cu == 4) TSA_SR(PP, BOV, 4); \
                              else TSA_SR(PP, BOV, 3); } while (0)
#define TSA_SRP(PP) do { if (bo) TSA_SRB(PP, true); else TSA_SRB(PP, false); } while (0)
    switch (total) {
        case 8: TSA_SRP(8); return true;
        case 16: TSA_SRP(16); return true;
        case 32: TSA_SRP(32); return true;
        case 64: TSA_SRP(64); return true;
        default: return false;
    }
#undef TSA_SRP
#undef TSA_SRB
#undef TSA_SR
}

}  // namespace

int hip_status(int e) { return e == (int)hipSuccess ? ALLRED_OK : ALLRED_ERR_HIP; }

int launch_bf16_add(uint16_t* dst, const uint16_t* src, size_t n, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (n == 0) return ALLRED_OK;
    if (!dst || !src) return ALLRED_ERR_ARG;
    if (aligned16(dst) && aligned16(src)) {
        const uint64_t nv = n / 8;
        if (nv) hipLaunchKernelGGL(k_add, dim3(grid_all(nv)), dim3(kBlock), 0, st,
                                   reinterpret_cast<uint4*>(dst), reinterpret_cast<const uint4*>(src), nv);
        const uint64_t tail = n - nv * 8;
        if (tail) hipLaunchKernelGGL(k_add_scalar, dim3(1), dim3(64), 0, st, dst + nv * 8, src + nv * 8, tail);
    } else {
        hipLaunchKernelGGL(k_add_scalar, dim3(grid_for(n)), dim3(kBlock), 0, st, dst, src, (uint64_t)n);
    }
    return last_error();
}

int launch_bf16_add_segs(uint16_t* dst, const uint16_t* src, const uint64_t* off, const uint64_t* len, int nsegs,
                         void* stream) {
    if (nsegs <= 0) return ALLRED_OK;
    if (nsegs > kMaxAddSegs || !aligned16(dst) || !aligned16(src)) return ALLRED_ERR_ARG;
    SegList segs{};
    uint64_t longest = 0;
    for (int i = 0; i < nsegs; ++i) {
        if (off[i] % 8 || len[i] % 8) return ALLRED_ERR_ARG;
        segs.off[i] = off[i] / 8;
        segs.len[i] = len[i] / 8;
        if (segs.len[i] > longest) longest = segs.len[i];
    }
    if (!longest) return ALLRED_OK;
    hipLaunchKernelGGL(k_add_segs, dim3(grid_all(longest), nsegs), dim3(kBlock), 0, (hipStream_t)stream,
                       reinterpret_cast<uint4*>(dst), reinterpret_cast<const uint4*>(src), segs);
    return last_error();
}

uint64_t fused_chunk_launches(uint64_t tiles) {
    const uint64_t chunk = (uint64_t)tune(Tune::fused_chunk_tiles);
    const uint64_t nl = chunk ? (tiles + chunk / 2) / chunk : 1;
    return nl < 1 ? 1 : nl;
}

// Kernel launches one fused execute of device-resident buckets enqueues: the
// same decisions launch_tree_fused (BO, rank-uniform LO), launch_lo_dag_reg /
// launch_butterfly (other LO) and mem_fused_impl (MEM) take, with the tune
// keys as they are now (allred_plan_launches asks at call time).
uint64_t fused_launches(int variant, bool lo_tree, int algo, int side, size_t n, int total) {
    const uint64_t nv = n / 8, tiles = nv / 32, bv = total > 0 ? nv / total : 0;
    const bool big64 = total == 64 && nv % 32 == 0 && bv % 32 == 0 && tiles >= 1024;
    if (variant == ALLRED_MEM) return big64 && fused_form() == 0 ? fused_chunk_launches(tiles) : 1;
    if (variant == ALLRED_LO && !lo_tree) {
        if (!tune(Tune::lo_dag_reg) || n % 256 || tiles < (uint64_t)tune(Tune::lo_dag_reg_min_tiles)) return 1;
#define TSA_X(D, A, S, T) \
    if (algo == (A) && total == (T) && ((A) == ALLRED_SWING_1D || side == (S))) return fused_chunk_launches(tiles);
        TSA_LO_DAGS(TSA_X)
#undef TSA_X
        return 1;   // the butterfly forms: one launch
    }
    return big64 && fused_form() == 0 ? fused_chunk_launches(tiles) : 1;
}

// The persistent lagged passes (k_tree_lds_lag, k_lo_dag_reg, k_mem_lds_lag)
// on large buckets: a sequence of launches over tile ranges a .. b-1 of about
// fused_chunk_tiles tiles each (1280 = config 2's 2.5 tiles per workgroup).
// Each launch opens with two tiles' loads on every workgroup — most of its
// reads in one burst before its first store — while one launch over many
// tiles per workgroup interleaves reads and writes throughout: 5.6-5.7 vs
// 5.0-5.5 TB/s at 1.3-5.2 MB per rank (profiles/r02_fused_chunk_ab.txt).
template <class F>
void for_each_chunk(uint64_t tiles, F&& launch) {
    const uint64_t nl = fused_chunk_launches(tiles);
    for (uint64_t l = 0; l < nl; ++l) launch(tiles * l / nl, tiles * (l + 1) / nl);
}

int launch_tree_fused(uint16_t* ranks, uint64_t stride, size_t n, int total, const uint8_t* order, void* stream,
                      bool host_memory) {
    if (n % (8 * (size_t)total) || stride % 8 || !aligned16(ranks)) return ALLRED_ERR_ARG;
    const uint64_t nv = n / 8, bv = nv / total, tiles = nv / 32;
    const int64_t form = fused_form();
    hipStream_t st = (hipStream_t)stream;
    const bool whole_tiles = total >= 8 && nv % 32 == 0 && bv % 32 == 0;
    // config 2 (64 ranks, >= 1024 tiles on HBM): k_tree_lds_lag, two workgroups
    // per CU (14.2-14.3 us vs 15.3 for k_tree_lds_pipe and 16.2 for one tile
    // per workgroup)
    if (whole_tiles && !host_memory && total == 64 && form == 0 && tiles >= 1024) {
        for_each_chunk(tiles, [&](uint64_t a, uint64_t b) {
            const unsigned grid = persistent_grid(b - a, 512);
            hipLaunchKernelGGL((k_tree_lds_lag<64>), dim3(grid), dim3(kBlock), 0, st, ranks, stride, order, bv, a,
                               b - a);
            note_launch(reinterpret_cast<const void*>(&k_tree_lds_lag<64>), "k_tree_lds_lag<64>", grid, kBlock);
        });
        return last_error();
    }
    // pinned host buckets (zero-copy: PCIe-bound, 32 workgroups keep both link
    // directions busy, tools/pcie_probe.py), or forced persistent form
    if (whole_tiles && (host_memory || form == 3)) {
        const unsigned grid = persistent_grid(tiles, host_memory ? 32 : 512);
        switch (total) {
            case 8: hipLaunchKernelGGL((k_tree_lds_pipe<8>), dim3(grid), dim3(kBlock), 0, st, ranks, stride, order, bv, tiles, nullptr); break;
            case 16: hipLaunchKernelGGL((k_tree_lds_pipe<16>), dim3(grid), dim3(kBlock), 0, st, ranks, stride, order, bv, tiles, nullptr); break;
            case 32: hipLaunchKernelGGL((k_tree_lds_pipe<32>), dim3(grid), dim3(kBlock), 0, st, ranks, stride, order, bv, tiles, nullptr); break;
            case 64: hipLaunchKernelGGL((k_tree_lds_pipe<64>), dim3(grid), dim3(kBlock), 0, st, ranks, stride, order, bv, tiles, nullptr); break;
            default: return ALLRED_ERR_UNSUPPORTED;
        }
        return last_error();
    }
    return tree_dispatch<true>(ranks, stride, nv, total, order, bv, nullptr, st);
}

int launch_lo_dag_reg(uint16_t* ranks, uint64_t stride, size_t n, int algo, int side, int total, void* stream) {
    if (n % 256 || stride % 8 || !aligned16(ranks)) return ALLRED_ERR_UNSUPPORTED;
    const uint64_t tiles = n / 256;
    hipStream_t st = (hipStream_t)stream;
#define TSA_X(D, A, S, T)                                                                             \
    if (algo == (A) && total == (T) && ((A) == ALLRED_SWING_1D || side == (S))) {                      \
        for_each_chunk(tiles, [&](uint64_t a, uint64_t b) {                                           \
            hipLaunchKernelGGL(k_lo_dag_reg<D>, dim3(persistent_grid(b - a, 512)), dim3(kBlock), 0, st, \
                               ranks, stride, a, b - a);                                              \
        });                                                                                           \
        return last_error();                                                                          \
    }
    TSA_LO_DAGS(TSA_X)
#undef TSA_X
    return ALLRED_ERR_UNSUPPORTED;
}

int launch_butterfly(uint16_t* ranks, uint64_t stride, size_t n, int total, const int16_t* d_partner, int steps,
                     const uint8_t* dag, void* stream) {
    if (n % 8 || stride % 8 || !aligned16(ranks)) return ALLRED_ERR_ARG;
    const uint64_t nv = n / 8, tiles = nv / 32;
    hipStream_t st = (hipStream_t)stream;
    const int64_t form = fused_form();
    // 64 ranks, whole tiles: the persistent double-buffered LDS pass — as the
    // DAG of distinct sums from lo_dag_min_tiles tiles (default 256: 128 kB per
    // rank), else the per-rank butterfly from 1024 tiles (640 kB: 23.9 vs
    // 25.2-26.0 us for one tile per workgroup).  Below: the one-tile LDS form
    // from 256 tiles, the register butterfly under that (latency-bound:
    // 16 kB 3.8 vs 5.7 us for the DAG pass, profiles/r01_lo_dag_min_ab.txt).
    const bool dag_pipe = dag && form != 2 && tiles >= (uint64_t)tune(Tune::lo_dag_min_tiles);
    if (total == 64 && nv % 32 == 0 && nv >= 32 &&
        (dag_pipe || (tiles >= 256 && (form == 3 || (tiles >= 1024 && form != 2))))) {
        const dim3 grid(persistent_grid(tiles, 512));
        if (dag)
            hipLaunchKernelGGL(k_butterfly_lds64_pipe<4>, grid, dim3(kBlock), 0, st, ranks, stride, d_partner, steps,
                               tiles, dag);
        else
            hipLaunchKernelGGL(k_butterfly_lds64_pipe<0>, grid, dim3(kBlock), 0, st, ranks, stride, d_partner, steps,
                               tiles, nullptr);
        return last_error();
    }
    if (total == 64 && nv % 32 == 0 && tiles >= 256) {  // >= 256 tiles: the LDS-staged form pays
        hipLaunchKernelGGL(k_butterfly_lds64, dim3((unsigned)tiles), dim3(kBlock), 0, st, ranks, stride, d_partner,
                           steps);
        return last_error();
    }
    const int Q = 64 / total;
    const bool small = nv < (uint64_t)Q * 8 * 1024;   // fewer than 1024 waves at U = 8: go wide instead
    const int U = small ? 1 : 8;
    uint64_t waves = (nv + (uint64_t)Q * U - 1) / ((uint64_t)Q * U);
    uint64_t blocks = (waves + 3) / 4;
    if (blocks < 1) blocks = 1;
    if (blocks > 256 * 16) blocks = 256 * 16;
    const dim3 grid((unsigned)blocks), blk(kBlock);
#define TSA_BFLY(PP)                                                                                          \
    if (small) hipLaunchKernelGGL((k_butterfly<PP, 1>), grid, blk, 0, st, ranks, stride, nv, d_partner, steps); \
    else hipLaunchKernelGGL((k_butterfly<PP, 8>), grid, blk, 0, st, ranks, stride, nv, d_partner, steps);
    switch (total) {
        case 1: return ALLRED_OK;  // one rank: nothing to reduce
        case 2: TSA_BFLY(2) break;
        case 4: TSA_BFLY(4) break;
        case 8: TSA_BFLY(8) break;
        case 16: TSA_BFLY(16) break;
        case 32: TSA_BFLY(32) break;
        case 64: TSA_BFLY(64) break;
        default: return ALLRED_ERR_UNSUPPORTED;
    }
#undef TSA_BFLY
    return last_error();
}

int launch_tree_reduce(const uint16_t* ranks, uint64_t stride, size_t n, int total, const uint8_t* order,
                       uint16_t* out, void* stream) {
    if (n % 8 || stride % 8 || !aligned16(ranks) || !aligned16(out)) return ALLRED_ERR_ARG;
    return tree_dispatch<false>(const_cast<uint16_t*>(ranks), stride, n / 8, total, order, 0, out,
                                (hipStream_t)stream);
}

int launch_tree_bcast_x(uint16_t* cur, uint16_t* prev, uint64_t stride, size_t n, int total, const uint8_t* order,
                        uint16_t* cur_partial, const uint16_t* prev_result, void* stream) {
    if (n % 8 || stride % 8 || stride < n || !aligned16(cur) || !aligned16(prev) || !aligned16(cur_partial) ||
        !aligned16(prev_result))
        return ALLRED_ERR_ARG;
    // 64 ranks in whole 256-element tiles: one fused pass; else the two launches (same bits)
    if (total == 64 && n % 256 == 0) {
        hipStream_t st = (hipStream_t)stream;
        for_each_chunk(n / 256, [&](uint64_t a, uint64_t b) {
            const dim3 grid(persistent_grid(b - a, 512));
            switch (tune(Tune::tree_bcast_lag) * 2 + tune(Tune::tree_bcast_bal)) {
#define TSA_TBX(L, B) hipLaunchKernelGGL((k_tree_bcast_x<L, B>), grid, dim3(kBlock), 0, st, cur, prev, stride, order, \
                                         cur_partial, prev_result, a, b - a)
                case 0: TSA_TBX(0, false); break;
                case 1: TSA_TBX(0, true); break;
                case 2: TSA_TBX(1, false); break;
                default: TSA_TBX(1, true); break;
#undef TSA_TBX
            }
        });
        return last_error();
    }
    int st = launch_broadcast(prev, stride, n, total, prev_result, stream);
    return st != ALLRED_OK ? st : launch_tree_reduce(cur, stride, n, total, order, cur_partial, stream);
}

int launch_broadcast(uint16_t* ranks, uint64_t stride, size_t n, int total, const uint16_t* src, void* stream) {
    if (n % 8 || stride % 8 || !aligned16(ranks) || !aligned16(src)) return ALLRED_ERR_ARG;
    const uint64_t nv = n / 8;
    hipLaunchKernelGGL(k_broadcast, dim3(grid_all(nv), (total + 7) / 8), dim3(kBlock), 0, (hipStream_t)stream, ranks,
                       stride, total, reinterpret_cast<const uint4*>(src), nv);
    return last_error();
}

int launch_bo_steps(uint16_t* ranks, uint64_t stride, int total, int steps, const uint8_t* d_tab,
                    const uint8_t* d_pipe_tab, const uint8_t* d_reg_tab, size_t block_elems, uint64_t* stamps,
                    void* stream) {
    if (steps == 0) return ALLRED_OK;   // one rank: nothing to exchange
    if (block_elems % 8 || stride % 8 || !aligned16(ranks) || total < 2 || total > ALLRED_MAX_NODES) return ALLRED_ERR_ARG;
    const uint64_t bv = block_elems / 8, slices = (bv + kStepSV - 1) / kStepSV, units = slices * (uint64_t)total;
    hipStream_t st = (hipStream_t)stream;
    // whole 512-byte slices, 8..64 ranks: the register-staged form (k_steps_reg), 3 workgroups per CU by
    // default (15.3-15.7 us at config 2 vs 16.8-17.2 with 4 per CU, profiles/r03_steps_wave_ab.txt)
    if (d_reg_tab && tune(Tune::steps_form) == 0 && bv % kStepSV == 0 && (1 << steps) == total) {
        const int g = (int)tune(Tune::steps_groups);
        if (launch_steps_reg(true, g ? g : 3, ranks, stride, total, d_reg_tab, d_reg_tab + (size_t)kBoPipeTabBytes * total,
                             bv, slices, units, stamps, st))
            return last_error();
    }
    const unsigned grid = (unsigned)(units < (uint64_t)kMaxGrid ? units : (uint64_t)kMaxGrid);
    hipLaunchKernelGGL(k_bo_steps, dim3(grid), dim3(kBlock), 0, st, ranks, stride, d_tab, total, steps,
                       bv, slices, units, stamps);
    return last_error();
}

uint64_t bo_steps_units(size_t block_elems, int total) {
    return (block_elems / 8 + kStepSV - 1) / kStepSV * (uint64_t)total;
}

int launch_lo_steps(uint16_t* ranks, uint64_t stride, int total, int steps, const uint8_t* d_pairs,
                    const uint8_t* d_pipe_tab, size_t n, uint64_t* stamps, void* stream) {
    if (steps == 0) return ALLRED_OK;   // one rank: nothing to exchange
    if (n % 8 || stride % 8 || !aligned16(ranks) || total < 2 || total > ALLRED_MAX_NODES) return ALLRED_ERR_ARG;
    const uint64_t nv = n / 8, units = (nv + kStepSV - 1) / kStepSV;
    hipStream_t st = (hipStream_t)stream;
    // whole 512-byte slices, 8..64 ranks: k_steps_reg, 4 workgroups per CU by default (15.6-15.8 us at 640 kB
    // vs 16.1-16.3 with 3), but 3 where 4 would give every wave exactly one strip (768 < units <= 1024: all
    // loads, then all stores, 17.1 vs 15.4 us at 512 kB; profiles/r03_steps_wave_ab.txt)
    if (d_pipe_tab && tune(Tune::steps_form) == 0 && nv % kStepSV == 0 && (1 << steps) == total) {
        const int g = (int)tune(Tune::steps_groups);
        const int per_cu = g ? g : (units > 768 && units <= 1024 ? 3 : 4);
        if (launch_steps_reg(false, per_cu, ranks, stride, total, d_pipe_tab, nullptr, 0, 1, units, stamps, st))
            return last_error();
    }
    const unsigned grid = (unsigned)(units < (uint64_t)kMaxGrid ? units : (uint64_t)kMaxGrid);
    hipLaunchKernelGGL(k_lo_steps, dim3(grid), dim3(kBlock), 0, st, ranks, stride, d_pairs, total,
                       steps, nv, units, stamps);
    return last_error();
}

uint64_t lo_steps_units(size_t n) { return (n / 8 + kStepSV - 1) / kStepSV; }

static int launch_step(bool add, uint16_t* ranks, uint64_t stride, int total, const int16_t* d_partner,
                       const int16_t* d_blocks, int blocks_per_rank, size_t block_elems, void* stream) {
    if (block_elems % 8 || stride % 8 || !aligned16(ranks)) return ALLRED_ERR_ARG;
    const uint64_t bv = block_elems / 8;
    const dim3 g((unsigned)(total * blocks_per_rank));
    if (add)
        hipLaunchKernelGGL((k_step_w<true, 8>), g, dim3(64), 0, (hipStream_t)stream, ranks, stride, d_partner, d_blocks,
                           blocks_per_rank, bv);
    else
        hipLaunchKernelGGL((k_step_w<false, 8>), g, dim3(64), 0, (hipStream_t)stream, ranks, stride, d_partner,
                           d_blocks, blocks_per_rank, bv);
    return last_error();
}

int launch_rs_step(uint16_t* ranks, uint64_t stride, int total, const int16_t* d_partner, const int16_t* d_blocks,
                   int blocks_per_rank, size_t block_elems, void* stream) {
    return launch_step(true, ranks, stride, total, d_partner, d_blocks, blocks_per_rank, block_elems, stream);
}

int launch_ag_step(uint16_t* ranks, uint64_t stride, int total, const int16_t* d_partner, const int16_t* d_blocks,
                   int blocks_per_rank, size_t block_elems, void* stream) {
    return launch_step(false, ranks, stride, total, d_partner, d_blocks, blocks_per_rank, block_elems, stream);
}

int launch_lo_step(const uint16_t* src, uint64_t src_stride, uint16_t* dst, uint64_t dst_stride, int total,
                   const int16_t* d_partner, size_t n, void* stream) {
    if (n % 8 || src_stride % 8 || dst_stride % 8 || !aligned16(src) || !aligned16(dst)) return ALLRED_ERR_ARG;
    const uint64_t nv = n / 8;
    hipLaunchKernelGGL(k_lo_step, dim3(grid_all(nv), total), dim3(kBlock), 0, (hipStream_t)stream, src, src_stride,
                       dst, dst_stride, d_partner, nv);
    return last_error();
}

int launch_copy_ranks(const uint16_t* src, uint64_t src_stride, uint16_t* dst, uint64_t dst_stride, int total,
                      size_t n, void* stream) {
    if (n % 8 || src_stride % 8 || dst_stride % 8 || !aligned16(src) || !aligned16(dst)) return ALLRED_ERR_ARG;
    const uint64_t nv = n / 8;
    hipLaunchKernelGGL(k_copy_ranks, dim3(grid_all(nv), total), dim3(kBlock), 0, (hipStream_t)stream, src, src_stride,
                       dst, dst_stride, nv);
    return last_error();
}

namespace {
template <bool ACC16>
int mem_reduce_impl(uint16_t* r, uint64_t stride, uint64_t nv, int total, uint16_t* dst, hipStream_t st) {
    const uint64_t bv = nv / total;
    // block rows in whole 256-element tiles: the fused pass's LDS form (every
    // rank's tile staged by LDS-DMA, one thread per dword sums from LDS in the
    // same order), one workgroup per tile, result to dst only: 640 kB 9.1 us vs
    // 13.6 for k_mem<false, 16> (160 workgroups: one thread per 16-byte
    // column), profiles/r01_mem_reduce_ab.txt
    if (tune(Tune::mem_reduce_lds) && bv % 32 == 0 && total >= 4 && total <= 64 && (total & (total - 1)) == 0) {
        const dim3 grid((unsigned)(nv / 32)), blk(128);
        switch (total) {
            case 4: hipLaunchKernelGGL((k_mem_lds<4, ACC16>), grid, blk, 0, st, r, stride, bv, dst); break;
            case 8: hipLaunchKernelGGL((k_mem_lds<8, ACC16>), grid, blk, 0, st, r, stride, bv, dst); break;
            case 16: hipLaunchKernelGGL((k_mem_lds<16, ACC16>), grid, blk, 0, st, r, stride, bv, dst); break;
            case 32: hipLaunchKernelGGL((k_mem_lds<32, ACC16>), grid, blk, 0, st, r, stride, bv, dst); break;
            default: hipLaunchKernelGGL((k_mem_lds<64, ACC16>), grid, blk, 0, st, r, stride, bv, dst); break;
        }
        return last_error();
    }
    // one column per thread reads all `total` ranks, sixteen ranks' loads in
    // flight per thread (22.1-22.3 vs 22.7 us with eight, profiles/r01_mem_batch_ab.txt)
    uint64_t g = (nv + kBlock - 1) / kBlock;
    if (g > (uint64_t)kMaxGrid) g = kMaxGrid;
    hipLaunchKernelGGL((k_mem<false, 16, ACC16>), dim3((unsigned)g), dim3(kBlock), 0, st, r, stride, total, nv, bv, dst);
    return last_error();
}

template <bool ACC16>
int mem_fused_impl(uint16_t* ranks, uint64_t stride, uint64_t nv, int total, hipStream_t st) {
    const uint64_t bv = nv / total, tiles = nv / 32;
    if (bv % 32 == 0 && total == 64 && tiles >= 1024 && fused_form() == 0) {
        // persistent, stores one iteration late (k_tree_lds_lag's schedule)
        for_each_chunk(tiles, [&](uint64_t a, uint64_t b) {
            hipLaunchKernelGGL((k_mem_lds_lag<ACC16>), dim3(persistent_grid(b - a, 512)), dim3(kBlock), 0, st, ranks,
                               stride, bv, a, b - a);
        });
        return last_error();
    }
    if (bv % 32 == 0 && total >= 4 && fused_form() != 1) {
        const dim3 grid((unsigned)tiles), blk(128);
        switch (total) {
            case 4: hipLaunchKernelGGL((k_mem_lds<4, ACC16>), grid, blk, 0, st, ranks, stride, bv, nullptr); return last_error();
            case 8: hipLaunchKernelGGL((k_mem_lds<8, ACC16>), grid, blk, 0, st, ranks, stride, bv, nullptr); return last_error();
            case 16: hipLaunchKernelGGL((k_mem_lds<16, ACC16>), grid, blk, 0, st, ranks, stride, bv, nullptr); return last_error();
            case 32: hipLaunchKernelGGL((k_mem_lds<32, ACC16>), grid, blk, 0, st, ranks, stride, bv, nullptr); return last_error();
            case 64: hipLaunchKernelGGL((k_mem_lds<64, ACC16>), grid, blk, 0, st, ranks, stride, bv, nullptr); return last_error();
            default: break;
        }
    }
    hipLaunchKernelGGL((k_mem<true, 8, ACC16>), dim3(grid_for(nv)), dim3(kBlock), 0, st, ranks, stride, total, nv, bv,
                       nullptr);
    return last_error();
}
}  // namespace

int launch_mem_reduce(const uint16_t* ranks, uint64_t stride, size_t n, int total, uint16_t* dst, bool acc16,
                      void* stream) {
    if (n % (8 * (size_t)total) || stride % 8 || !aligned16(ranks) || !aligned16(dst)) return ALLRED_ERR_ARG;
    uint16_t* r = const_cast<uint16_t*>(ranks);
    return acc16 ? mem_reduce_impl<true>(r, stride, n / 8, total, dst, (hipStream_t)stream)
                 : mem_reduce_impl<false>(r, stride, n / 8, total, dst, (hipStream_t)stream);
}

int launch_rows_sum(const uint16_t* rows, uint64_t stride, size_t n, int nrows, uint16_t* dst, bool acc16,
                    void* stream) {
    if (n % 8 || stride % 8 || nrows < 1 || !aligned16(rows) || !aligned16(dst)) return ALLRED_ERR_ARG;
    const uint64_t nv = n / 8;
    if (!nv) return ALLRED_OK;
    uint64_t g = (nv + kBlock - 1) / kBlock;
    if (g > (uint64_t)kMaxGrid) g = kMaxGrid;
    uint16_t* r = const_cast<uint16_t*>(rows);
    // k_mem with one block (block_vec = n_vec): owner row 0 first, then rows 1 .. nrows-1 in order
    if (acc16)
        hipLaunchKernelGGL((k_mem<false, 16, true>), dim3((unsigned)g), dim3(kBlock), 0, (hipStream_t)stream, r, stride,
                           nrows, nv, nv, dst);
    else
        hipLaunchKernelGGL((k_mem<false, 16, false>), dim3((unsigned)g), dim3(kBlock), 0, (hipStream_t)stream, r,
                           stride, nrows, nv, nv, dst);
    return last_error();
}

int launch_mem_fused(uint16_t* ranks, uint64_t stride, size_t n, int total, bool acc16, void* stream) {
    if (n % (8 * (size_t)total) || stride % 8 || !aligned16(ranks)) return ALLRED_ERR_ARG;
    return acc16 ? mem_fused_impl<true>(ranks, stride, n / 8, total, (hipStream_t)stream)
                 : mem_fused_impl<false>(ranks, stride, n / 8, total, (hipStream_t)stream);
}

}  // namespace tsa
