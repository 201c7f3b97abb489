// kernels.hip — CDNA4 (gfx950) kernels of the allreduce engine.
//
// Every kernel is HBM-bound integer/bf16 streaming work: 16-byte (8 x bf16)
// accesses per lane, fp32 add, v_cvt_pk_bf16_f32 (round-to-nearest-even)
// back to bf16.  No MFMA: a pointwise add is not a contraction.
//
// Replaces the Tensix compute kernels of the reference:
//   add_tiles + pack_tile<true>      allred_BO_2D/kernels/compute_kernel.cpp:53-60
//   LO_2D add loop                   allred_LO_2D/kernels/compute_kernel.cpp:50-62
//   mem_2D dest-reuse accumulate     allred_mem_2D/kernels/compute_kernel.cpp:43-72
// and the NoC block moves of the dataflow kernels (RS / AG loops,
// allred_BO_2D/kernels/dataflow_kernel.cpp:152-267) for ranks resident in
// one GPU's HBM, where a "send" is a load of the partner's bytes.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "internal.hpp"

namespace tsa {
namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float lo_f(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_f(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// two fp32 -> packed bf16x2, round to nearest even (one v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pack_rne(float lo, float hi) {
    f32x2 v = {lo, hi};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}

__device__ __forceinline__ uint32_t add2(uint32_t a, uint32_t b) {
    return pack_rne(lo_f(a) + lo_f(b), hi_f(a) + hi_f(b));
}

// 8 x bf16 add with one bf16 rounding per element (Tensix add_tiles with
// fp32_dest_acc_en = false, allred_helper.cpp:331-335)
__device__ __forceinline__ uint4 add8(uint4 a, uint4 b) {
    uint4 o;
    o.x = add2(a.x, b.x);
    o.y = add2(a.y, b.y);
    o.z = add2(a.z, b.z);
    o.w = add2(a.w, b.w);
    return o;
}

__device__ __forceinline__ uint4 shfl_xor4(uint4 v, int m) {
    uint4 o;
    o.x = (uint32_t)__shfl_xor((int)v.x, m);
    o.y = (uint32_t)__shfl_xor((int)v.y, m);
    o.z = (uint32_t)__shfl_xor((int)v.z, m);
    o.w = (uint32_t)__shfl_xor((int)v.w, m);
    return o;
}

// Streaming (nontemporal) 16-byte accesses: every byte of a bucket is read
// once and written once per pass, so nothing is worth keeping in L2 / MALL
// (measured: the fused tree pass 19.2 -> 16.0 us, the tile-sum 5.9 -> 6.4 TB/s).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt(const uint4* p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_nt(uint4* p, uint4 v) {
    const u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
}

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(1))) const uint32_t global_u32;

__device__ __forceinline__ uint64_t gtid() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ uint64_t gthreads() { return (uint64_t)gridDim.x * blockDim.x; }

constexpr int kBlock = 256;          // 4 waves per workgroup
constexpr int kMaxGrid = 256 * 8;    // 256 CUs x 8 resident workgroups, then grid-stride

// one item per thread up to 2^30 threads
inline unsigned grid_all(uint64_t work_items) {
    uint64_t g = (work_items + kBlock - 1) / kBlock;
    if (g < 1) g = 1;
    if (g > (1ull << 22)) g = 1ull << 22;
    return (unsigned)g;
}

inline unsigned grid_for(uint64_t work_items) {
    uint64_t g = (work_items + kBlock - 1) / kBlock;
    if (g < 1) g = 1;
    if (g > (uint64_t)kMaxGrid) g = kMaxGrid;
    return (unsigned)g;
}

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
// dst[b] += src[b] for the blocks b listed (one BO compute step of one rank)
// ---------------------------------------------------------------------------
struct BlockList {
    uint8_t b[ALLRED_MAX_NODES];
};

__global__ __launch_bounds__(kBlock) void k_add_blocks(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                       BlockList list, uint64_t block_vec) {
    const uint64_t off = (uint64_t)list.b[blockIdx.y] * block_vec;
    for (uint64_t v = gtid(); v < block_vec; v += gthreads())
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
// so the pass is safe in place.
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
// k_tree_lds with a persistent grid and D+1 LDS tile buffers (prefetch depth
// D): tile j+D's loads are issued before tile j is reduced and stored, and
// the wait before tile j is an exact s_waitcnt vmcnt(n) that leaves every op
// issued after tile j's loads in flight (CDNA3/4 count VMEM loads, LDS-DMA
// loads and stores on one in-order vmcnt).  Loads of later tiles and stores
// of earlier ones overlap: on pinned HOST buckets (zero-copy end to end) the
// two PCIe directions run at once; on HBM it hides the per-tile ramp.
// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int OPS, int D>
__device__ __forceinline__ void wait_tile(int after) {  // after = tiles' worth of ops issued after this tile's loads
    static_assert(2 * D * OPS <= 63, "vmcnt is 6 bits");
    switch (after) {
        case 0: wait_vm<0>(); break;
        case 1: wait_vm<OPS>(); break;
        case 2: wait_vm<2 * OPS>(); break;
        case 3: if constexpr (D >= 2) { wait_vm<3 * OPS>(); break; } else { wait_vm<0>(); break; }
        default: wait_vm<0>(); break;
    }
}

// vmcnt(k * OPS) for a run-time k in 0..7
template <int OPS>
__device__ __forceinline__ void wait_units(int k) {
    switch (k) {
        case 0: wait_vm<0>(); break;
        case 1: wait_vm<OPS>(); break;
        case 2: wait_vm<(2 * OPS < 63 ? 2 * OPS : 63)>(); break;
        case 3: wait_vm<(3 * OPS < 63 ? 3 * OPS : 63)>(); break;
        case 4: wait_vm<(4 * OPS < 63 ? 4 * OPS : 63)>(); break;
        case 5: wait_vm<(5 * OPS < 63 ? 5 * OPS : 63)>(); break;
        case 6: wait_vm<(6 * OPS < 63 ? 6 * OPS : 63)>(); break;
        default: wait_vm<(7 * OPS < 63 ? 7 * OPS : 63)>(); break;
    }
}

// vmcnt(n) for a run-time n in 0..63 (larger n waits for 63: conservative)
__device__ __forceinline__ void wait_any(int n) {
    switch (n) {
        case 0: wait_vm<0>(); break;
        case 1: wait_vm<1>(); break;
        case 2: wait_vm<2>(); break;
        case 3: wait_vm<3>(); break;
        case 4: wait_vm<4>(); break;
        case 5: wait_vm<5>(); break;
        case 6: wait_vm<6>(); break;
        case 7: wait_vm<7>(); break;
        case 8: wait_vm<8>(); break;
        case 9: wait_vm<9>(); break;
        case 10: wait_vm<10>(); break;
        case 11: wait_vm<11>(); break;
        case 12: wait_vm<12>(); break;
        case 13: wait_vm<13>(); break;
        case 14: wait_vm<14>(); break;
        case 15: wait_vm<15>(); break;
        case 16: wait_vm<16>(); break;
        case 17: wait_vm<17>(); break;
        case 18: wait_vm<18>(); break;
        case 19: wait_vm<19>(); break;
        case 20: wait_vm<20>(); break;
        case 21: wait_vm<21>(); break;
        case 22: wait_vm<22>(); break;
        case 23: wait_vm<23>(); break;
        case 24: wait_vm<24>(); break;
        case 25: wait_vm<25>(); break;
        case 26: wait_vm<26>(); break;
        case 27: wait_vm<27>(); break;
        case 28: wait_vm<28>(); break;
        case 29: wait_vm<29>(); break;
        case 30: wait_vm<30>(); break;
        case 31: wait_vm<31>(); break;
        case 32: wait_vm<32>(); break;
        case 33: wait_vm<33>(); break;
        case 34: wait_vm<34>(); break;
        case 35: wait_vm<35>(); break;
        case 36: wait_vm<36>(); break;
        case 37: wait_vm<37>(); break;
        case 38: wait_vm<38>(); break;
        case 39: wait_vm<39>(); break;
        case 40: wait_vm<40>(); break;
        case 41: wait_vm<41>(); break;
        case 42: wait_vm<42>(); break;
        case 43: wait_vm<43>(); break;
        case 44: wait_vm<44>(); break;
        case 45: wait_vm<45>(); break;
        case 46: wait_vm<46>(); break;
        case 47: wait_vm<47>(); break;
        case 48: wait_vm<48>(); break;
        case 49: wait_vm<49>(); break;
        case 50: wait_vm<50>(); break;
        case 51: wait_vm<51>(); break;
        case 52: wait_vm<52>(); break;
        case 53: wait_vm<53>(); break;
        case 54: wait_vm<54>(); break;
        case 55: wait_vm<55>(); break;
        case 56: wait_vm<56>(); break;
        case 57: wait_vm<57>(); break;
        case 58: wait_vm<58>(); break;
        case 59: wait_vm<59>(); break;
        case 60: wait_vm<60>(); break;
        case 61: wait_vm<61>(); break;
        case 62: wait_vm<62>(); break;
        case 63: wait_vm<63>(); break;
        default: wait_vm<63>(); break;
    }
}

// LDS-DMA load issued as inline asm: the compiler's waitcnt pass then does
// not see an LDS write in flight and does not put vmcnt(0) in front of every
// LDS read (which would serialise the pipeline); wait_tile() is the only wait.
// (m0 is reserved for the compiler; nothing else in the kernels that use this
// reads it — checked in the ISA — so clobbering it here is safe.)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void lds_dma16(const void* src, uint32_t lds_base) {
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off nt" ::"v"(src), "s"(lds_base) : "memory", "m0");
}
#pragma clang diagnostic pop

// workgroup barrier without the release fence of __syncthreads (which waits
// vmcnt(0)); LDS traffic is ordered by the lgkmcnt wait
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// TV = 16-byte vectors per rank row of a tile (32: 32 KiB tiles at P = 64, two
// workgroups per CU; 16: 16 KiB tiles, four per CU).  A wave-instruction
// stages RPI = 64 / TV rank rows (1 KiB contiguous per row group).
// WRITE_ALL = false: the hierarchical partial — the tree of every tile goes to
// `out` (one row; wave 0 issues its one store per tile, so its wait leaves
// that one store in flight and the other waves wait for their loads alone).
// REL (early release, two buffers): tile j+2's loads go into tile j's buffer
// as soon as every wave has read tile j out of LDS (after the partials'
// barrier), before tile j's stores and before the wait for tile j+1 — so two
// tiles' loads are in flight per workgroup most of the time instead of one.
template <int P, int D, int TV, bool WRITE_ALL = true, bool REL = false>
__global__ __launch_bounds__(kBlock) void k_tree_lds_pipe(uint16_t* __restrict__ ranks, uint64_t stride,
                                                          const uint8_t* __restrict__ order, uint64_t block_vec,
                                                          uint64_t ntiles, uint16_t* __restrict__ out) {
    constexpr int RPI = 64 / TV, RPW = P / 4, OPS = RPW / RPI, LPL = OPS, NB = D + 1;
    static_assert(OPS >= 1, "tile too narrow for this rank count");
    static_assert(WRITE_ALL || D == 1, "partial form is double-buffered only");
    static_assert(!REL || (WRITE_ALL && (2 * NB - 1) * OPS <= 63), "early release: full form, vmcnt <= 63");
    __shared__ __attribute__((aligned(16))) uint4 buf[NB][P * TV];
    __shared__ __attribute__((aligned(16))) uint4 part[4 * TV];
    __shared__ __attribute__((aligned(16))) uint8_t ord_lds[P * ALLRED_MAX_NODES];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane % TV, q = lane / TV;
    const uint32_t wbase = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&buf[0][0] +
        (uint32_t)(RPW * w * TV * 16));
    auto issue = [&](uint64_t t, int b) {
#pragma unroll
        for (int k = 0; k < OPS; ++k) {
            const int r = RPW * w + RPI * k + q;
            const uint4* src = reinterpret_cast<const uint4*>(ranks + (uint64_t)r * stride) + t * TV + c;
            lds_dma16(src, wbase + (uint32_t)(b * P * TV * 16 + RPI * k * TV * 16));
        }
    };
    const uint64_t G = gridDim.x;
    // tiles of this WG: blockIdx.x + j * G, so the workgroups in flight together
    // read adjacent 512-byte segments of every rank row (a contiguous run per
    // workgroup instead measured 18.8 vs 15.6 us: DRAM page locality across
    // workgroups is what counts; 16-vector tiles, 256 B per row, 17.1-17.7)
    const uint64_t first = blockIdx.x, step = G;
    const int mine = blockIdx.x < ntiles ? (int)((ntiles - 1 - blockIdx.x) / G + 1) : 0;
    // the order rows of all P blocks, once, then the first tiles' loads
    // (issuing those first measured slower: 15.65 vs 15.3 us at config 2)
    for (int i = threadIdx.x; i < P * ALLRED_MAX_NODES / 16; i += kBlock)
        reinterpret_cast<uint4*>(ord_lds)[i] = reinterpret_cast<const uint4*>(order)[i];
    __syncthreads();
#pragma unroll
    for (int d = 0; d < (REL ? NB : D); ++d)
        if (d < mine) issue(first + d * step, d);
    for (int j = 0; j < mine; ++j) {
        const int rem = mine - 1 - j;
        if (REL && WRITE_ALL) {
            // issued after tile j's loads (OPS ops each): the stores of tiles
            // j-NB .. j-1 (those that exist) and the loads of tiles j+1 .. j+NB-1
            // (prologue or earlier iterations, those that exist)
            wait_units<OPS>((j < NB ? j : NB) + (rem < NB - 1 ? rem : NB - 1));
        } else if (WRITE_ALL) {
            wait_tile<OPS, D>((j < D ? j : D) + (rem < D - 1 ? rem : D - 1));
        } else if (j > 0 && w == 0) {
            wait_vm<1>();   // tile j-1's partial store may stay in flight
        } else {
            wait_vm<0>();
        }
        lds_barrier();
        if (!REL && j + D < mine) issue(first + (uint64_t)(j + D) * step, (j + D) % NB);
        const uint4* tile = buf[j % NB];
        const uint64_t v0 = (first + (uint64_t)j * step) * TV;
        const uint8_t* ord = ord_lds + (block_vec ? v0 / block_vec : 0) * ALLRED_MAX_NODES + RPW * w + LPL * q;
        uint4 x[LPL];
#pragma unroll
        for (int i = 0; i < LPL; ++i) x[i] = tile[(int)ord[i] * TV + c];
#pragma unroll
        for (int s = 1; s < LPL; s *= 2)
#pragma unroll
            for (int i = 0; i < LPL; i += 2 * s) x[i] = add8(x[i], x[i + s]);
        uint4 pw = x[0];
#pragma unroll
        for (int s = TV; s < 64; s *= 2) pw = add8(pw, shfl_xor4(pw, s));   // tree levels across lane groups
        if (q == 0) part[w * TV + c] = pw;
        lds_barrier();   // every wave has read tile j out of buf[j % NB]
        if (REL && j + NB < mine) issue(first + (uint64_t)(j + NB) * step, j % NB);
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
// k_tree_lds_lag: the fused BO pass of k_tree_lds_pipe (same tree, same bits)
// with every tile's stores one iteration late.  Iteration j: wait for tile j's
// loads, reduce it out of LDS, issue tile j+2's loads into its buffer (early
// release), then store tile j-1's result, kept in registers from the previous
// iteration.  A tile's stores thus always queue behind the next tile's loads
// (k_tree_lds_pipe issues them between two loads), and the waves never wait
// for a store before a load.  Measured on the hierarchical step's data path
// (tools/ubench/ws_trace.hip): 14.6 us vs 15.4 us with stores in iteration j.
// VAR (A/B arms, tools/ubench/fused_ab.hip, profiles/r01_fused_ab_arms.txt):
// 7 the product = 2 with tile j+2's loads and tile j-1's stores interleaved op
// by op (14.22-14.26 vs 14.32-14.36 us, profiles/r01_fused_ab_interleave.txt);
// 2: the first two tiles' loads issued before the 4 KiB tree-order
// table is staged (14.23-14.29 vs 14.39-14.40 us); 0 the table first; 1 = 0
// with an LDS-counter barrier instead of s_barrier (no gain); 3 no table at
// all (leaf order = rank order: timing only, wrong bits for Swing; no faster);
// 7 = 2 with tile j+2's loads and tile j-1's stores interleaved op by op.
// Issue order per wave: L0 L1 | L2 | L3 S0 | L4 S1 | ..., so after tile j's
// loads come tile j+1's loads and the stores of tiles j-2 and j-3.
// ---------------------------------------------------------------------------
template <int P, int TV, int VAR, int NW = 4>   // NW waves per workgroup (A/B: 2)
__global__ __launch_bounds__(64 * NW) void k_tree_lds_lag(uint16_t* __restrict__ ranks, uint64_t stride,
                                                         const uint8_t* __restrict__ order, uint64_t block_vec,
                                                         uint64_t ntiles) {
    constexpr int RPI = 64 / TV, RPW = P / NW, OPS = RPW / RPI, LPL = OPS;
    static_assert(NW == 2 || NW == 4 || NW == 8, "2, 4 or 8 waves");
    static_assert(OPS >= 1 && 3 * OPS <= 63, "vmcnt is 6 bits");
    __shared__ __attribute__((aligned(16))) uint4 buf[2][P * TV];
    __shared__ __attribute__((aligned(16))) uint4 part[2][NW * TV];
    __shared__ __attribute__((aligned(16))) uint8_t ord_lds[P * ALLRED_MAX_NODES];
    __shared__ uint32_t bar_ctr;
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
    auto store = [&](uint64_t t, uint4 res) {
#pragma unroll
        for (int k = 0; k < OPS; ++k) {
            const int r = RPW * w + RPI * k + q;
            st_nt(reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + t * TV + c, res);
        }
    };
    uint32_t bar = 0;
    auto barrier = [&]() {
        if (VAR == 1) {
            bar += NW;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) __hip_atomic_fetch_add(&bar_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            while (__hip_atomic_load(&bar_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < bar) {
            }
            asm volatile("" ::: "memory");
        } else {
            lds_barrier();
        }
    };
    const uint64_t G = gridDim.x;
    const int mine = blockIdx.x < ntiles ? (int)((ntiles - 1 - blockIdx.x) / G + 1) : 0;
    auto tile_of = [&](int j) { return blockIdx.x + (uint64_t)j * G; };
    if (VAR == 2 || VAR >= 7) {
        if (mine > 0) issue(tile_of(0), 0);
        if (mine > 1) issue(tile_of(1), 1);
    }
    if (VAR != 3)
        for (int i = threadIdx.x; i < P * ALLRED_MAX_NODES / 16; i += 64 * NW)
            reinterpret_cast<uint4*>(ord_lds)[i] = reinterpret_cast<const uint4*>(order)[i];
    if (threadIdx.x == 0) bar_ctr = 0;
    __syncthreads();
    if (VAR != 2 && VAR < 7) {
        if (mine > 0) issue(tile_of(0), 0);
        if (mine > 1) issue(tile_of(1), 1);
    }
    uint4 prev = make_uint4(0, 0, 0, 0);
    for (int j = 0; j < mine; ++j) {
        if (VAR == 7)   // after L(j): the last op of S(j-3) (interleaved with L(j)), L(j+1), S(j-2)
            wait_any((j >= 3 ? 1 : 0) + (j + 1 < mine ? OPS : 0) + (j >= 2 ? OPS : 0));
        else if (VAR == 8)   // S(k) before L(k): nothing of S(j-3) after L(j)'s last op
            wait_any((j + 1 < mine ? OPS : 0) + (j >= 2 ? OPS : 0));
        else if (VAR == 9)   // pairs L L S S: S(j-3)'s last two ops after L(j)'s last op
            wait_any((j >= 3 ? 2 : 0) + (j + 1 < mine ? OPS : 0) + (j >= 2 ? OPS : 0));
        else
            wait_units<OPS>((j + 1 < mine ? 1 : 0) + (j >= 2 ? 1 : 0) + (j >= 3 ? 1 : 0));
        barrier();   // every wave's rows of tile j are in LDS
        const uint4* tile = buf[j & 1];
        const uint64_t t = tile_of(j), v0 = t * TV;
        const uint8_t* ord = ord_lds + (block_vec ? v0 / block_vec : 0) * ALLRED_MAX_NODES + RPW * w + LPL * q;
        uint4 x[LPL];
#pragma unroll
        for (int i = 0; i < LPL; ++i) x[i] = tile[(VAR == 3 ? RPW * w + LPL * q + i : (int)ord[i]) * TV + c];
#pragma unroll
        for (int s = 1; s < LPL; s *= 2)
#pragma unroll
            for (int i = 0; i < LPL; i += 2 * s) x[i] = add8(x[i], x[i + s]);
        uint4 pw = x[0];
#pragma unroll
        for (int s = TV; s < 64; s *= 2) pw = add8(pw, shfl_xor4(pw, s));   // tree levels across lane groups
        if (q == 0) part[j & 1][w * TV + c] = pw;
        barrier();   // every wave has read tile j out of buf[j & 1]; the partials are in
        if (VAR >= 7) {   // tile j+2's loads and tile j-1's stores interleaved (7: L S, 8: S L, 9: L L S S)
            const uint64_t tl = tile_of(j + 2), ts = tile_of(j - 1);
            const uint32_t bl = wbase + (uint32_t)((j & 1) * P * TV * 16);
            auto ld = [&](int k) {
                if (j + 2 < mine)
                    lds_dma16(reinterpret_cast<const uint4*>(ranks + (uint64_t)(RPW * w + RPI * k + q) * stride) +
                                  tl * TV + c,
                              bl + (uint32_t)(RPI * k * TV * 16));
            };
            auto sv = [&](int k) {
                if (j >= 1) st_nt(reinterpret_cast<uint4*>(ranks + (uint64_t)(RPW * w + RPI * k + q) * stride) +
                                      ts * TV + c, prev);
            };
            if (VAR == 9) {
#pragma unroll
                for (int k = 0; k < OPS; k += 2) {
                    ld(k);
                    ld(k + 1);
                    sv(k);
                    sv(k + 1);
                }
            } else {
#pragma unroll
                for (int k = 0; k < OPS; ++k) {
                    if (VAR == 8) sv(k);
                    ld(k);
                    if (VAR == 7) sv(k);
                }
            }
        } else if (j + 2 < mine) {
            issue(tile_of(j + 2), j & 1);
        }
        const uint4* pp = part[j & 1];
        uint4 res;
        if (NW == 2) {
            res = add8(pp[0 * TV + c], pp[1 * TV + c]);
        } else if (NW == 4) {
            res = add8(add8(pp[0 * TV + c], pp[1 * TV + c]), add8(pp[2 * TV + c], pp[3 * TV + c]));
        } else {
            res = add8(add8(add8(pp[0 * TV + c], pp[1 * TV + c]), add8(pp[2 * TV + c], pp[3 * TV + c])),
                       add8(add8(pp[4 * TV + c], pp[5 * TV + c]), add8(pp[6 * TV + c], pp[7 * TV + c])));
        }
        if (VAR < 7 && j >= 1) store(tile_of(j - 1), prev);
        prev = res;
    }
    if (mine > 0) store(tile_of(mine - 1), prev);
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
// mem_2D one-pass through LDS: tile of 256 elements of all P ranks (32 KiB at
// P = 64); thread t owns dword t of the tile row and accumulates the P copies
// in fp32 in the reference order (owner's block first, then ranks 0..P-1),
// rounds once, and the result row is stored to every rank (1 KiB per
// wave-instruction).  128 threads: 2 waves.
// ---------------------------------------------------------------------------
template <int P>
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
        a0 += lo_f(y);
        a1 += hi_f(y);
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
// fp32 owner first, then every other rank ascending, one rounding) as a
// persistent double-buffered pipeline with the k_tree_lds_lag schedule, 64
// ranks: one thread per element of a 256-element tile, results through a
// small LDS row, each tile's 64 row stores one iteration late, behind tile
// j+2's loads.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_mem_lds_lag(uint16_t* __restrict__ ranks, uint64_t stride,
                                                        uint64_t block_vec, uint64_t ntiles) {
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
    auto tile_of = [&](int j) { return blockIdx.x + (uint64_t)j * G; };
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
        for (int r = 0; r < P; ++r) a += __uint_as_float((uint32_t)t16[r * TV * 8 + e] << 16);
        // one rounding; pairs of threads pack their two elements
        const float b = __shfl_xor(a, 1);
        if ((e & 1) == 0) reinterpret_cast<uint32_t*>(resb[j & 1])[e >> 1] = pack_rne(a, b);
        lds_barrier();   // the tile is read out of buf[j & 1]; resb[j & 1] is complete
        const uint4 res = resb[j & 1][c];
        {   // tile j+2's loads and tile j-1's stores interleaved op by op (k_tree_lds_lag VAR 7)
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
// Schedule-faithful steps: all ranks' step-k work in one launch.
// RS: ranks[r][b] += ranks[p][b] for b in recv_mask_k(r)   (in place: the
//     pair's recv masks are disjoint, so nobody reads what another writes)
// AG: ranks[r][b]  = ranks[p][b] for b in send_mask_k(r) (= recv_mask_k(p))
// grid.y = rank * blocks_per_rank + j
// ---------------------------------------------------------------------------
// k_step with one wave per (rank, block) and U vectors' loads in flight per
// lane (the default step kernel; k_step below with ALLRED_STEP_FORM=0).
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

template <bool ADD>
__global__ __launch_bounds__(kBlock) void k_step(uint16_t* __restrict__ ranks, uint64_t stride,
                                                 const int16_t* __restrict__ partner,
                                                 const int16_t* __restrict__ blocks, int blocks_per_rank,
                                                 uint64_t block_vec) {
    const int t = blockIdx.y;
    const int r = t / blocks_per_rank;
    const int p = partner[r];
    const uint64_t off = (uint64_t)blocks[t] * block_vec;
    uint4* L = reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + off;
    const uint4* R = reinterpret_cast<const uint4*>(ranks + (uint64_t)p * stride) + off;
    for (uint64_t v = gtid(); v < block_vec; v += gthreads()) st_nt(L + v, ADD ? add8(ld_nt(L + v), ld_nt(R + v)) : ld_nt(R + v));
}

// LO step (full vector): dst[r] = src[r] + src[p(r)], ping-pong buffers
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
// mem_2D: block b (owner rank b) summed over every rank's copy in fp32,
// starting from the owner's own block, then ranks 0..N-1 in order, rounded
// once (allred_mem_2D/kernels/compute_kernel.cpp:43-72 with the own-block
// seed).  WRITE_ALL: store to every rank (fused one-shot form);
// else store to `out` (the shared dst buffer, allred_mem_2D dataflow :169-174).
// ---------------------------------------------------------------------------
template <bool WRITE_ALL, int B = 8>   // B ranks' loads in flight per thread before their adds
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
                a[0] += lo_f(y[i].x); a[1] += hi_f(y[i].x);
                a[2] += lo_f(y[i].y); a[3] += hi_f(y[i].y);
                a[4] += lo_f(y[i].z); a[5] += hi_f(y[i].z);
                a[6] += lo_f(y[i].w); a[7] += hi_f(y[i].w);
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
// Peer-mapped one-shot allreduce (allred_mem_2D over xGMI): every GPU's window
// is IPC-mapped into every other GPU; flags live in fine-grained (uncached)
// memory and are written / polled with system-scope atomics.  Kernel
// boundaries on the stream carry the system-scope release / acquire of the
// window bytes (HIP dispatch packets fence at system scope).
// ---------------------------------------------------------------------------
// bounded waits: 2^22 polls of an uncached word (~1 us each) ~ 4 s, far above
// any legitimate skew between ranks, short enough that a broken peer set
// degrades to a status bit within seconds per wait instead of hanging
constexpr uint64_t kPeerSpinLimit = 1ull << 22;

struct PeerPtrs {
    uint16_t* win[ALLRED_MAX_NODES];     // window of rank q (this parity), as mapped here
    uint32_t* flags[ALLRED_MAX_NODES];   // flag array of rank q, as mapped here
};

// one workgroup: tell every peer "rank `me` reached `epoch`", then wait for all.
// Bounded: on timeout bit 0 of *status is set and the kernel returns.
__global__ void k_peer_barrier(PeerPtrs pp, int nranks, int me, uint32_t epoch, uint32_t* status) {
    const int t = threadIdx.x;
    if (t < nranks)
        __hip_atomic_store(pp.flags[t] + me, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (t < nranks) {
        uint32_t* mine = pp.flags[me] + t;
        for (uint64_t spin = 0;; ++spin) {
            if (__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= epoch) break;
            if (spin > kPeerSpinLimit) {  // ~ seconds: a peer never arrived
                atomicOr(status, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// reduce-scatter: block `me` of every window, owner first then ranks in order
// (fp32, one rounding), written to my window (peers gather it) and to my bucket
__global__ __launch_bounds__(kBlock) void k_peer_rs(PeerPtrs pp, int nranks, int me, uint16_t* __restrict__ bucket,
                                                    uint64_t blk_vec) {
    const uint64_t off = (uint64_t)me * blk_vec;
    for (uint64_t v = gtid(); v < blk_vec; v += gthreads()) {
        const uint4 s = ld_nt(reinterpret_cast<const uint4*>(pp.win[me]) + off + v);
        float a[8] = {lo_f(s.x), hi_f(s.x), lo_f(s.y), hi_f(s.y), lo_f(s.z), hi_f(s.z), lo_f(s.w), hi_f(s.w)};
        uint4 y[ALLRED_MAX_NODES > 8 ? 8 : ALLRED_MAX_NODES];
        for (int q0 = 0; q0 < nranks; q0 += 8) {
            const int q1 = q0 + 8 < nranks ? q0 + 8 : nranks;
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (q0 + i < q1 && q0 + i != me) y[i] = ld_nt(reinterpret_cast<const uint4*>(pp.win[q0 + i]) + off + v);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (q0 + i >= q1 || q0 + i == me) continue;
                a[0] += lo_f(y[i].x); a[1] += hi_f(y[i].x);
                a[2] += lo_f(y[i].y); a[3] += hi_f(y[i].y);
                a[4] += lo_f(y[i].z); a[5] += hi_f(y[i].z);
                a[6] += lo_f(y[i].w); a[7] += hi_f(y[i].w);
            }
        }
        uint4 o;
        o.x = pack_rne(a[0], a[1]);
        o.y = pack_rne(a[2], a[3]);
        o.z = pack_rne(a[4], a[5]);
        o.w = pack_rne(a[6], a[7]);
        st_nt(reinterpret_cast<uint4*>(pp.win[me]) + off + v, o);
        st_nt(reinterpret_cast<uint4*>(bucket) + off + v, o);
    }
}

// all-gather: bucket[block q] = window_q[block q] for every q != me (grid.y = q)
__global__ __launch_bounds__(kBlock) void k_peer_ag(PeerPtrs pp, int me, uint16_t* __restrict__ bucket,
                                                    uint64_t blk_vec) {
    const int q = blockIdx.y;
    if (q == me) return;
    const uint64_t off = (uint64_t)q * blk_vec;
    for (uint64_t v = gtid(); v < blk_vec; v += gthreads())
        st_nt(reinterpret_cast<uint4*>(bucket) + off + v, ld_nt(reinterpret_cast<const uint4*>(pp.win[q]) + off + v));
}

// ---- one-kernel form (latency regime) --------------------------------------
// Workgroup g owns sub-slice g of every block and only ever synchronises with
// workgroup g of the other GPUs, so there is no grid-wide barrier:
//   1. copy sub-slice g of every block but mine to my window, signal phase 0
//   2. wait phase 0 from all ranks; reduce sub-slice g of my block (own copy
//      from the bucket, then ranks in order), write it to window + bucket,
//      signal phase 1
//   3. wait phase 1; gather sub-slice g of every other block from its owner.
// Flag slot [phase][g][q] of rank r's fused flag area is written only by
// workgroup g of rank q.  Windows and flags are uncached (MTYPE UC) device
// memory, so a store is in HBM once it is acknowledged: every wave waits for
// its stores (s_waitcnt vmcnt(0)) before the workgroup barrier, then the flag
// goes out as a system-scope store, and the poll reads memory directly (no
// L2 writeback / invalidate, which cost ~20 us at 128 KiB).  allred_peer
// only selects this form when both allocations really are uncached.
__device__ inline void peer_signal_wait(const PeerPtrs& pp, int nranks, int me, uint32_t slot_base, uint32_t epoch,
                                        uint32_t* status) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int t = threadIdx.x;
    if (t < nranks)
        __hip_atomic_store(pp.flags[t] + slot_base + me, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (t < nranks) {
        uint32_t* mine = pp.flags[me] + slot_base + t;
        for (uint64_t spin = 0;; ++spin) {
            if (__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= epoch) break;
            if (spin > kPeerSpinLimit) {
                atomicOr(status, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(kBlock) void k_peer_oneshot(PeerPtrs pp, int nranks, int me, uint16_t* __restrict__ bucket,
                                                         uint64_t blk_vec, uint64_t chunk, uint32_t epoch,
                                                         uint32_t* status) {
    const int g = blockIdx.x;
    const uint64_t lo = (uint64_t)g * chunk;
    const uint64_t hi = lo + chunk < blk_vec ? lo + chunk : blk_vec;
    const uint64_t len = hi > lo ? hi - lo : 0;
    const uint4* src = reinterpret_cast<const uint4*>(bucket);
    uint4* mywin = reinterpret_cast<uint4*>(pp.win[me]);
    // 1. my copy of every block but mine -> my window
    for (uint64_t i = threadIdx.x; i < (uint64_t)nranks * len; i += blockDim.x) {
        const uint64_t q = i / len, v = q * blk_vec + lo + i % len;
        if ((int)q != me) st_nt(mywin + v, ld_nt(src + v));
    }
    const uint32_t base0 = kPeerFusedFlagOff + (uint32_t)g * 64u;
    const uint32_t base1 = kPeerFusedFlagOff + (uint32_t)(kPeerFusedMaxGroups + g) * 64u;
    peer_signal_wait(pp, nranks, me, base0, epoch, status);
    // 2. reduce my block's sub-slice g
    const uint64_t off = (uint64_t)me * blk_vec;
    for (uint64_t v = lo + threadIdx.x; v < hi; v += blockDim.x) {
        const uint4 s = ld_nt(src + off + v);
        float a[8] = {lo_f(s.x), hi_f(s.x), lo_f(s.y), hi_f(s.y), lo_f(s.z), hi_f(s.z), lo_f(s.w), hi_f(s.w)};
        uint4 y[8];
        for (int q0 = 0; q0 < nranks; q0 += 8) {
            const int q1 = q0 + 8 < nranks ? q0 + 8 : nranks;
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (q0 + i < q1 && q0 + i != me) y[i] = ld_nt(reinterpret_cast<const uint4*>(pp.win[q0 + i]) + off + v);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (q0 + i >= q1 || q0 + i == me) continue;
                a[0] += lo_f(y[i].x); a[1] += hi_f(y[i].x);
                a[2] += lo_f(y[i].y); a[3] += hi_f(y[i].y);
                a[4] += lo_f(y[i].z); a[5] += hi_f(y[i].z);
                a[6] += lo_f(y[i].w); a[7] += hi_f(y[i].w);
            }
        }
        uint4 o;
        o.x = pack_rne(a[0], a[1]);
        o.y = pack_rne(a[2], a[3]);
        o.z = pack_rne(a[4], a[5]);
        o.w = pack_rne(a[6], a[7]);
        st_nt(mywin + off + v, o);
        st_nt(reinterpret_cast<uint4*>(bucket) + off + v, o);
    }
    peer_signal_wait(pp, nranks, me, base1, epoch, status);
    // 3. gather every other block's sub-slice g from its owner
    for (uint64_t i = threadIdx.x; i < (uint64_t)nranks * len; i += blockDim.x) {
        const uint64_t q = i / len, v = q * blk_vec + lo + i % len;
        if ((int)q != me)
            st_nt(reinterpret_cast<uint4*>(bucket) + v, ld_nt(reinterpret_cast<const uint4*>(pp.win[q]) + v));
    }
}

// ---- scheduled form: the Swing / RecDub BO or LO program over peer windows --
// The RCCL program of dist.cpp with every exchange turned into a direct read
// of the partner's IPC-mapped window: step k of rank r waits until its
// partner p has finished step k-1 (p's progress slot in r's flag area), then
// reads p's blocks straight over xGMI and adds them into its own window.
// Workgroup g = channel g % C, sub-slice g / C of every block of the channel;
// it only ever waits for workgroup g of its partners.  Progress values for a
// call are base+1 (window filled) .. base+2S (all-gather step S-2 done).
// Hazards (why no ack is needed in BO): at RS step k rank r writes only
// recv_r[k], which no partner reads at step k or later; at AG step i it writes
// send_r[i], whose only earlier reader is the same partner p_i, which has
// finished its whole reduce-scatter before it can serve AG step i.
// LO ping-pongs two halves of the window: step k reads half k&1 and writes
// half (k+1)&1, after p_{k-1} (the previous reader of that half) finished k-1.
__device__ inline void sched_signal(const PeerPtrs& pp, const PeerProg& pr, int c, int me, uint32_t slot,
                                    uint32_t value) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int t = threadIdx.x;
    if (t < pr.S)
        __hip_atomic_store(pp.flags[pr.peer[c][t]] + slot + me, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ inline void sched_wait(const PeerPtrs& pp, int me, uint32_t slot, int q0, int q1, uint32_t value,
                                  uint32_t* status) {
    const int t = threadIdx.x;
    const int q = t == 0 ? q0 : (t == 1 ? q1 : -1);
    if (q >= 0) {
        uint32_t* f = pp.flags[me] + slot + q;
        for (uint64_t spin = 0;; ++spin) {
            if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= value) break;
            if (spin > kPeerSpinLimit) {
                atomicOr(status, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(kBlock) void k_peer_sched(PeerPtrs pp, PeerProg pr, int me, uint16_t* __restrict__ bucket,
                                                       uint64_t half_vec, uint32_t base, uint32_t* status) {
    const int C = pr.C, S = pr.S, N = pr.N;
    const int g = blockIdx.x, c = g % C, Gc = gridDim.x / C, j = g / C;
    const uint32_t slot = kPeerSchedFlagOff + (uint32_t)g * 64u;
    uint4* bk = reinterpret_cast<uint4*>(bucket);
    uint4* mine = reinterpret_cast<uint4*>(pp.win[me]);
    const uint64_t cb = pr.base[c];
    const int tid = threadIdx.x;
    if (!pr.lo) {
        const uint64_t blk = pr.len[c] / N;
        const uint64_t chunk = (blk + Gc - 1) / Gc;
        const uint64_t lo = (uint64_t)j * chunk, hi = lo + chunk < blk ? lo + chunk : blk;
        for (int b = 0; b < N; ++b)
            for (uint64_t v = cb + b * blk + lo + tid; v < cb + b * blk + hi; v += kBlock) st_nt(mine + v, ld_nt(bk + v));
        sched_signal(pp, pr, c, me, slot, base + 1);
        for (int k = 0; k < S; ++k) {  // reduce-scatter
            const int p = pr.peer[c][k];
            sched_wait(pp, me, slot, p, -1, base + 1 + k, status);
            const uint4* theirs = reinterpret_cast<const uint4*>(pp.win[p]);
            const bool last = k == S - 1;
            for (uint64_t m = pr.recv[c][k]; m; m &= m - 1) {
                const int b = __builtin_ctzll(m);
                for (uint64_t v = cb + b * blk + lo + tid; v < cb + b * blk + hi; v += kBlock) {
                    const uint4 o = add8(ld_nt(mine + v), ld_nt(theirs + v));
                    st_nt(mine + v, o);
                    if (last) st_nt(bk + v, o);
                }
            }
            sched_signal(pp, pr, c, me, slot, base + 2 + k);
        }
        for (int t = 0; t < S; ++t) {  // all-gather, steps in reverse
            const int i = S - 1 - t, pos = S + t;
            const int p = pr.peer[c][i];
            sched_wait(pp, me, slot, p, -1, base + 1 + pos, status);
            const uint4* theirs = reinterpret_cast<const uint4*>(pp.win[p]);
            const bool keep = t < S - 1;  // later partners read these blocks from my window
            for (uint64_t m = pr.send[c][i]; m; m &= m - 1) {
                const int b = __builtin_ctzll(m);
                for (uint64_t v = cb + b * blk + lo + tid; v < cb + b * blk + hi; v += kBlock) {
                    const uint4 y = ld_nt(theirs + v);
                    if (keep) st_nt(mine + v, y);
                    st_nt(bk + v, y);
                }
            }
            if (keep) sched_signal(pp, pr, c, me, slot, base + 2 + pos);
        }
        return;
    }
    // LO: full exchange + add every step, two window halves
    const uint64_t L = pr.len[c];
    const uint64_t chunk = (L + Gc - 1) / Gc;
    const uint64_t lo = cb + (uint64_t)j * chunk, hi = (uint64_t)j * chunk + chunk < L ? lo + chunk : cb + L;
    for (uint64_t v = lo + tid; v < hi; v += kBlock) st_nt(mine + v, ld_nt(bk + v));
    sched_signal(pp, pr, c, me, slot, base + 1);
    for (int k = 0; k < S; ++k) {
        const int p = pr.peer[c][k];
        const bool last = k == S - 1;
        sched_wait(pp, me, slot, p, (k >= 1 && !last) ? pr.peer[c][k - 1] : -1, base + 1 + k, status);
        const uint4* a = mine + (k & 1) * half_vec;
        const uint4* b = reinterpret_cast<const uint4*>(pp.win[p]) + (k & 1) * half_vec;
        uint4* dst = last ? bk : mine + ((k + 1) & 1) * half_vec;
        for (uint64_t v = lo + tid; v < hi; v += kBlock) st_nt(dst + v, add8(ld_nt(a + v), ld_nt(b + v)));
        if (!last) sched_signal(pp, pr, c, me, slot, base + 2 + k);
    }
}

// ---- hierarchical one-kernel form: 64 local ranks per GPU -------------------
// The whole hierarchical step (local tree of the 64 virtual ranks -> mem_2D
// across the W GPUs -> broadcast back to the 64 ranks) as ONE persistent
// launch with per-tile flags, so the xGMI latency of one tile hides behind
// the HBM streaming of the others.  Tile = 256 elements (512 B per rank row);
// owner(t) = t / (tiles / W), i.e. the block ownership of allred_mem_2D, so
// the bits equal tree_reduce + allred_peer_allreduce + broadcast.
//   A (all my tiles, double-buffered LDS as k_tree_lds_pipe): partial of tile
//     t -> my window's partial region (local, uncached); flagA[t][me] -> owner.
//   R (my tiles that I own): wait flagA[t][*]; read the W partials (remote
//     loads), fp32 sum owner first then ascending, one rounding -> my result
//     region; flagB[t] -> every GPU.
//   B (all my tiles): wait flagB[t]; read the result from the owner's window;
//     store it to the 64 rank rows.
// A never waits, R waits only for A, B only for R: with the grid resident
// (2 workgroups per CU) every wait is reached and satisfied.
struct HierPtrs {
    uint16_t* win[ALLRED_MAX_NODES];   // GPU q's window, this parity: [partial n][result n]
    uint32_t* hfl[ALLRED_MAX_NODES];   // GPU q's per-tile flags: [tile][W + 1]
};

__device__ inline void hier_wait(const uint32_t* f, uint32_t epoch, uint32_t* status) {
    for (uint64_t spin = 0;; ++spin) {
        if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= epoch) return;
        if (spin > kPeerSpinLimit) {
            atomicOr(status, 1u);
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

__global__ __launch_bounds__(kBlock) void k_hier_oneshot(uint16_t* __restrict__ ranks, uint64_t stride,
                                                         const uint8_t* __restrict__ order, HierPtrs hp, int W, int me,
                                                         uint64_t n, uint64_t ntiles, uint64_t tiles_per_owner,
                                                         uint32_t epoch, uint32_t* status) {
    constexpr int P = 64, TV = 32, RPW = 16, LPL = 8, OPS = 8;
    __shared__ __attribute__((aligned(16))) uint4 buf[2][P * TV];
    __shared__ __attribute__((aligned(16))) uint4 part[4 * TV];
    __shared__ __attribute__((aligned(16))) uint8_t ord_lds[ALLRED_MAX_NODES];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane & 31, h = lane >> 5;
    if (threadIdx.x < ALLRED_MAX_NODES) ord_lds[threadIdx.x] = order[threadIdx.x];
    __syncthreads();
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
    const uint64_t G = gridDim.x, nvec = n / 8;
    const int mine = blockIdx.x < ntiles ? (int)((ntiles - 1 - blockIdx.x) / G + 1) : 0;
    const uint32_t F = (uint32_t)W + 1;
    uint4* my_partial = reinterpret_cast<uint4*>(hp.win[me]);
    uint4* my_result = my_partial + nvec;
    auto tile_of = [&](int j) { return blockIdx.x + (uint64_t)j * G; };
    auto owner_of = [&](uint64_t t) { return (int)(t / tiles_per_owner); };
    // ---- A: local trees, partials published.  Each iteration starts with
    // vmcnt(0): tile j's LDS-DMA and tile j-1's partial store are then done, so
    // tile j-1's flag goes out there, one iteration late, without draining the
    // prefetch of tile j+1 (issued after that wait).  (Interleaving R and B
    // into this loop measured slower: 22.6 vs 19.6 us at W = 1 — each
    // uncached round trip is then paid once per tile instead of once per batch.)
    auto publish = [&](uint64_t t) {
        if (threadIdx.x == 0)
            __hip_atomic_store(hp.hfl[owner_of(t)] + t * F + me, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    };
    if (mine > 0) issue(tile_of(0), 0);
    for (int j = 0; j < mine; ++j) {
        wait_vm<0>();
        lds_barrier();
        if (j > 0) publish(tile_of(j - 1));
        if (j + 1 < mine) issue(tile_of(j + 1), (j + 1) & 1);
        const uint4* tile = buf[j & 1];
        const uint64_t v0 = tile_of(j) * TV;
        const uint8_t* ord = ord_lds + RPW * w + LPL * h;
        uint4 x[LPL];
#pragma unroll
        for (int i = 0; i < LPL; ++i) x[i] = tile[(int)ord[i] * TV + c];
#pragma unroll
        for (int s2 = 1; s2 < LPL; s2 *= 2)
#pragma unroll
            for (int i = 0; i < LPL; i += 2 * s2) x[i] = add8(x[i], x[i + s2]);
        const uint4 pw = add8(x[0], shfl_xor4(x[0], 32));
        if (h == 0) part[w * TV + c] = pw;
        lds_barrier();
        if (w == 0 && h == 0)
            st_nt(my_partial + v0 + c,
                  add8(add8(part[0 * TV + c], part[1 * TV + c]), add8(part[2 * TV + c], part[3 * TV + c])));
    }
    wait_vm<0>();
    if (mine > 0) publish(tile_of(mine - 1));
    // ---- R: the tiles I own, 8 at a time: every flag, then every remote load in flight at once
    {
        int owned[8];
        int no = 0;
        auto flush = [&]() {
            for (int i = threadIdx.x; i < no * W; i += kBlock)
                hier_wait(hp.hfl[me] + tile_of(owned[i / W]) * F + i % W, epoch, status);
            lds_barrier();
            const int b = threadIdx.x / TV;
            if (b < no) {
                const uint64_t v0 = tile_of(owned[b]) * TV;
                const uint4 s0 = ld_nt(my_partial + v0 + c);
                float a[8] = {lo_f(s0.x), hi_f(s0.x), lo_f(s0.y), hi_f(s0.y),
                              lo_f(s0.z), hi_f(s0.z), lo_f(s0.w), hi_f(s0.w)};
                for (int q0 = 0; q0 < W; q0 += 8) {   // 8 remote partials in flight at once
                    uint4 y[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        if (q0 + i < W && q0 + i != me) y[i] = ld_nt(reinterpret_cast<const uint4*>(hp.win[q0 + i]) + v0 + c);
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        if (q0 + i >= W || q0 + i == me) continue;
                        a[0] += lo_f(y[i].x); a[1] += hi_f(y[i].x);
                        a[2] += lo_f(y[i].y); a[3] += hi_f(y[i].y);
                        a[4] += lo_f(y[i].z); a[5] += hi_f(y[i].z);
                        a[6] += lo_f(y[i].w); a[7] += hi_f(y[i].w);
                    }
                }
                uint4 o;
                o.x = pack_rne(a[0], a[1]);
                o.y = pack_rne(a[2], a[3]);
                o.z = pack_rne(a[4], a[5]);
                o.w = pack_rne(a[6], a[7]);
                st_nt(my_result + v0 + c, o);
            }
            wait_vm<0>();     // results are in HBM (uncached) before their flags
            lds_barrier();
            for (int i = threadIdx.x; i < no * W; i += kBlock)
                __hip_atomic_store(hp.hfl[i % W] + tile_of(owned[i / W]) * F + W, epoch, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            no = 0;
        };
        for (int j = 0; j < mine; ++j) {
            if (owner_of(tile_of(j)) != me) continue;
            owned[no++] = j;
            if (no == 8) flush();
        }
        if (no) flush();
    }
    // ---- B: results back to the 64 rank rows, 4 tiles' remote loads in flight at once
    constexpr int BB = 4;
    for (int j0 = 0; j0 < mine; j0 += BB) {
        const int nb = mine - j0 < BB ? mine - j0 : BB;
        if (threadIdx.x < (unsigned)nb) hier_wait(hp.hfl[me] + tile_of(j0 + (int)threadIdx.x) * F + W, epoch, status);
        lds_barrier();
        uint4 res[BB];
#pragma unroll
        for (int b = 0; b < BB; ++b) {
            if (b >= nb) break;
            const uint64_t t = tile_of(j0 + b);
            res[b] = ld_nt(reinterpret_cast<const uint4*>(hp.win[owner_of(t)]) + nvec + t * TV + c);
        }
#pragma unroll
        for (int b = 0; b < BB; ++b) {
            if (b >= nb) break;
            const uint64_t v0 = tile_of(j0 + b) * TV;
#pragma unroll
            for (int k = 0; k < OPS; ++k) {
                const int r = RPW * w + 2 * k + h;
                st_nt(reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + v0 + c, res[b]);
            }
        }
    }
}

// ---- hierarchical one-kernel form, LL (push) variant ------------------------
// Same bits as k_hier_oneshot (local tree per tile -> mem_2D across the W GPUs,
// fp32 owner first then ascending, one rounding -> every GPU's 64 rank rows),
// but every cross-GPU transfer is a PUSH of self-validating 8-byte words
// (4 bytes of data + the call's epoch, RCCL's "LL" idea): the producer's
// relaxed system-scope stores go straight into the consumer's uncached LL
// area and the consumer polls its OWN memory until every word carries the
// epoch.  No flag follows the data and no remote load is ever waited for, so
// each hand-off costs one one-way xGMI trip instead of a flag trip plus a
// remote read round trip (k_hier_oneshot: A publish -> R remote loads -> B
// remote loads).
//   A (all my tiles, double-buffered LDS): tile t's partial -> owner o's inbox
//     slot [t - o*tpo][me] (1 KiB of LL words per tile).
//   R (my tiles that I own): poll the W slots, fp32 sum owner first then
//     ascending, one rounding -> every GPU's result box [t].
//   B (all my tiles): poll my result box [t], store to the 64 rank rows.
// A never waits, R waits only for A, B only for R; the grid is resident (2
// workgroups per CU), so every wait is reached and satisfied.  Epochs grow by
// one per call and the LL areas alternate by call parity, so a word of an
// earlier call never carries the awaited epoch.
constexpr int kLLMaxGpus = 8;
struct LLPtrs {
    uint64_t* ll[kLLMaxGpus];   // GPU q's LL area, this parity: [inbox: tiles x 128 words][result box: same]
};

__device__ __forceinline__ void ll_put(uint64_t* dst, uint4 v, uint32_t e) {
    const uint64_t hi = (uint64_t)e << 32;
    __hip_atomic_store(dst + 0, hi | v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(dst + 1, hi | v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(dst + 2, hi | v.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(dst + 3, hi | v.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// poll 4 LL words until all carry epoch e (bounded: status bit 0 on timeout)
__device__ __forceinline__ uint4 ll_get(const uint64_t* src, uint32_t e, uint32_t* status) {
    uint64_t w0, w1, w2, w3;
    for (uint64_t spin = 0;; ++spin) {
        w0 = __hip_atomic_load(src + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        w1 = __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        w2 = __hip_atomic_load(src + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        w3 = __hip_atomic_load(src + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((uint32_t)(w0 >> 32) == e && (uint32_t)(w1 >> 32) == e && (uint32_t)(w2 >> 32) == e &&
            (uint32_t)(w3 >> 32) == e)
            break;
        if (spin > kPeerSpinLimit) {
            atomicOr(status, 1u);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return make_uint4((uint32_t)w0, (uint32_t)w1, (uint32_t)w2, (uint32_t)w3);
}

__global__ __launch_bounds__(kBlock) void k_hier_ll(uint16_t* __restrict__ ranks, uint64_t stride,
                                                    const uint8_t* __restrict__ order, LLPtrs lp, int W, int me,
                                                    uint64_t ntiles, uint64_t tiles_per_owner, uint64_t box_words,
                                                    uint32_t epoch, uint32_t* status) {
    constexpr int P = 64, TV = 32, RPW = 16, LPL = 8, OPS = 8;
    __shared__ __attribute__((aligned(16))) uint4 buf[2][P * TV];
    __shared__ __attribute__((aligned(16))) uint4 part[4 * TV];
    __shared__ __attribute__((aligned(16))) uint8_t ord_lds[ALLRED_MAX_NODES];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane & 31, h = lane >> 5;
    if (threadIdx.x < ALLRED_MAX_NODES) ord_lds[threadIdx.x] = order[threadIdx.x];
    __syncthreads();
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
    const uint64_t G = gridDim.x;
    const int mine = blockIdx.x < ntiles ? (int)((ntiles - 1 - blockIdx.x) / G + 1) : 0;
    auto tile_of = [&](int j) { return blockIdx.x + (uint64_t)j * G; };
    auto owner_of = [&](uint64_t t) { return (int)(t / tiles_per_owner); };
    uint64_t* const my_ll = lp.ll[me];
    // ---- A: local trees, partials pushed to their owners
    if (mine > 0) issue(tile_of(0), 0);
    for (int j = 0; j < mine; ++j) {
        // in flight after tile j's loads: wave 0's four LL stores of tile j-1
        // (wave-uniform branch: vmcnt is per wave)
        if (j > 0 && w == 0) wait_vm<4>(); else wait_vm<0>();
        lds_barrier();
        if (j + 1 < mine) issue(tile_of(j + 1), (j + 1) & 1);
        const uint4* tile = buf[j & 1];
        const uint64_t t = tile_of(j);
        const uint8_t* ord = ord_lds + RPW * w + LPL * h;
        uint4 x[LPL];
#pragma unroll
        for (int i = 0; i < LPL; ++i) x[i] = tile[(int)ord[i] * TV + c];
#pragma unroll
        for (int s2 = 1; s2 < LPL; s2 *= 2)
#pragma unroll
            for (int i = 0; i < LPL; i += 2 * s2) x[i] = add8(x[i], x[i + s2]);
        const uint4 pw = add8(x[0], shfl_xor4(x[0], 32));
        if (h == 0) part[w * TV + c] = pw;
        lds_barrier();
        if (w == 0 && h == 0) {
            const int o = owner_of(t);
            const uint4 res = add8(add8(part[0 * TV + c], part[1 * TV + c]), add8(part[2 * TV + c], part[3 * TV + c]));
            ll_put(lp.ll[o] + ((t - (uint64_t)o * tiles_per_owner) * W + me) * 128 + c * 4, res, epoch);
        }
    }
    __syncthreads();   // every wave is past A: buf may be reused below
    uint4* xs = buf[0];   // [8 GPUs][32 columns] partials, then [32] results / [4][32] B rows
    // ---- R: the tiles I own: W partials from my inbox -> every GPU's result box
    for (int j = 0; j < mine; ++j) {
        const uint64_t t = tile_of(j);
        if (owner_of(t) != me) continue;
        const uint64_t li = t - (uint64_t)me * tiles_per_owner;
        const int q = threadIdx.x >> 5;   // source GPU of this lane's slot
        if (q < W) xs[q * 32 + c] = ll_get(my_ll + (li * W + q) * 128 + c * 4, epoch, status);
        __syncthreads();
        if (threadIdx.x < 32) {
            const uint4 s0 = xs[me * 32 + c];
            float a[8] = {lo_f(s0.x), hi_f(s0.x), lo_f(s0.y), hi_f(s0.y), lo_f(s0.z), hi_f(s0.z), lo_f(s0.w), hi_f(s0.w)};
            for (int qq = 0; qq < W; ++qq) {
                if (qq == me) continue;
                const uint4 y = xs[qq * 32 + c];
                a[0] += lo_f(y.x); a[1] += hi_f(y.x);
                a[2] += lo_f(y.y); a[3] += hi_f(y.y);
                a[4] += lo_f(y.z); a[5] += hi_f(y.z);
                a[6] += lo_f(y.w); a[7] += hi_f(y.w);
            }
            uint4 o;
            o.x = pack_rne(a[0], a[1]);
            o.y = pack_rne(a[2], a[3]);
            o.z = pack_rne(a[4], a[5]);
            o.w = pack_rne(a[6], a[7]);
            xs[8 * 32 + c] = o;
        }
        __syncthreads();
        if (q < W) ll_put(lp.ll[q] + box_words + t * 128 + c * 4, xs[8 * 32 + c], epoch);
        __syncthreads();   // xs is reused by the next owned tile
    }
    // ---- B: my result box -> the 64 rank rows, 4 tiles at a time
    constexpr int BB = 4;
    for (int j0 = 0; j0 < mine; j0 += BB) {
        const int nb = mine - j0 < BB ? mine - j0 : BB;
        const int b = threadIdx.x >> 5;
        if (b < nb) xs[16 * 32 + b * 32 + c] = ll_get(my_ll + box_words + tile_of(j0 + b) * 128 + c * 4, epoch, status);
        __syncthreads();
        uint4 res[BB];
#pragma unroll
        for (int bb = 0; bb < BB; ++bb)
            if (bb < nb) res[bb] = xs[16 * 32 + bb * 32 + c];
        __syncthreads();   // xs is reused by the next batch
#pragma unroll
        for (int bb = 0; bb < BB; ++bb) {
            if (bb >= nb) break;
            const uint64_t v0 = tile_of(j0 + bb) * TV;
#pragma unroll
            for (int k = 0; k < OPS; ++k) {
                const int r = RPW * w + 2 * k + h;
                st_nt(reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + v0 + c, res[bb]);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// k_peer_mem_ll: allred_mem_2D across GPUs for small buckets with LL hand-offs
// (the flat counterpart of k_hier_ll).  A: every vector is pushed as four
// data+epoch words to its block owner's inbox; R: the owner polls the W
// copies of each of its vectors (all loads in flight at once), sums them in
// fp32 owner first then ascending, one rounding (allred_mem_2D semantics, the
// bits of k_peer_oneshot), and pushes the result into every GPU's box; B:
// every GPU polls its box and writes its bucket.  Two one-way trips, no flag,
// no remote read.  A never waits and the grid is resident (<= 128 groups), so
// every wait of R and B is reached.  LL layout of the call's parity:
// [inbox: owned vectors][W][4 words], then [box: vectors][4 words].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_peer_mem_ll(LLPtrs lp, int W, int me, uint16_t* __restrict__ bucket,
                                                        uint64_t nv, uint64_t bv, uint32_t epoch, uint32_t* status) {
    const uint64_t gt = gtid(), GT = gthreads();
    uint4* bk = reinterpret_cast<uint4*>(bucket);
    uint64_t* const my_ll = lp.ll[me];
    const uint64_t box = nv * 4;
    for (uint64_t v = gt; v < nv; v += GT) {   // A
        const int o = (int)(v / bv);
        // the owner's area by an unrolled select over the (scalar) kernarg pointers: a
        // per-lane index into lp.ll would be a vector load waiting behind every store
        uint64_t* dst = lp.ll[0];
#pragma unroll
        for (int q = 1; q < kLLMaxGpus; ++q)
            if (o == q) dst = lp.ll[q];
        ll_put(dst + ((v - (uint64_t)o * bv) * W + me) * 4, ld_nt(bk + v), epoch);
    }
    for (uint64_t u = gt; u < bv; u += GT) {   // R: my block
        const uint64_t* slots = my_ll + u * W * 4;
        uint4 y[kLLMaxGpus];
        for (uint64_t spin = 0;; ++spin) {
            uint64_t wv[kLLMaxGpus][4];
#pragma unroll
            for (int q = 0; q < kLLMaxGpus; ++q)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    wv[q][e] = q < W ? __hip_atomic_load(slots + q * 4 + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                     : (uint64_t)epoch << 32;
            uint32_t bad = 0;
#pragma unroll
            for (int q = 0; q < kLLMaxGpus; ++q) {
#pragma unroll
                for (int e = 0; e < 4; ++e) bad |= (uint32_t)(wv[q][e] >> 32) ^ epoch;
                y[q] = make_uint4((uint32_t)wv[q][0], (uint32_t)wv[q][1], (uint32_t)wv[q][2], (uint32_t)wv[q][3]);
            }
            if (bad == 0) break;
            if (spin > kPeerSpinLimit) {
                atomicOr(status, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        float a[8];
#pragma unroll
        for (int q = 0; q < kLLMaxGpus; ++q) {
            if (q != me) continue;
            a[0] = lo_f(y[q].x); a[1] = hi_f(y[q].x); a[2] = lo_f(y[q].y); a[3] = hi_f(y[q].y);
            a[4] = lo_f(y[q].z); a[5] = hi_f(y[q].z); a[6] = lo_f(y[q].w); a[7] = hi_f(y[q].w);
        }
#pragma unroll
        for (int q = 0; q < kLLMaxGpus; ++q) {
            if (q >= W || q == me) continue;
            a[0] += lo_f(y[q].x); a[1] += hi_f(y[q].x);
            a[2] += lo_f(y[q].y); a[3] += hi_f(y[q].y);
            a[4] += lo_f(y[q].z); a[5] += hi_f(y[q].z);
            a[6] += lo_f(y[q].w); a[7] += hi_f(y[q].w);
        }
        const uint4 r = make_uint4(pack_rne(a[0], a[1]), pack_rne(a[2], a[3]), pack_rne(a[4], a[5]), pack_rne(a[6], a[7]));
        const uint64_t v = (uint64_t)me * bv + u;
        for (int q = 0; q < W; ++q) ll_put(lp.ll[q] + box + v * 4, r, epoch);
    }
    for (uint64_t v = gt; v < nv; v += GT) st_nt(bk + v, ll_get(my_ll + box + v * 4, epoch, status));   // B
}

// ---------------------------------------------------------------------------
// k_peer_lo_ll: the LO program of allred_peer_dist_allreduce (one channel)
// for small buckets with LL hand-offs: step k, every lane pushes its 16 bytes
// as four self-validating 8-byte words (4 data bytes + the call's epoch) into
// partner p_k's step-k slot, then polls its OWN step-k slot until the four
// words of p_k carry the epoch, and adds (one bf16 rounding, the same add as
// every LO form).  Per step one one-way xGMI trip instead of k_peer_sched's
// progress flag + remote read round trip; no window, no flag area.  Slots
// [step][vector][4 words] in the LL area of the call's parity; call k+2 may
// reuse a parity because finishing call k+1 needs every rank to have started
// it (the partners of all steps reach every rank of the schedule).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_peer_lo_ll(LLPtrs lp, PeerProg pr, int me, uint16_t* __restrict__ bucket,
                                                       uint64_t nv, uint32_t epoch, uint32_t* status) {
    const uint64_t v = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (v >= nv) return;
    uint4* bk = reinterpret_cast<uint4*>(bucket);
    uint4 cur = ld_nt(bk + v);
    const uint64_t* mine = lp.ll[me];
    for (int k = 0; k < pr.S; ++k) {
        const int p = pr.peer[0][k];
        ll_put(lp.ll[p] + ((uint64_t)k * nv + v) * 4, cur, epoch);
        cur = add8(cur, ll_get(mine + ((uint64_t)k * nv + v) * 4, epoch, status));
    }
    st_nt(bk + v, cur);
}

// ---------------------------------------------------------------------------
// k_hier_ws: the k_hier_ll step (same bits) with the local pass and the
// cross-GPU hand-offs pipelined per tile on specialised waves.  k_hier_ll
// runs its phases one after the other (all reads, then all writes), so HBM
// reads and writes never overlap; here they do, as in the one-GPU pass.
//   waves 0-3 (data): the double-buffered LDS tree of k_tree_lds_pipe with
//     early release.  Iteration j: wait for tile j's loads, tree -> partial
//     in LDS, issue tile j+2's loads into tile j's buffer, then store tile
//     j-1's result to the 64 rank rows, behind the loads in flight.  Their
//     only waits are exact vmcnt counts of their own loads and LDS counters.
//   wave 4 (pusher): stores only, never waits on memory.  Sums tile j's four
//     wave partials and pushes it to the owner's inbox (its own partial, when
//     this GPU owns tile j, goes to the poller through LDS); pushes the result
//     of every tile this GPU owns to the other GPUs' boxes.  It serves
//     whichever is ready first, so a slow result never holds a partial back.
//   wave 5 (poller): loads only, so each poll costs one load latency and never
//     waits for a store's acknowledgement.  Owned tile: the W-1 other partials
//     from the inbox + its own from LDS, fp32 owner first then ascending, one
//     rounding; other tiles: the result from this GPU's box.  -> LDS.
// Waves talk through monotonic LDS counters instead of s_barrier, so a
// polling wave never holds the others at a barrier.  Deadlock-free with a
// resident grid: workgroup g runs the same tile sequence on every GPU; the
// data waves publish tile j's partial before they wait for tile j-1's
// result, and a tile-j hand-off needs nothing of a later tile anywhere.
// Same LL layout, epochs and parities as k_hier_ll.  With W = 1 every tile
// is owned and nothing leaves LDS.
// ---------------------------------------------------------------------------
constexpr int kWsBlock = 384;   // 4 data waves, the pusher, the poller

// ALLRED_WS_TRACE (tools/ubench only): per-workgroup s_memrealtime stamps (100 MHz)
// kept in LDS (an extra store would upset the data waves' exact vmcnt counts)
// and written out by each wave at its end: [0] start, [1+j] tile j's loads
// landed, [4+j] tile j's result seen by the data waves, [7] data end, [8+j]
// result j in LDS (poller), [11+j] partial j pushed (pusher), 3 tiles at most.
#ifdef ALLRED_WS_TRACE
__device__ uint64_t g_ws_trace[1024 * 16];
#define WS_MARK(slot)                                                        \
    do {                                                                     \
        if ((slot) < 16 && lane == 0) ws_tr[slot] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#define WS_FLUSH(lo, hi)                                                     \
    do {                                                                     \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                  \
        if (lane >= (lo) && lane < (hi)) g_ws_trace[blockIdx.x * 16 + lane] = ws_tr[lane]; \
    } while (0)
#else
#define WS_MARK(slot) do { } while (0)
#define WS_FLUSH(lo, hi) do { } while (0)
#endif

#ifndef ALLRED_WS_NAP
#define ALLRED_WS_NAP 1   // s_sleep argument of the waves' LDS waits (64-clock units; A/B knob)
#endif
__device__ __forceinline__ void ws_nap() {
    if (ALLRED_WS_NAP > 0) __builtin_amdgcn_s_sleep(ALLRED_WS_NAP);
}
__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// spin until *p >= target (LDS; wave-uniform), then keep later LDS reads behind it.
// Bounded like every peer wait: a counter that never arrives (a bug) sets status
// bit 0 and lets the wave run to the end instead of hanging the GPU.
__device__ __forceinline__ void lds_wait_ge(const uint32_t* p, uint32_t target, bool nap, uint32_t* status) {
    for (uint64_t spin = 0; lds_ld(p) < target; ++spin) {
        if (spin > kPeerSpinLimit) {
            atomicOr(status, 1u);
            break;
        }
        if (nap) ws_nap();
    }
    asm volatile("" ::: "memory");
}
// publish: this wave's earlier LDS accesses complete, then one lane bumps / sets the counter
__device__ __forceinline__ void lds_signal_add(uint32_t* p, int lane) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_signal_set(uint32_t* p, uint32_t v, int lane) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// MODE (A/B diagnostics, tools/ubench/ws_trace.hip; W = 1 only for 1 and 2):
// 0 the product; 1 the data waves alone, storing tile j from the four wave
// partials in iteration j; 2 the same with the stores one iteration late.
template <int MODE = 0>
__global__ __launch_bounds__(kWsBlock) void k_hier_ws(uint16_t* __restrict__ ranks, uint64_t stride,
                                                      const uint8_t* __restrict__ order, LLPtrs lp, int W, int me,
                                                      uint64_t ntiles, uint64_t tiles_per_owner, uint64_t box_words,
                                                      uint32_t epoch, uint32_t* status) {
    constexpr int P = 64, TV = 32, RPW = 16, LPL = 8, OPS = 8;
    enum { kBar = 0, kPartReady, kPartFree, kOwnReady, kOwnFree, kResReady, kResFree, kPushDone, kCtrs };
    __shared__ __attribute__((aligned(16))) uint4 buf[2][P * TV];
    __shared__ __attribute__((aligned(16))) uint4 part[2][4 * TV];
    __shared__ __attribute__((aligned(16))) uint4 ownp[2][TV];
    __shared__ __attribute__((aligned(16))) uint4 resb[2][TV];
    __shared__ __attribute__((aligned(16))) uint8_t ord_lds[ALLRED_MAX_NODES];
    __shared__ uint32_t ctr[kCtrs];
#ifdef ALLRED_WS_TRACE
    __shared__ uint64_t ws_tr[16];
#endif
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane & 31, h = lane >> 5;
    if (threadIdx.x < ALLRED_MAX_NODES) ord_lds[threadIdx.x] = order[threadIdx.x];
    if (threadIdx.x < kCtrs) ctr[threadIdx.x] = 0;
    __syncthreads();   // the only s_barrier: from here on the waves sync through ctr[]
    if (w == 0) WS_MARK(0);
    const uint64_t G = gridDim.x;
    const int mine = blockIdx.x < ntiles ? (int)((ntiles - 1 - blockIdx.x) / G + 1) : 0;
    auto tile_of = [&](int j) { return blockIdx.x + (uint64_t)j * G; };
    auto owner_of = [&](uint64_t t) { return (int)(t / tiles_per_owner); };
    if (w < 4) {
        // ---------------- data waves
#ifdef ALLRED_WS_PRIO
        __builtin_amdgcn_s_setprio(ALLRED_WS_PRIO);   // A/B: issue priority over the helper waves
#endif
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
        auto store_result = [&](int j) {   // tile j's result (poller) -> my 16 rank rows
            lds_wait_ge(&ctr[kResReady], (uint32_t)j + 1u, true, status);
            if (w == 0 && j < 3) WS_MARK(4 + j);
            const uint4 res = resb[j & 1][c];
            lds_signal_add(&ctr[kResFree], lane);
            const uint64_t v0 = tile_of(j) * TV;
#pragma unroll
            for (int k = 0; k < OPS; ++k) {
                const int r = RPW * w + 2 * k + h;
                st_nt(reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + v0 + c, res);
            }
        };
        uint32_t bar = 0;
        auto data_barrier = [&]() {   // the 4 data waves only
            bar += 4;
            lds_signal_add(&ctr[kBar], lane);
            lds_wait_ge(&ctr[kBar], bar, false, status);
        };
        auto store_rows = [&](int j, uint4 res) {
            const uint64_t v0 = tile_of(j) * TV;
#pragma unroll
            for (int k = 0; k < OPS; ++k) {
                const int r = RPW * w + 2 * k + h;
                st_nt(reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + v0 + c, res);
            }
        };
        uint4 res_prev = make_uint4(0, 0, 0, 0);
        if (mine > 0) issue(tile_of(0), 0);
        if (mine > 1) issue(tile_of(1), 1);
        for (int j = 0; j < mine; ++j) {
            // issued after tile j's loads: tile j+1's loads, and the stores of
            // tiles j-2 and j-3 (issue order L0 L1 | L2 | L3 S0 | L4 S1 | ...)
            if (MODE == 1)   // L0 L1 | L2 S0 | L3 S1 | ...
                wait_units<OPS>((j + 1 < mine ? 1 : 0) + (j >= 1 ? 1 : 0) + (j >= 2 ? 1 : 0));
            else
                wait_units<OPS>((j + 1 < mine ? 1 : 0) + (j >= 2 ? 1 : 0) + (j >= 3 ? 1 : 0));
            data_barrier();   // every wave's rows of tile j are in LDS
            if (w == 0 && j < 3) WS_MARK(1 + j);
            const uint4* tile = buf[j & 1];
            const uint8_t* ord = ord_lds + RPW * w + LPL * h;
            uint4 x[LPL];
#pragma unroll
            for (int i = 0; i < LPL; ++i) x[i] = tile[(int)ord[i] * TV + c];
#pragma unroll
            for (int s2 = 1; s2 < LPL; s2 *= 2)
#pragma unroll
                for (int i = 0; i < LPL; i += 2 * s2) x[i] = add8(x[i], x[i + s2]);
            const uint4 pw = add8(x[0], shfl_xor4(x[0], 32));
            if (MODE == 0 && j >= 2) lds_wait_ge(&ctr[kPartFree], (uint32_t)j - 1u, true, status);   // pusher took partial j-2
            if (h == 0) part[j & 1][w * TV + c] = pw;
            lds_signal_add(&ctr[kPartReady], lane);
            data_barrier();   // every wave has read tile j out of buf[j & 1]
            if (j + 2 < mine) issue(tile_of(j + 2), j & 1);
            if (MODE == 0) {
                if (j >= 1) store_result(j - 1);
            } else {
                const uint4* pp = part[j & 1];
                const uint4 res = add8(add8(pp[0 * TV + c], pp[1 * TV + c]), add8(pp[2 * TV + c], pp[3 * TV + c]));
                if (MODE == 1) store_rows(j, res);
                if (MODE >= 2 && j >= 1) store_rows(j - 1, res_prev);
                res_prev = res;
            }
        }
        if (MODE == 0 && mine > 0) store_result(mine - 1);
        if (MODE >= 2 && mine > 0) store_rows(mine - 1, res_prev);
        if (MODE >= 3) lds_signal_add(&ctr[kPushDone], lane);   // (5: nobody waits for it)
        if (MODE == 4) asm volatile("s_wakeup" ::: "memory");
        if (w == 0) {
            WS_MARK(7);
            WS_FLUSH(0, 8);
        }
        return;
    }
    if (MODE == 3) {   // the two extra waves only spin on LDS until the data waves are done
        lds_wait_ge(&ctr[kPushDone], 4u, true, status);
        return;
    }
    if (MODE == 6) {   // the helpers sleep without touching LDS, then leave
#ifndef ALLRED_WS_SLEEPS
#define ALLRED_WS_SLEEPS 110
#endif
#ifdef ALLRED_WS_NOPS
        for (int i = 0; i < ALLRED_WS_NOPS; ++i) asm volatile("s_nop 7");   // busy, not asleep
#else
        for (int i = 0; i < ALLRED_WS_SLEEPS; ++i) __builtin_amdgcn_s_sleep(1);
#endif
        return;
    }
    if (MODE == 5) {   // 3, but the helpers leave once tile 0's partial is published (alive ~1/3 of the kernel)
        lds_wait_ge(&ctr[kPartReady], 4u, true, status);
        return;
    }
    if (MODE == 4) {   // the same, sleeping 127 x 64 clocks per check, woken by the data waves' s_wakeup
        for (uint64_t spin = 0; lds_ld(&ctr[kPushDone]) < 4u && spin < kPeerSpinLimit; ++spin)
            __builtin_amdgcn_s_sleep(127);
        return;
    }
    if (MODE != 0) return;
    if (w == 4) {
        // ---------------- pusher: partials to owners, owned results to every other GPU
        uint64_t* box[4];   // lane (h, c) serves GPUs 4h .. 4h+3 (loaded once: a per-lane
                            // kernarg index is a vector load, and its wait would take every store)
#pragma unroll
        for (int k = 0; k < 4; ++k) box[k] = 4 * h + k < W ? lp.ll[4 * h + k] + box_words : nullptr;
        int jp = 0, jr = 0;
        for (uint64_t idle = 0; jr < mine;) {
            bool moved = false;
            if (jp < mine && lds_ld(&ctr[kPartReady]) >= 4u * (uint32_t)(jp + 1)) {
                const uint64_t t = tile_of(jp);
                const int o = owner_of(t);
                if (o != me || jp < 2 || lds_ld(&ctr[kOwnFree]) >= (uint32_t)jp - 1u) {
                    asm volatile("" ::: "memory");
                    const uint4* pp = part[jp & 1];
                    const uint4 pv =
                        add8(add8(pp[0 * TV + c], pp[1 * TV + c]), add8(pp[2 * TV + c], pp[3 * TV + c]));
                    if (o == me) {
                        if (h == 0) ownp[jp & 1][c] = pv;
                    } else if (h == 0) {
                        ll_put(lp.ll[o] + ((t - (uint64_t)o * tiles_per_owner) * W + me) * 128 + c * 4, pv, epoch);
                    }
                    lds_signal_set(&ctr[kPartFree], (uint32_t)jp + 1u, lane);
                    lds_signal_set(&ctr[kOwnReady], (uint32_t)jp + 1u, lane);
                    if (jp < 3) WS_MARK(11 + jp);
                    ++jp;
                    moved = true;
                }
            }
            if (jr < jp) {
                const uint64_t t = tile_of(jr);
                if (owner_of(t) != me) {
                    lds_signal_set(&ctr[kPushDone], (uint32_t)jr + 1u, lane);
                    ++jr;
                    moved = true;
                } else if (lds_ld(&ctr[kResReady]) >= (uint32_t)jr + 1u) {
                    asm volatile("" ::: "memory");
                    const uint4 r = resb[jr & 1][c];
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (4 * h + k < W && 4 * h + k != me) ll_put(box[k] + t * 128 + c * 4, r, epoch);
                    lds_signal_set(&ctr[kPushDone], (uint32_t)jr + 1u, lane);
                    ++jr;
                    moved = true;
                }
            }
            if (moved) {
                idle = 0;
            } else if (++idle > kPeerSpinLimit) {   // bounded like every wait (status bit 0)
                atomicOr(status, 1u);
                break;
            } else {
                ws_nap();
            }
        }
        WS_FLUSH(11, 14);
        return;
    }
    // ---------------- poller (wave 5)
    uint64_t* const my_ll = lp.ll[me];
    for (int j = 0; j < mine; ++j) {
        const uint64_t t = tile_of(j);
        uint4 r;
        if (owner_of(t) == me) {
            // lane (h, c) polls the slots of GPUs 4h .. 4h+3 except its own at once
            const uint64_t* inbox = my_ll + (t - (uint64_t)me * tiles_per_owner) * W * 128 + c * 4;
            uint4 y[4];
            for (uint64_t spin = 0;; ++spin) {
                uint64_t v[4][4];
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        v[k][e] = (4 * h + k < W && 4 * h + k != me)
                                      ? __hip_atomic_load(inbox + (4 * h + k) * 128 + e, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_SYSTEM)
                                      : (uint64_t)epoch << 32;
                uint32_t bad = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) bad |= (uint32_t)(v[k][e] >> 32) ^ epoch;
                    y[k] = make_uint4((uint32_t)v[k][0], (uint32_t)v[k][1], (uint32_t)v[k][2], (uint32_t)v[k][3]);
                }
                if (bad == 0) break;
                if (spin > kPeerSpinLimit) {
                    atomicOr(status, 1u);
                    break;
                }
                ws_nap();
            }
            if (j == 0) WS_MARK(14);
            lds_wait_ge(&ctr[kOwnReady], (uint32_t)j + 1u, true, status);
            if (j == 0) WS_MARK(15);
            const uint4 own = ownp[j & 1][c];
            lds_signal_set(&ctr[kOwnFree], (uint32_t)j + 1u, lane);
            uint4 yo[4];   // the other half's slots
#pragma unroll
            for (int k = 0; k < 4; ++k) yo[k] = shfl_xor4(y[k], 32);
            auto slot = [&](int q) { return q == me ? own : ((q >> 2) == h) ? y[q & 3] : yo[q & 3]; };
            float a[8] = {lo_f(own.x), hi_f(own.x), lo_f(own.y), hi_f(own.y),
                          lo_f(own.z), hi_f(own.z), lo_f(own.w), hi_f(own.w)};
#pragma unroll
            for (int q = 0; q < kLLMaxGpus; ++q) {
                if (q >= W || q == me) continue;
                const uint4 yq = slot(q);
                a[0] += lo_f(yq.x); a[1] += hi_f(yq.x);
                a[2] += lo_f(yq.y); a[3] += hi_f(yq.y);
                a[4] += lo_f(yq.z); a[5] += hi_f(yq.z);
                a[6] += lo_f(yq.w); a[7] += hi_f(yq.w);
            }
            r = make_uint4(pack_rne(a[0], a[1]), pack_rne(a[2], a[3]), pack_rne(a[4], a[5]), pack_rne(a[6], a[7]));
        } else {
            r = ll_get(my_ll + box_words + t * 128 + c * 4, epoch, status);
            lds_signal_set(&ctr[kOwnFree], (uint32_t)j + 1u, lane);   // in tile order, owned or not
        }
        if (j >= 2) {   // slot j & 1 free: the data waves and the pusher are done with tile j-2
            lds_wait_ge(&ctr[kResFree], 4u * (uint32_t)(j - 1), true, status);
            lds_wait_ge(&ctr[kPushDone], (uint32_t)j - 1u, true, status);
        }
        if (h == 0) resb[j & 1][c] = r;
        lds_signal_set(&ctr[kResReady], (uint32_t)j + 1u, lane);
        if (j < 3) WS_MARK(8 + j);
    }
    WS_FLUSH(8, 11);
    WS_FLUSH(14, 16);
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// ALLRED_TREE=registers selects the register-only k_tree for the fused BO pass
// (A/B and fallback); the LDS-staged k_tree_lds is the default.
bool tree_force_registers() {
    static const bool v = [] {
        const char* e = std::getenv("ALLRED_TREE");
        return e && e[0] == 'r';
    }();
    return v;
}

// ALLRED_TREE=pipe forces the persistent double-buffered forms on device
// memory for every shape, ALLRED_TREE=lds the one-tile-per-workgroup forms (A/B)
bool tree_force_pipe() {
    static const bool v = [] {
        const char* e = std::getenv("ALLRED_TREE");
        return e && e[0] == 'p';
    }();
    return v;
}

bool tree_force_lds() {
    static const bool v = [] {
        const char* e = std::getenv("ALLRED_TREE");
        return e && e[0] == 'l';
    }();
    return v;
}

// early-release pipelined tree forms (default; ALLRED_PIPE_REL=0 selects the
// plain double-buffered form, 3 / 4 the one-workgroup-per-CU 3 / 4 buffer forms: A/B)
int pipe_rel() {
    static const int v = [] {
        const char* e = std::getenv("ALLRED_PIPE_REL");
        return e ? std::atoi(e) : 1;
    }();
    return v;
}

// ALLRED_PIPE_LAG=0 selects the round-1 k_tree_lds_pipe (stores in the tile's own
// iteration) for the fused BO pass on HBM; default: k_tree_lds_lag (A/B)
bool pipe_lag() {
    static const bool v = [] {
        const char* e = std::getenv("ALLRED_PIPE_LAG");
        return !(e && e[0] == '0');
    }();
    return v;
}

int last_error() { return hip_status((int)hipGetLastError()); }

template <bool WRITE_ALL>
int tree_dispatch(uint16_t* ranks, uint64_t stride, uint64_t n_vec, int total, const uint8_t* order,
                  uint64_t block_vec, uint16_t* out, hipStream_t st) {
    // hierarchical partial of 64 ranks, >= 1024 tiles: the persistent
    // double-buffered form (2 workgroups per CU), as the fused pass
    if (!WRITE_ALL && total == 64 && n_vec % 32 == 0 && block_vec == 0 && !tree_force_lds() &&
        !tree_force_registers() && (n_vec / 32 >= 1024 || tree_force_pipe())) {
        const uint64_t tiles = n_vec / 32;
        // (the early-release form measured slower here: 10.4 vs 9.6 us, read-only stream)
        hipLaunchKernelGGL((k_tree_lds_pipe<64, 1, 32, false>), dim3((unsigned)(tiles < 512 ? tiles : 512)),
                           dim3(kBlock), 0, st, ranks, stride, order, (uint64_t)0, tiles, out);
        return last_error();
    }
    // LDS-staged form: whole 32-vector tiles inside one block (any tile when block_vec == 0)
    if (total >= 8 && n_vec % 32 == 0 && (block_vec == 0 || block_vec % 32 == 0) && (block_vec || !WRITE_ALL) &&
        !tree_force_registers()) {
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

}  // namespace

int launch_peer_allreduce(uint16_t* const* wins, uint32_t* const* flags, int nranks, int me, uint16_t* bucket,
                          size_t n, uint32_t epoch, uint32_t* status, void* stream) {
    if (n % (8 * (size_t)nranks) || !aligned16(bucket) || nranks > ALLRED_MAX_NODES) return ALLRED_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    PeerPtrs pp{};
    for (int q = 0; q < nranks; ++q) {
        pp.win[q] = wins[q];
        pp.flags[q] = flags[q];
    }
    const uint64_t nv = n / 8, bv = nv / nranks;
    // 1. my bucket -> my window (the bytes peers will read)
    hipLaunchKernelGGL(k_copy_ranks, dim3(grid_all(nv), 1), dim3(kBlock), 0, st, bucket, 0, wins[me], 0, nv);
    // 2. everyone's window is written
    hipLaunchKernelGGL(k_peer_barrier, dim3(1), dim3(64), 0, st, pp, nranks, me, epoch, status);
    // 3. reduce my block from every window
    hipLaunchKernelGGL(k_peer_rs, dim3(grid_all(bv)), dim3(kBlock), 0, st, pp, nranks, me, bucket, bv);
    // 4. every block is reduced
    hipLaunchKernelGGL(k_peer_barrier, dim3(1), dim3(64), 0, st, pp, nranks, me, epoch + 1, status);
    // 5. gather the other blocks
    hipLaunchKernelGGL(k_peer_ag, dim3(grid_all(bv), nranks), dim3(kBlock), 0, st, pp, me, bucket, bv);
    return last_error();
}

int launch_peer_barrier(uint32_t* const* flags, int nranks, int me, uint32_t epoch, uint32_t* status, void* stream) {
    if (nranks > ALLRED_MAX_NODES) return ALLRED_ERR_ARG;
    PeerPtrs pp{};
    for (int q = 0; q < nranks; ++q) pp.flags[q] = flags[q];
    hipLaunchKernelGGL(k_peer_barrier, dim3(1), dim3(64), 0, (hipStream_t)stream, pp, nranks, me, epoch, status);
    return last_error();
}

int launch_peer_sched(uint16_t* const* wins, uint32_t* const* flags, int me, uint16_t* bucket, const PeerProg& prog,
                      uint64_t half_vec, uint32_t base_epoch, uint32_t* status, void* stream) {
    if (!aligned16(bucket) || prog.N > ALLRED_MAX_NODES || prog.C < 1 || prog.C > kPeerMaxChannels ||
        prog.S > kPeerMaxSteps)
        return ALLRED_ERR_ARG;
    PeerPtrs pp{};
    for (int q = 0; q < prog.N; ++q) {
        pp.win[q] = wins[q];
        pp.flags[q] = flags[q];
    }
    uint64_t per = 0;  // vectors per workgroup sub-slice unit (largest channel)
    for (int c = 0; c < prog.C; ++c) {
        const uint64_t u = prog.lo ? prog.len[c] : prog.len[c] / prog.N;
        if (u > per) per = u;
    }
    uint64_t gc = (per + kBlock - 1) / kBlock;
    const uint64_t gmax = kPeerSchedMaxGroups / prog.C;
    if (gc > gmax) gc = gmax;
    if (gc < 1) gc = 1;
    hipLaunchKernelGGL(k_peer_sched, dim3((unsigned)(gc * prog.C)), dim3(kBlock), 0, (hipStream_t)stream, pp, prog, me,
                       bucket, half_vec, base_epoch, status);
    return last_error();
}

int launch_peer_mem_ll(uint64_t* const* ll, int nranks, int me, uint16_t* bucket, size_t n, uint64_t area_words,
                       uint32_t epoch, uint32_t* status, unsigned max_groups, void* stream) {
    const uint64_t nv = n / 8;
    if (n % (8 * (size_t)nranks) || !aligned16(bucket) || nranks > kLLMaxGpus || 8 * nv > area_words)
        return ALLRED_ERR_ARG;
    LLPtrs lp{};
    for (int q = 0; q < nranks; ++q) lp.ll[q] = ll[q];
    uint64_t groups = (nv + kBlock - 1) / kBlock;
    const uint64_t cap = max_groups && max_groups < kPeerFusedMaxGroups ? max_groups : kPeerFusedMaxGroups;
    if (groups > cap) groups = cap;   // resident: every wait is reached
    hipLaunchKernelGGL(k_peer_mem_ll, dim3((unsigned)groups), dim3(kBlock), 0, (hipStream_t)stream, lp, nranks, me,
                       bucket, nv, nv / nranks, epoch, status);
    return last_error();
}

int launch_peer_lo_ll(uint64_t* const* ll, int nranks, int me, uint16_t* bucket, const PeerProg& prog, size_t n,
                      uint64_t area_words, uint32_t epoch, uint32_t* status, void* stream) {
    const uint64_t nv = n / 8;
    if (n % 8 || !aligned16(bucket) || nranks > kLLMaxGpus || !prog.lo || prog.C != 1 ||
        nv * 4 * (uint64_t)prog.S > area_words)
        return ALLRED_ERR_ARG;
    LLPtrs lp{};
    for (int q = 0; q < nranks; ++q) lp.ll[q] = ll[q];
    hipLaunchKernelGGL(k_peer_lo_ll, dim3((unsigned)((nv + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       (hipStream_t)stream, lp, prog, me, bucket, nv, epoch, status);
    return last_error();
}

int launch_hier_oneshot(uint16_t* ranks, uint64_t stride, const uint8_t* order, uint16_t* const* wins,
                        uint32_t* const* hflags, int nranks, int me, size_t n, uint32_t epoch, uint32_t* status,
                        unsigned max_grid, void* stream) {
    const uint64_t nv = n / 8, ntiles = nv / 32;
    if (nranks < 1 || nranks > ALLRED_MAX_NODES || nv % 32 || ntiles % nranks || stride % 8 || !aligned16(ranks))
        return ALLRED_ERR_ARG;
    HierPtrs hp{};
    for (int q = 0; q < nranks; ++q) {
        hp.win[q] = wins[q];
        hp.hfl[q] = hflags[q];
    }
    // 2 per CU: the whole grid resident (max_grid < 512 when processes share the GPU)
    const unsigned cap = max_grid && max_grid < 512 ? max_grid : 512;
    const unsigned grid = (unsigned)(ntiles < cap ? ntiles : cap);
    hipLaunchKernelGGL(k_hier_oneshot, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, ranks, stride, order, hp,
                       nranks, me, (uint64_t)n, ntiles, ntiles / nranks, epoch, status);
    return last_error();
}

int launch_hier_ll(uint16_t* ranks, uint64_t stride, const uint8_t* order, uint64_t* const* ll, int nranks, int me,
                   size_t n, uint64_t box_words, uint32_t epoch, uint32_t* status, unsigned max_grid,
                   void* stream) {
    const uint64_t nv = n / 8, ntiles = nv / 32;
    if (nranks < 1 || nranks > kLLMaxGpus || nv % 32 || ntiles % nranks || stride % 8 || !aligned16(ranks) ||
        ntiles * 128 > box_words)
        return ALLRED_ERR_ARG;
    LLPtrs lp{};
    for (int q = 0; q < nranks; ++q) lp.ll[q] = ll[q];
    // 2 per CU: the whole grid resident (max_grid < 512 when processes share the GPU)
    const unsigned cap = max_grid && max_grid < 512 ? max_grid : 512;
    const unsigned grid = (unsigned)(ntiles < cap ? ntiles : cap);
    hipLaunchKernelGGL(k_hier_ll, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, ranks, stride, order, lp, nranks,
                       me, ntiles, ntiles / nranks, box_words, epoch, status);
    return last_error();
}

int launch_hier_ws(uint16_t* ranks, uint64_t stride, const uint8_t* order, uint64_t* const* ll, int nranks, int me,
                   size_t n, uint64_t box_words, uint32_t epoch, uint32_t* status, unsigned max_grid,
                   void* stream) {
    const uint64_t nv = n / 8, ntiles = nv / 32;
    if (nranks < 1 || nranks > kLLMaxGpus || nv % 32 || ntiles % nranks || stride % 8 || !aligned16(ranks) ||
        ntiles * 128 > box_words)
        return ALLRED_ERR_ARG;
    LLPtrs lp{};
    for (int q = 0; q < nranks; ++q) lp.ll[q] = ll[q];
    // 2 per CU (70 KiB of LDS each): the whole grid resident
    const unsigned cap = max_grid && max_grid < 512 ? max_grid : 512;
    const unsigned grid = (unsigned)(ntiles < cap ? ntiles : cap);
    hipLaunchKernelGGL(k_hier_ws<0>, dim3(grid), dim3(kWsBlock), 0, (hipStream_t)stream, ranks, stride, order, lp, nranks,
                       me, ntiles, ntiles / nranks, box_words, epoch, status);
    return last_error();
}

int launch_peer_oneshot(uint16_t* const* wins, uint32_t* const* flags, int nranks, int me, uint16_t* bucket,
                        size_t n, uint32_t epoch, uint32_t* status, void* stream) {
    if (n % (8 * (size_t)nranks) || !aligned16(bucket) || nranks > ALLRED_MAX_NODES) return ALLRED_ERR_ARG;
    PeerPtrs pp{};
    for (int q = 0; q < nranks; ++q) {
        pp.win[q] = wins[q];
        pp.flags[q] = flags[q];
    }
    const uint64_t bv = n / 8 / nranks;
    uint64_t groups = (bv + 63) / 64;
    if (groups > kPeerFusedMaxGroups) groups = kPeerFusedMaxGroups;
    if (groups < 1) groups = 1;
    const uint64_t chunk = (bv + groups - 1) / groups;
    hipLaunchKernelGGL(k_peer_oneshot, dim3((unsigned)groups), dim3(kBlock), 0, (hipStream_t)stream, pp, nranks, me,
                       bucket, bv, chunk, epoch, status);
    return last_error();
}

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

int launch_bf16_add_blocks(uint16_t* dst, const uint16_t* src, const uint8_t* blocks, int nblocks,
                           size_t block_elems, void* stream) {
    if (nblocks <= 0) return ALLRED_OK;
    if (nblocks > ALLRED_MAX_NODES || block_elems % 8 || !aligned16(dst) || !aligned16(src)) return ALLRED_ERR_ARG;
    BlockList list{};
    for (int i = 0; i < nblocks; ++i) list.b[i] = blocks[i];
    const uint64_t bv = block_elems / 8;
    hipLaunchKernelGGL(k_add_blocks, dim3(grid_all(bv), nblocks), dim3(kBlock), 0,
                       (hipStream_t)stream, reinterpret_cast<uint4*>(dst), reinterpret_cast<const uint4*>(src),
                       list, bv);
    return last_error();
}

int launch_tree_fused(uint16_t* ranks, uint64_t stride, size_t n, int total, const uint8_t* order, void* stream,
                      bool host_memory) {
    if (n % (8 * (size_t)total) || stride % 8 || !aligned16(ranks)) return ALLRED_ERR_ARG;
    const uint64_t nv = n / 8, bv = nv / total;
    // persistent double-buffered form: host buckets always; HBM buckets of 64
    // ranks with >= 1024 tiles (config 2: 15.2 vs 16.5 us for one tile per
    // workgroup, 2 workgroups per CU = 512, each CU 5 tiles)
    const bool pipe_hbm = total == 64 && nv / 32 >= 1024 && !tree_force_lds() && !tree_force_registers();
    if ((host_memory || pipe_hbm || tree_force_pipe()) && total >= 8 && nv % 32 == 0 && bv % 32 == 0) {
        // PCIe-bound host buckets: 32 workgroups keep both link directions busy (tools/pcie_probe.py);
        // ALLRED_PIPE_GRID / ALLRED_PIPE_DEPTH override (A/B)
        static const uint64_t cap_env = [] {
            const char* e = std::getenv("ALLRED_PIPE_GRID");
            return e ? std::strtoull(e, nullptr, 10) : 0ull;
        }();
        static const int depth = [] {
            const char* e = std::getenv("ALLRED_PIPE_DEPTH");
            return e ? std::atoi(e) : 1;
        }();
        static const int tvsel = [] {  // ALLRED_PIPE_TV=16 selects 16-vector tiles (A/B)
            const char* e = std::getenv("ALLRED_PIPE_TV");
            return e ? std::atoi(e) : 32;
        }();
        const int rel = pipe_rel();
        const int TVs = (tvsel == 16 && total >= 16 && bv % 16 == 0) ? 16 : 32;
        const uint64_t tiles = nv / TVs;
        const uint64_t cap = cap_env ? cap_env : (host_memory ? 32 : (TVs == 16 ? 1024 : 512));
        const unsigned grid = (unsigned)(tiles < cap ? tiles : cap);
        hipStream_t st = (hipStream_t)stream;
#define TSA_PIPE(PP, DD, TT) \
    hipLaunchKernelGGL((k_tree_lds_pipe<PP, DD, TT>), dim3(grid), dim3(kBlock), 0, st, ranks, stride, order, bv, tiles, nullptr)
        if (TVs == 16) {
            switch (total) {
                case 16: TSA_PIPE(16, 1, 16); break;
                case 32: TSA_PIPE(32, 1, 16); break;
                case 64: if (depth >= 2) TSA_PIPE(64, 2, 16); else TSA_PIPE(64, 1, 16); break;
                default: return ALLRED_ERR_UNSUPPORTED;
            }
        } else if (depth >= 2) {
            switch (total) {
                case 8: TSA_PIPE(8, 2, 32); break;
                case 16: TSA_PIPE(16, 2, 32); break;
                case 32: TSA_PIPE(32, 2, 32); break;
                case 64: TSA_PIPE(64, 2, 32); break;
                default: return ALLRED_ERR_UNSUPPORTED;
            }
        } else if (pipe_lag() && total == 64 && !host_memory) {
            // stores one iteration late, behind the next tile's loads (config 2:
            // 14.44 vs 15.30 us for k_tree_lds_pipe, tools/ubench/fused_ab.hip)
            hipLaunchKernelGGL((k_tree_lds_lag<64, 32, 7>), dim3(grid), dim3(kBlock), 0, st, ranks, stride, order,
                               bv, tiles);
        } else if (rel && total == 64 && !host_memory) {
            // REL: NB = rel buffers; NB >= 3 needs one workgroup per CU (grid <= 256)
            const unsigned g1 = (unsigned)(tiles < 256 ? tiles : 256);
            if (rel >= 4) hipLaunchKernelGGL((k_tree_lds_pipe<64, 3, 32, true, true>), dim3(cap_env ? grid : g1),
                                             dim3(kBlock), 0, st, ranks, stride, order, bv, tiles, nullptr);
            else if (rel == 3) hipLaunchKernelGGL((k_tree_lds_pipe<64, 2, 32, true, true>), dim3(cap_env ? grid : g1),
                                                  dim3(kBlock), 0, st, ranks, stride, order, bv, tiles, nullptr);
            else hipLaunchKernelGGL((k_tree_lds_pipe<64, 1, 32, true, true>), dim3(grid), dim3(kBlock), 0, st, ranks,
                                    stride, order, bv, tiles, nullptr);
        } else {
            switch (total) {
                case 8: TSA_PIPE(8, 1, 32); break;
                case 16: TSA_PIPE(16, 1, 32); break;
                case 32: TSA_PIPE(32, 1, 32); break;
                case 64: TSA_PIPE(64, 1, 32); break;
                default: return ALLRED_ERR_UNSUPPORTED;
            }
        }
#undef TSA_PIPE
        return last_error();
    }
    return tree_dispatch<true>(ranks, stride, nv, total, order, bv, nullptr, (hipStream_t)stream);
}

int launch_butterfly(uint16_t* ranks, uint64_t stride, size_t n, int total, const int16_t* d_partner, int steps,
                     const uint8_t* dag, void* stream) {
    if (n % 8 || stride % 8 || !aligned16(ranks)) return ALLRED_ERR_ARG;
    const uint64_t nv = n / 8;
    hipStream_t st = (hipStream_t)stream;
    // persistent pipelined form for >= 1024 tiles (640 kB: 23.9 vs 25.2-26.0 us);
    // its DAG form (dag != null) from ALLRED_BFLY_DAG_MIN tiles (default 256)
    static const uint64_t dag_min = [] {
        const char* e = std::getenv("ALLRED_BFLY_DAG_MIN");
        return e ? std::strtoull(e, nullptr, 10) : 256ull;
    }();
    const bool dag_pipe = dag && !tree_force_lds() && nv / 32 >= dag_min;
    if (total == 64 && nv % 32 == 0 && nv >= 32 &&
        (dag_pipe || (nv >= 32 * 256 && (tree_force_pipe() || (nv >= 32 * 1024 && !tree_force_lds()))))) {
        static const uint64_t cap = [] {
            const char* e = std::getenv("ALLRED_PIPE_GRID");
            return e ? std::strtoull(e, nullptr, 10) : 512ull;
        }();
        const uint64_t tiles = nv / 32;
        // (the k_tree_lds_lag schedule — stores one iteration late — measured slower
        // here: 26.6 vs 24.1 us at 640 kB; the butterfly is not bound by HBM order)
        // ALLRED_BFLY_EX=0: the register butterfly (A/B).  Measured and removed: the
        // DAG with loads two tiles ahead, final rows in a small LDS set and stores
        // interleaved with those loads, 19.0 vs 17.0 us at 640 kB (profiles/r01_lo_lag_ab.txt)
        static const bool force_bpermute = [] {
            const char* e = std::getenv("ALLRED_BFLY_EX");
            return e && std::atoi(e) == 0;
        }();
        const dim3 grid((unsigned)(tiles < cap ? tiles : cap));
        if (dag && !force_bpermute)
            hipLaunchKernelGGL(k_butterfly_lds64_pipe<4>, grid, dim3(kBlock), 0, st, ranks, stride, d_partner, steps,
                               tiles, dag);
        else
            hipLaunchKernelGGL(k_butterfly_lds64_pipe<0>, grid, dim3(kBlock), 0, st, ranks, stride, d_partner, steps,
                               tiles, nullptr);
        return last_error();
    }
    if (total == 64 && nv % 32 == 0 && nv >= 32 * 256) {  // >= 256 tiles: the LDS-staged form pays
        hipLaunchKernelGGL(k_butterfly_lds64, dim3((unsigned)(nv / 32)), dim3(kBlock), 0, st, ranks, stride, d_partner,
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

int launch_broadcast(uint16_t* ranks, uint64_t stride, size_t n, int total, const uint16_t* src, void* stream) {
    if (n % 8 || stride % 8 || !aligned16(ranks) || !aligned16(src)) return ALLRED_ERR_ARG;
    const uint64_t nv = n / 8;
    hipLaunchKernelGGL(k_broadcast, dim3(grid_all(nv), (total + 7) / 8), dim3(kBlock), 0, (hipStream_t)stream, ranks,
                       stride, total,
                       reinterpret_cast<const uint4*>(src), nv);
    return last_error();
}

static int launch_step(bool add, uint16_t* ranks, uint64_t stride, int total, const int16_t* d_partner,
                       const int16_t* d_blocks, int blocks_per_rank, size_t block_elems, void* stream) {
    if (block_elems % 8 || stride % 8 || !aligned16(ranks)) return ALLRED_ERR_ARG;
    const uint64_t bv = block_elems / 8;
    // one wave per rank block, 8 vectors' loads in flight per lane (default) vs one
    // thread per vector over a grid covering the block (ALLRED_STEP_FORM=0, A/B):
    // the 12-launch config-2 program 67.8 vs 71.7 us, 256 kB 39.9 vs 45.5, 128 kB
    // 34.0 vs 38.6 (profiles/r01_step_form_ab.txt)
    static const int form = [] {
        const char* e = std::getenv("ALLRED_STEP_FORM");
        return e ? std::atoi(e) : 1;
    }();
    if (form == 1) {
        const dim3 g((unsigned)(total * blocks_per_rank));
        if (add)
            hipLaunchKernelGGL((k_step_w<true, 8>), g, dim3(64), 0, (hipStream_t)stream, ranks, stride, d_partner,
                               d_blocks, blocks_per_rank, bv);
        else
            hipLaunchKernelGGL((k_step_w<false, 8>), g, dim3(64), 0, (hipStream_t)stream, ranks, stride, d_partner,
                               d_blocks, blocks_per_rank, bv);
        return last_error();
    }
    const unsigned gx = grid_all(bv);
    const dim3 grid(gx, (unsigned)(total * blocks_per_rank));
    if (add)
        hipLaunchKernelGGL(k_step<true>, grid, dim3(kBlock), 0, (hipStream_t)stream, ranks, stride, d_partner,
                           d_blocks, blocks_per_rank, bv);
    else
        hipLaunchKernelGGL(k_step<false>, grid, dim3(kBlock), 0, (hipStream_t)stream, ranks, stride, d_partner,
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
    const unsigned gx = grid_all(nv);
    hipLaunchKernelGGL(k_lo_step, dim3(gx, total), dim3(kBlock), 0, (hipStream_t)stream, src, src_stride, dst,
                       dst_stride, d_partner, nv);
    return last_error();
}

int launch_copy_ranks(const uint16_t* src, uint64_t src_stride, uint16_t* dst, uint64_t dst_stride, int total,
                      size_t n, void* stream) {
    if (n % 8 || src_stride % 8 || dst_stride % 8 || !aligned16(src) || !aligned16(dst)) return ALLRED_ERR_ARG;
    const uint64_t nv = n / 8;
    const unsigned gx = grid_all(nv);
    hipLaunchKernelGGL(k_copy_ranks, dim3(gx, total), dim3(kBlock), 0, (hipStream_t)stream, src, src_stride, dst,
                       dst_stride, nv);
    return last_error();
}

int launch_mem_reduce(const uint16_t* ranks, uint64_t stride, size_t n, int total, uint16_t* dst, void* stream) {
    if (n % (8 * (size_t)total) || stride % 8 || !aligned16(ranks) || !aligned16(dst)) return ALLRED_ERR_ARG;
    const uint64_t nv = n / 8;
    // one column per thread reads all `total` ranks: a 640 kB bucket has only 40,960
    // columns (160 workgroups), so bytes in flight come from loads per thread:
    // 16 (default) vs 8 ranks' loads before their adds, 256 threads: 640 kB 22.1-22.3
    // vs 22.7 us, 256 kB 15.9 vs 17.1, 128 kB 11.9 vs 13.1; one-wave workgroups
    // (640 of them, every CU busy) were slower: 29.8 us at 640 kB
    // (profiles/r01_mem_batch_ab.txt).  ALLRED_MEM_BATCH (8/16/32), ALLRED_MEM_BLOCK (A/B)
    static const int batch = [] {
        const char* e = std::getenv("ALLRED_MEM_BATCH");
        return e ? std::atoi(e) : 16;
    }();
    static const unsigned block = [] {
        const char* e = std::getenv("ALLRED_MEM_BLOCK");
        const unsigned b = e ? (unsigned)std::atoi(e) : (unsigned)kBlock;
        return b == 64 || b == 128 ? b : (unsigned)kBlock;
    }();
    uint16_t* r = const_cast<uint16_t*>(ranks);
    // block rows in whole 256-element tiles: the fused pass's LDS form (every rank's
    // tile staged by LDS-DMA, one thread per dword sums from LDS in the same order),
    // one workgroup per tile, result to dst only: 640 kB 13.6 us for k_mem<false, 16>
    // (3.1 TB/s of reads; 160 workgroups) -> see profiles/r01_mem_reduce_ab.txt.
    // ALLRED_MEM_REDUCE_LDS=0: k_mem<false, B> (A/B)
    static const bool lds_form = [] {
        const char* e = std::getenv("ALLRED_MEM_REDUCE_LDS");
        return !(e && std::atoi(e) == 0);
    }();
    const uint64_t bv = nv / total;
    if (lds_form && bv % 32 == 0 && total >= 4 && total <= 64 && (total & (total - 1)) == 0) {
        const dim3 grid((unsigned)(nv / 32)), blk(128);
        hipStream_t st = (hipStream_t)stream;
        switch (total) {
            case 4: hipLaunchKernelGGL(k_mem_lds<4>, grid, blk, 0, st, r, stride, bv, dst); break;
            case 8: hipLaunchKernelGGL(k_mem_lds<8>, grid, blk, 0, st, r, stride, bv, dst); break;
            case 16: hipLaunchKernelGGL(k_mem_lds<16>, grid, blk, 0, st, r, stride, bv, dst); break;
            case 32: hipLaunchKernelGGL(k_mem_lds<32>, grid, blk, 0, st, r, stride, bv, dst); break;
            default: hipLaunchKernelGGL(k_mem_lds<64>, grid, blk, 0, st, r, stride, bv, dst); break;
        }
        return last_error();
    }
    uint64_t g = (nv + block - 1) / block;
    if (g > (uint64_t)kMaxGrid) g = kMaxGrid;
    if (batch == 32)
        hipLaunchKernelGGL((k_mem<false, 32>), dim3((unsigned)g), dim3(block), 0, (hipStream_t)stream, r, stride, total,
                           nv, nv / total, dst);
    else if (batch == 16)
        hipLaunchKernelGGL((k_mem<false, 16>), dim3((unsigned)g), dim3(block), 0, (hipStream_t)stream, r, stride, total,
                           nv, nv / total, dst);
    else
        hipLaunchKernelGGL((k_mem<false, 8>), dim3((unsigned)g), dim3(block), 0, (hipStream_t)stream, r, stride, total,
                           nv, nv / total, dst);
    return last_error();
}

int launch_mem_fused(uint16_t* ranks, uint64_t stride, size_t n, int total, void* stream) {
    if (n % (8 * (size_t)total) || stride % 8 || !aligned16(ranks)) return ALLRED_ERR_ARG;
    const uint64_t nv = n / 8;
    const uint64_t bv = nv / total;
    if (bv % 32 == 0 && total == 64 && nv / 32 >= 1024 && pipe_lag()) {
        // persistent, stores one iteration late (640 kB: ALLRED_PIPE_LAG=0 gives k_mem_lds)
        const uint64_t tiles = nv / 32;
        hipLaunchKernelGGL(k_mem_lds_lag, dim3((unsigned)(tiles < 512 ? tiles : 512)), dim3(kBlock), 0,
                           (hipStream_t)stream, ranks, stride, bv, tiles);
        return last_error();
    }
    if (bv % 32 == 0 && total >= 4) {
        const dim3 grid((unsigned)(nv / 32)), blk(128);
        hipStream_t st = (hipStream_t)stream;
        switch (total) {
            case 4: hipLaunchKernelGGL(k_mem_lds<4>, grid, blk, 0, st, ranks, stride, bv); return last_error();
            case 8: hipLaunchKernelGGL(k_mem_lds<8>, grid, blk, 0, st, ranks, stride, bv); return last_error();
            case 16: hipLaunchKernelGGL(k_mem_lds<16>, grid, blk, 0, st, ranks, stride, bv); return last_error();
            case 32: hipLaunchKernelGGL(k_mem_lds<32>, grid, blk, 0, st, ranks, stride, bv); return last_error();
            case 64: hipLaunchKernelGGL(k_mem_lds<64>, grid, blk, 0, st, ranks, stride, bv); return last_error();
            default: break;
        }
    }
    hipLaunchKernelGGL(k_mem<true>, dim3(grid_for(nv)), dim3(kBlock), 0, (hipStream_t)stream, ranks, stride,
                       total, nv, nv / total, nullptr);
    return last_error();
}

}  // namespace tsa
