// fused_ab.hip — A/B of the fused BO pass forms at config 2 (64 ranks x
// 327,680 bf16, stride n + 64) in ONE process, interleaved rounds, 32 rotating
// bucket sets: k_tree_lds_pipe_ab<64,1,32,true,true> (the round-1 product),
// and the k_tree_lds_lag_ab<64,32,VAR> arms — the A/B arms of round 1, kept
// here (the product library carries only VAR 7 as k_tree_lds_lag<64>).  First checks that all forms give identical bits on random
// bf16 with a random per-block tree order table.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../include \
//         -I../../tenstorrentallreduce_amd/csrc fused_ab.hip -o fused_ab -L../../tenstorrentallreduce_amd/lib -lallred
#include "../../tenstorrentallreduce_amd/csrc/kernels.hip"

namespace tsa {
namespace {
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
__global__ __launch_bounds__(kBlock) void k_tree_lds_pipe_ab(uint16_t* __restrict__ ranks, uint64_t stride,
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
__global__ __launch_bounds__(64 * NW) void k_tree_lds_lag_ab(uint16_t* __restrict__ ranks, uint64_t stride,
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
}  // namespace
}  // namespace tsa

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

using namespace tsa;

__global__ void k_fill(uint16_t* p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = (uint16_t)(0x3F80 + x % (0x42C8 - 0x3F80));
    }
}

int main(int argc, char** argv) {
    const int P = 64, SETS = 32, REPS = argc > 1 ? std::atoi(argv[1]) : 200;
    const size_t n = 327680, stride = n + 64, nv = n / 8, bv = nv / P, tiles = nv / 32;
    const unsigned grid = 512;
    std::vector<uint16_t*> sets(SETS);
    for (int i = 0; i < SETS; ++i) {
        CK(hipMalloc(&sets[i], (size_t)P * stride * 2));
        hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, sets[i], (size_t)P * stride, 77u + i);
    }
    // random per-block leaf orders (each row a permutation of 0..63)
    std::vector<uint8_t> ord(P * 64);
    std::mt19937 g(5);
    for (int b = 0; b < P; ++b) {
        std::iota(ord.begin() + b * 64, ord.begin() + b * 64 + 64, 0);
        std::shuffle(ord.begin() + b * 64, ord.begin() + b * 64 + 64, g);
    }
    uint8_t* order;
    CK(hipMalloc(&order, ord.size()));
    CK(hipMemcpy(order, ord.data(), ord.size(), hipMemcpyHostToDevice));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    constexpr int NF = 13;
    auto run = [&](int form, uint16_t* r) {
        if (form == 0)
            hipLaunchKernelGGL((k_tree_lds_pipe_ab<64, 1, 32, true, true>), dim3(grid), dim3(kBlock), 0, st, r, stride,
                               order, bv, tiles, nullptr);
        else if (form == 1)
            hipLaunchKernelGGL((k_tree_lds_lag_ab<64, 32, 0>), dim3(grid), dim3(kBlock), 0, st, r, stride, order, bv, tiles);
        else if (form == 2)
            hipLaunchKernelGGL((k_tree_lds_lag_ab<64, 32, 1>), dim3(grid), dim3(kBlock), 0, st, r, stride, order, bv, tiles);
        else if (form == 3)
            hipLaunchKernelGGL((k_tree_lds_lag_ab<64, 32, 2>), dim3(grid), dim3(kBlock), 0, st, r, stride, order, bv, tiles);
        else if (form == 4)
            hipLaunchKernelGGL((k_tree_lds_lag_ab<64, 32, 3>), dim3(grid), dim3(kBlock), 0, st, r, stride, order, bv, tiles);
        else if (form == 5)   // 64-vector (1 KiB per row) tiles, one workgroup per CU
            hipLaunchKernelGGL((k_tree_lds_lag_ab<64, 64, 2>), dim3(256), dim3(kBlock), 0, st, r, stride, order, bv,
                               tiles / 2);
        else if (form == 6)   // two waves per workgroup (32 rank rows each)
            hipLaunchKernelGGL((k_tree_lds_lag_ab<64, 32, 2, 2>), dim3(grid), dim3(128), 0, st, r, stride, order, bv, tiles);
        else if (form == 7)   // eight waves per workgroup (8 rank rows each)
            hipLaunchKernelGGL((k_tree_lds_lag_ab<64, 32, 2, 8>), dim3(grid), dim3(512), 0, st, r, stride, order, bv, tiles);
        else if (form == 8)   // loads and stores interleaved
            hipLaunchKernelGGL((k_tree_lds_lag_ab<64, 32, 7>), dim3(grid), dim3(kBlock), 0, st, r, stride, order, bv, tiles);
        else if (form == 9)
            hipLaunchKernelGGL((k_tree_lds_lag_ab<64, 32, 8>), dim3(grid), dim3(kBlock), 0, st, r, stride, order, bv, tiles);
        else if (form == 10)
            hipLaunchKernelGGL((k_tree_lds_lag_ab<64, 32, 9>), dim3(grid), dim3(kBlock), 0, st, r, stride, order, bv, tiles);
        else if (form == 11)   // 256-byte rows (16 KiB tiles): 2560 tiles, 5 per workgroup (no half-loaded tail)
            hipLaunchKernelGGL((k_tree_lds_lag_ab<64, 16, 7>), dim3(grid), dim3(kBlock), 0, st, r, stride, order, bv,
                               tiles * 2);
        else   // 256-byte rows, 4 workgroups per CU (2.5 tiles each)
            hipLaunchKernelGGL((k_tree_lds_lag_ab<64, 16, 7>), dim3(2 * grid), dim3(kBlock), 0, st, r, stride, order, bv,
                               tiles * 2);
    };
    const char* names[NF] = {"k_tree_lds_pipe<64,1,32,true,true>", "k_tree_lds_lag<64,32,0> table first",
                             "k_tree_lds_lag<64,32,1> lds-counter barrier", "k_tree_lds_lag<64,32,2> loads before table",
                             "k_tree_lds_lag<64,32,3> no table (timing only)",
                             "k_tree_lds_lag<64,64,2> 1 KiB rows, grid 256", "k_tree_lds_lag<64,32,2,2> two waves",
                             "k_tree_lds_lag<64,32,2,8> eight waves", "k_tree_lds_lag<64,32,7> interleaved (product)",
                             "k_tree_lds_lag<64,32,8> interleaved S L", "k_tree_lds_lag<64,32,9> interleaved L L S S",
                             "k_tree_lds_lag<64,16,7> 256-B rows, grid 512", "k_tree_lds_lag<64,16,7> 256-B rows, grid 1024"};
    // bits: every form on a copy of set 0
    const size_t bytes = (size_t)P * stride * 2;
    std::vector<uint16_t> ref(P * stride), got(P * stride);
    uint16_t* tmp;
    CK(hipMalloc(&tmp, bytes));
    for (int form = 0; form < NF; ++form) {
        CK(hipMemcpy(tmp, sets[0], bytes, hipMemcpyDeviceToDevice));
        run(form, tmp);
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(form ? got.data() : ref.data(), tmp, bytes, hipMemcpyDeviceToHost));
        if (form) {
            size_t bad = 0;
            for (int r = 0; r < P; ++r)
                for (size_t i = 0; i < n; ++i) bad += got[r * stride + i] != ref[r * stride + i];
            std::printf("{\"form\": \"%s\", \"mismatches_vs_pipe\": %zu}\n", names[form], bad);
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int round = 0; round < 3; ++round) {
        for (int form = 0; form < NF; ++form) {
            for (int i = 0; i < 20; ++i) run(form, sets[i % SETS]);
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < REPS; ++i) run(form, sets[i % SETS]);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / REPS;
            std::printf("{\"form\": \"%s\", \"round\": %d, \"us\": %.3f, \"hbm_frac\": %.4f}\n", names[form], round, us,
                        2.0 * P * n * 2 / (us * 1e-6) / 8e12);
        }
    }
    return 0;
}
