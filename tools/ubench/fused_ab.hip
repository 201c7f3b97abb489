// fused_ab.hip — A/B of the fused BO pass forms at config 2 (64 ranks x
// 327,680 bf16, stride n + 64) in ONE process, interleaved rounds, 32 rotating
// bucket sets: k_tree_lds_pipe<64,1,32,true,true> (the round-1 product),
// and the k_tree_lds_lag<64,32,VAR> arms (kernels.hip).  First checks that all forms give identical bits on random
// bf16 with a random per-block tree order table.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../include \
//         -I../../tenstorrentallreduce_amd/csrc fused_ab.hip -o fused_ab
#include "../../tenstorrentallreduce_amd/csrc/kernels.hip"

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
    constexpr int NF = 11;
    auto run = [&](int form, uint16_t* r) {
        if (form == 0)
            hipLaunchKernelGGL((k_tree_lds_pipe<64, 1, 32, true, true>), dim3(grid), dim3(kBlock), 0, st, r, stride,
                               order, bv, tiles, nullptr);
        else if (form == 1)
            hipLaunchKernelGGL((k_tree_lds_lag<64, 32, 0>), dim3(grid), dim3(kBlock), 0, st, r, stride, order, bv, tiles);
        else if (form == 2)
            hipLaunchKernelGGL((k_tree_lds_lag<64, 32, 1>), dim3(grid), dim3(kBlock), 0, st, r, stride, order, bv, tiles);
        else if (form == 3)
            hipLaunchKernelGGL((k_tree_lds_lag<64, 32, 2>), dim3(grid), dim3(kBlock), 0, st, r, stride, order, bv, tiles);
        else if (form == 4)
            hipLaunchKernelGGL((k_tree_lds_lag<64, 32, 3>), dim3(grid), dim3(kBlock), 0, st, r, stride, order, bv, tiles);
        else if (form == 5)   // 64-vector (1 KiB per row) tiles, one workgroup per CU
            hipLaunchKernelGGL((k_tree_lds_lag<64, 64, 2>), dim3(256), dim3(kBlock), 0, st, r, stride, order, bv,
                               tiles / 2);
        else if (form == 6)   // two waves per workgroup (32 rank rows each)
            hipLaunchKernelGGL((k_tree_lds_lag<64, 32, 2, 2>), dim3(grid), dim3(128), 0, st, r, stride, order, bv, tiles);
        else if (form == 7)   // eight waves per workgroup (8 rank rows each)
            hipLaunchKernelGGL((k_tree_lds_lag<64, 32, 2, 8>), dim3(grid), dim3(512), 0, st, r, stride, order, bv, tiles);
        else if (form == 8)   // loads and stores interleaved
            hipLaunchKernelGGL((k_tree_lds_lag<64, 32, 7>), dim3(grid), dim3(kBlock), 0, st, r, stride, order, bv, tiles);
        else if (form == 9)
            hipLaunchKernelGGL((k_tree_lds_lag<64, 32, 8>), dim3(grid), dim3(kBlock), 0, st, r, stride, order, bv, tiles);
        else
            hipLaunchKernelGGL((k_tree_lds_lag<64, 32, 9>), dim3(grid), dim3(kBlock), 0, st, r, stride, order, bv, tiles);
    };
    const char* names[NF] = {"k_tree_lds_pipe<64,1,32,true,true>", "k_tree_lds_lag<64,32,0> table first",
                             "k_tree_lds_lag<64,32,1> lds-counter barrier", "k_tree_lds_lag<64,32,2> loads before table",
                             "k_tree_lds_lag<64,32,3> no table (timing only)",
                             "k_tree_lds_lag<64,64,2> 1 KiB rows, grid 256", "k_tree_lds_lag<64,32,2,2> two waves",
                             "k_tree_lds_lag<64,32,2,8> eight waves", "k_tree_lds_lag<64,32,7> interleaved (product)",
                             "k_tree_lds_lag<64,32,8> interleaved S L", "k_tree_lds_lag<64,32,9> interleaved L L S S"};
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
