// pmc_calib.hip — calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access
// widths of the hierarchical hand-offs (MI355X_MICROARCH.md §HBM: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").  Each kernel
// moves exactly B bytes once:
//   k_wide_load   16 B per lane nontemporal loads, cached memory (the guide's calibrated case: x 1/2)
//   k_wide_store  16 B per lane nontemporal stores, cached memory (calibrated: exact)
//   k_word_load   8 B per lane relaxed system-scope atomic loads, uncached memory (h_load / ll_load)
//   k_word_store  8 B per lane relaxed system-scope atomic stores, uncached memory (h_put / ll_put)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 pmc_calib.hip -o pmc_calib
//   rocprofv3 --pmc FETCH_SIZE -- ./pmc_calib ; rocprofv3 --pmc WRITE_SIZE -- ./pmc_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_wide_load(const uint4* __restrict__ src, uint64_t nv, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t v = blockIdx.x * 256ull + threadIdx.x; v < nv; v += (uint64_t)gridDim.x * 256) {
        u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + v));
        acc ^= x.x ^ x.y ^ x.z ^ x.w;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;   // keeps the loads; never true for the zero-filled buffer
}
__global__ __launch_bounds__(256) void k_wide_store(uint4* __restrict__ dst, uint64_t nv) {
    for (uint64_t v = blockIdx.x * 256ull + threadIdx.x; v < nv; v += (uint64_t)gridDim.x * 256) {
        u32x4 x = {(uint32_t)v, 1u, 2u, 3u};
        __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(dst + v));
    }
}
__global__ __launch_bounds__(256) void k_word_load(const uint64_t* __restrict__ src, uint64_t nw, uint32_t* sink) {
    uint64_t acc = 0;
    for (uint64_t w = blockIdx.x * 256ull + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * 256)
        acc ^= __hip_atomic_load(src + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (acc == 0x9e3779b97f4a7c15ull) sink[0] = (uint32_t)acc;
}
__global__ __launch_bounds__(256) void k_word_store(uint64_t* __restrict__ dst, uint64_t nw) {
    for (uint64_t w = blockIdx.x * 256ull + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * 256)
        __hip_atomic_store(dst + w, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main(int argc, char** argv) {
    const uint64_t bytes = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 512ull) << 20;   // MiB
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    void *cached = nullptr, *uc = nullptr;
    uint32_t* sink = nullptr;
    CK(hipMalloc(&cached, bytes));
    CK(hipExtMallocWithFlags(&uc, bytes, hipDeviceMallocUncached));
    CK(hipMalloc((void**)&sink, 4));
    CK(hipMemset(cached, 0, bytes));
    CK(hipMemset(uc, 0, bytes));
    CK(hipDeviceSynchronize());
    const dim3 grid(1024), blk(256);
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(k_wide_load, grid, blk, 0, nullptr, (const uint4*)cached, bytes / 16, sink);
        hipLaunchKernelGGL(k_wide_store, grid, blk, 0, nullptr, (uint4*)cached, bytes / 16);
        hipLaunchKernelGGL(k_word_load, grid, blk, 0, nullptr, (const uint64_t*)uc, bytes / 8, sink);
        hipLaunchKernelGGL(k_word_store, grid, blk, 0, nullptr, (uint64_t*)uc, bytes / 8);
    }
    CK(hipDeviceSynchronize());
    std::printf("{\"bytes_per_kernel\": %llu, \"reps\": %d}\n", (unsigned long long)bytes, reps);
    CK(hipFree(cached));
    CK(hipFree(uc));
    CK(hipFree(sink));
    return 0;
}
