// stream_ubench.hip — A/B variants of the engine's streaming kernels in ONE
// process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24).
// Includes the product kernels translation unit so the baseline arms are the
// shipped kernels; candidate arms are defined here.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include -I../../tenstorrentallreduce_amd/csrc \
//         stream_ubench.hip -o stream_ubench -L../../tenstorrentallreduce_amd/lib -lallred
#include "../../tenstorrentallreduce_amd/csrc/kernels.hip"

#include <algorithm>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

namespace tsa {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ntl(const uint4* p) {
    u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nts(uint4 v, uint4* p) {
    u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
}

// ---- candidate: tree kernel with nontemporal data path + SGPR order row ----
template <int P, int NTM, int LEAVES>
__global__ __launch_bounds__(kBlock) void k_tree_v3(uint16_t* __restrict__ ranks, uint64_t stride, uint64_t n_vec,
                                                    const uint8_t* __restrict__ order, uint64_t block_vec, int iters) {
    constexpr bool NTL = NTM & 1, NTS = NTM & 2;
    constexpr int LANES = P / LEAVES;
    constexpr int CH = 64 / LANES;
    const int lane = threadIdx.x & 63;
    const int g = lane / CH;
    const int c = lane % CH;
    const uint64_t wave = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const uint64_t waves = (uint64_t)gridDim.x * (kBlock / 64);
    uint64_t cur = ~0ull;
    uint4* rows[LEAVES];
    for (uint64_t base = wave * CH; base < n_vec; base += waves * CH) {
        const uint64_t v = base + c;
        const bool ok = v < n_vec;
        const uint64_t b = (block_vec && ok) ? v / block_vec : 0;
        if (b != cur) {
            cur = b;
#pragma unroll
            for (int i = 0; i < LEAVES; ++i)
                rows[i] = reinterpret_cast<uint4*>(ranks + (uint64_t)order[b * 64 + g * LEAVES + i] * stride);
        }
        uint4 x[LEAVES];
#pragma unroll
        for (int i = 0; i < LEAVES; ++i) {
            if (NTL) x[i] = ok ? ntl(rows[i] + v) : make_uint4(0, 0, 0, 0);
            else x[i] = ok ? rows[i][v] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int w = 1; w < LEAVES; w *= 2)
#pragma unroll
            for (int i = 0; i < LEAVES; i += 2 * w) x[i] = add8(x[i], x[i + w]);
        uint4 acc = x[0];
#pragma unroll
        for (int m = CH; m < 64; m *= 2) acc = add8(acc, shfl_xor4(acc, m));
        if (ok) {
#pragma unroll
            for (int i = 0; i < LEAVES; ++i) {
                if (NTS) nts(acc, rows[i] + v);
                else rows[i][v] = acc;
            }
        }
    }
}

// ---- candidate: LDS-staged transpose.  One workgroup = one tile of 256
// elements (512 B) of all 64 ranks.  Each wave-instruction moves 1 KiB
// contiguous (two ranks' rows) HBM -> LDS (global_load_lds); each wave then
// reduces 16 leaves of every column from LDS, partials meet in LDS, and the
// result row is stored to every rank with 1 KiB contiguous wave-stores.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(1))) const uint32_t g_u32;

template <bool NT>
__global__ __launch_bounds__(256) void k_tree_lds(uint16_t* __restrict__ ranks, uint64_t stride, uint64_t n_vec,
                                                  const uint8_t* __restrict__ order, uint64_t block_vec) {
    constexpr int TV = 32;                       // 16-byte vectors per rank per tile
    __shared__ __attribute__((aligned(16))) uint4 tile[64 * TV + 4 * TV];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t v0 = (uint64_t)blockIdx.x * TV;
    // stage: wave w loads ranks 16w .. 16w+15, two ranks per instruction
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int r = 16 * w + 2 * k + (lane >> 5);
        const uint4* src = reinterpret_cast<const uint4*>(ranks + (uint64_t)r * stride) + v0 + (lane & 31);
        __builtin_amdgcn_global_load_lds((g_u32*)src, (lds_u32*)&tile[(16 * w + 2 * k) * TV], 16, 0, NT ? 2 : 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint64_t b = v0 / block_vec;
    const int c = lane & 31, h = lane >> 5;
    uint4 x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = tile[(int)order[b * 64 + 16 * w + 8 * h + i] * TV + c];
#pragma unroll
    for (int s2 = 1; s2 < 8; s2 *= 2)
#pragma unroll
        for (int i = 0; i < 8; i += 2 * s2) x[i] = add8(x[i], x[i + s2]);
    uint4 acc = add8(x[0], shfl_xor4(x[0], 32));
    if (h == 0) tile[64 * TV + w * TV + c] = acc;
    __syncthreads();
    const uint4 p0 = tile[64 * TV + 0 * TV + c], p1 = tile[64 * TV + 1 * TV + c];
    const uint4 p2 = tile[64 * TV + 2 * TV + c], p3 = tile[64 * TV + 3 * TV + c];
    const uint4 res = add8(add8(p0, p1), add8(p2, p3));
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int r = 16 * w + 2 * k + h;
        uint4* dst = reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + v0 + c;
        if (NT) nts(res, dst); else *dst = res;
    }
}

// generic LDS-staged tree: TV 16-B vectors per rank row, NW waves per workgroup
template <int TV, int NW, bool NT>
__global__ __launch_bounds__(64 * NW) void k_tree_lds2(uint16_t* __restrict__ ranks, uint64_t stride, uint64_t n_vec,
                                                       const uint8_t* __restrict__ order, uint64_t block_vec) {
    constexpr int RPI = 64 / TV;            // rank rows per wave-instruction
    constexpr int RPW = 64 / NW;            // ranks per wave
    constexpr int LPL = RPW / RPI;          // leaves per lane
    __shared__ __attribute__((aligned(16))) uint4 tile[64 * TV + NW * TV];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t v0 = (uint64_t)blockIdx.x * TV;
    const int c = lane % TV, h = lane / TV;
#pragma unroll
    for (int k = 0; k < RPW / RPI; ++k) {
        const int r = RPW * w + RPI * k + h;
        const uint4* src = reinterpret_cast<const uint4*>(ranks + (uint64_t)r * stride) + v0 + c;
        __builtin_amdgcn_global_load_lds((g_u32*)src, (lds_u32*)&tile[(RPW * w + RPI * k) * TV], 16, 0, NT ? 2 : 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint64_t b = v0 / block_vec;
    uint4 x[LPL];
#pragma unroll
    for (int i = 0; i < LPL; ++i) x[i] = tile[(int)order[b * 64 + RPW * w + LPL * h + i] * TV + c];
#pragma unroll
    for (int s2 = 1; s2 < LPL; s2 *= 2)
#pragma unroll
        for (int i = 0; i < LPL; i += 2 * s2) x[i] = add8(x[i], x[i + s2]);
    uint4 acc = x[0];
#pragma unroll
    for (int m = TV; m < 64; m *= 2) acc = add8(acc, shfl_xor4(acc, m));
    if (NW > 1) {
        if (h == 0) tile[64 * TV + w * TV + c] = acc;
        __syncthreads();
        uint4 p[NW];
#pragma unroll
        for (int i = 0; i < NW; ++i) p[i] = tile[64 * TV + i * TV + c];
#pragma unroll
        for (int s2 = 1; s2 < NW; s2 *= 2)
#pragma unroll
            for (int i = 0; i < NW; i += 2 * s2) p[i] = add8(p[i], p[i + s2]);
        acc = p[0];
    }
#pragma unroll
    for (int k = 0; k < RPW / RPI; ++k) {
        const int r = RPW * w + RPI * k + h;
        uint4* dst = reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + v0 + c;
        if (NT) nts(acc, dst); else *dst = acc;
    }
}

// k_tree_lds with the partials reusing the tile (32 KiB LDS -> 5 workgroups per CU, one round)
template <bool NT>
__global__ __launch_bounds__(256) void k_tree_lds5(uint16_t* __restrict__ ranks, uint64_t stride, uint64_t n_vec,
                                                   const uint8_t* __restrict__ order, uint64_t block_vec) {
    constexpr int TV = 32;
    __shared__ __attribute__((aligned(16))) uint4 tile[64 * TV];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t v0 = (uint64_t)blockIdx.x * TV;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int r = 16 * w + 2 * k + (lane >> 5);
        const uint4* src = reinterpret_cast<const uint4*>(ranks + (uint64_t)r * stride) + v0 + (lane & 31);
        __builtin_amdgcn_global_load_lds((g_u32*)src, (lds_u32*)&tile[(16 * w + 2 * k) * TV], 16, 0, NT ? 2 : 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint64_t b = v0 / block_vec;
    const int c = lane & 31, h = lane >> 5;
    uint4 x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = tile[(int)order[b * 64 + 16 * w + 8 * h + i] * TV + c];
#pragma unroll
    for (int s2 = 1; s2 < 8; s2 *= 2)
#pragma unroll
        for (int i = 0; i < 8; i += 2 * s2) x[i] = add8(x[i], x[i + s2]);
    uint4 acc = add8(x[0], shfl_xor4(x[0], 32));
    __syncthreads();                       // every wave has read its leaves: rows 0-3 are free
    if (h == 0) tile[w * TV + c] = acc;
    __syncthreads();
    const uint4 res = add8(add8(tile[0 * TV + c], tile[1 * TV + c]), add8(tile[2 * TV + c], tile[3 * TV + c]));
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int r = 16 * w + 2 * k + h;
        uint4* dst = reinterpret_cast<uint4*>(ranks + (uint64_t)r * stride) + v0 + c;
        if (NT) nts(res, dst); else *dst = res;
    }
}

template <bool NT, int UNROLL>
__global__ __launch_bounds__(kBlock) void k_add_v2(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                   uint64_t n_vec) {
    const uint64_t T = gthreads();
    uint64_t i = gtid();
    for (; i + (UNROLL - 1) * T < n_vec; i += UNROLL * T) {
        uint4 a[UNROLL], b[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            if (NT) { a[u] = ntl(dst + i + u * T); b[u] = ntl(src + i + u * T); }
            else { a[u] = dst[i + u * T]; b[u] = src[i + u * T]; }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            if (NT) nts(add8(a[u], b[u]), dst + i + u * T);
            else dst[i + u * T] = add8(a[u], b[u]);
        }
    }
    for (; i < n_vec; i += T) dst[i] = add8(dst[i], src[i]);
}

__global__ __launch_bounds__(kBlock) void k_copy(uint4* __restrict__ dst, const uint4* __restrict__ src, uint64_t n_vec) {
    for (uint64_t i = gtid(); i < n_vec; i += gthreads()) dst[i] = src[i];
}

}  // namespace
}  // namespace tsa

using namespace tsa;

struct Arm {
    std::string name;
    double bytes;
    std::function<void(int, hipStream_t)> run;  // arg: rotation index
    std::vector<float> us;
};

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
    const int reps = 50;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    // ---------- config-2 buckets: 64 ranks x 327,680 bf16, 8 rotating sets, two strides
    const int P = 64;
    const size_t n = 327680;
    const int sets = 8;
    const size_t pads[] = {0, 64, 2048 + 64};
    uint16_t* base[3];
    for (int k = 0; k < 3; ++k) {
        CK(hipMalloc(&base[k], (size_t)sets * P * (n + pads[k]) * 2));
        {
            std::vector<uint16_t> h((size_t)sets * P * (n + pads[k]));
            uint32_t x = 12345u + k;
            for (auto& e : h) { x = x * 1664525u + 1013904223u; e = (uint16_t)(0x3f80 + ((x >> 16) % 0x348)); }
            CK(hipMemcpy(base[k], h.data(), h.size() * 2, hipMemcpyHostToDevice));
        }
    }
    allred_schedule s;
    build_schedule(ALLRED_SWING, 8, 64, &s, nullptr);
    uint8_t* d_order;
    CK(hipMalloc(&d_order, 64 * 64));
    CK(hipMemcpy(d_order, &s.tree_order[0][0], 64 * 64, hipMemcpyHostToDevice));
    const double tree_bytes = 2.0 * P * n * 2;
    std::vector<Arm> arms;
    for (int k = 0; k < 3; ++k) {
        const size_t stride = n + pads[k];
        uint16_t* b0 = base[k];
        arms.push_back({"tree shipped(lds) pad=" + std::to_string(pads[k] * 2) + "B", tree_bytes, [=](int i, hipStream_t q) {
            launch_tree_fused(b0 + (size_t)(i % sets) * P * stride, stride, n, P, d_order, q); }, {}});
    }
    {
        const size_t stride = n + pads[1];
        uint16_t* b0 = base[1];
        auto add_tree = [&](const char* nm, int leaves, auto kern) {
            const int lanes = 64 / leaves, ch = 64 / lanes;
            const int waves = (int)((n / 8 + ch - 1) / ch);
            for (int per : {1, 2}) {
                const int grid = (waves / per + 3) / 4;
                arms.push_back({std::string(nm) + " L=" + std::to_string(leaves) + " grid=" + std::to_string(grid), tree_bytes,
                                [=](int i, hipStream_t q) {
                                    uint16_t* r = b0 + (size_t)(i % sets) * P * stride;
                                    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, q, r, stride, n / 8, d_order, n / 8 / 64, 1);
                                }, {}});
            }
        };
        add_tree("tree nt-ls", 8, k_tree_v3<64, 3, 8>);
        add_tree("tree nt-l ", 8, k_tree_v3<64, 1, 8>);
        add_tree("tree nt-s ", 8, k_tree_v3<64, 2, 8>);
        add_tree("tree nt-ls", 16, k_tree_v3<64, 3, 16>);
        auto add_lds = [&](const char* nm, int tv, int nw, auto kern) {
            const int grid = (int)(n / 8 / tv);
            arms.push_back({std::string(nm) + " TV=" + std::to_string(tv) + " NW=" + std::to_string(nw) + " grid=" + std::to_string(grid), tree_bytes,
                            [=](int i, hipStream_t q) {
                                uint16_t* r = b0 + (size_t)(i % sets) * P * stride;
                                hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * nw), 0, q, r, stride, n / 8, d_order, n / 8 / 64);
                            }, {}});
        };
        add_lds("lds5 nt", 32, 4, k_tree_lds5<true>);
        add_lds("lds5   ", 32, 4, k_tree_lds5<false>);
        add_lds("lds2 nt", 32, 4, k_tree_lds2<32, 4, true>);
        add_lds("lds2 nt", 16, 4, k_tree_lds2<16, 4, true>);
        add_lds("lds2 nt", 64, 4, k_tree_lds2<64, 4, true>);
        add_lds("lds2 nt", 64, 8, k_tree_lds2<64, 8, true>);
        add_lds("lds2   ", 32, 4, k_tree_lds2<32, 4, false>);
        for (int nt = 0; nt < 2; ++nt)
            arms.push_back({std::string("tree lds-stage") + (nt ? " nt" : "") + " grid=1280", tree_bytes,
                            [=](int i, hipStream_t q) {
                                uint16_t* r = b0 + (size_t)(i % sets) * P * stride;
                                if (nt) hipLaunchKernelGGL((k_tree_lds<true>), dim3(1280), dim3(256), 0, q, r, stride, n / 8, d_order, n / 8 / 64);
                                else hipLaunchKernelGGL((k_tree_lds<false>), dim3(1280), dim3(256), 0, q, r, stride, n / 8, d_order, n / 8 / 64);
                            }, {}});
    }
    // ---------- floor for the tree's traffic: copy 40 MiB -> 40 MiB (same rotating sets), one vector per thread
    {
        const size_t stride = n + pads[1];
        uint16_t* b0 = base[1];
        const uint64_t half_vec = (uint64_t)P * stride / 8 / 2;
        for (int nt = 0; nt < 2; ++nt)
            arms.push_back({std::string("copy 40MiB (tree floor)") + (nt ? " nt" : ""), tree_bytes, [=](int i, hipStream_t q) {
                uint4* r = (uint4*)(b0 + (size_t)(i % sets) * P * stride);
                if (nt) hipLaunchKernelGGL((k_add_v2<true, 1>), dim3((unsigned)(half_vec / 256)), dim3(256), 0, q, r, r + half_vec, half_vec);
                else hipLaunchKernelGGL(k_copy, dim3((unsigned)(half_vec / 256)), dim3(256), 0, q, r, r + half_vec, half_vec);
            }, {}});
    }
    // ---------- tile-sum: 256 MiB pairs x 4
    const size_t tn = (256u << 20) / 2;
    const int tp = 4;
    uint16_t *ta, *tb;
    CK(hipMalloc(&ta, tn * 2 * tp));
    CK(hipMalloc(&tb, tn * 2 * tp));
    CK(hipMemset(ta, 0x3f, tn * 2 * tp));
    CK(hipMemset(tb, 0x3f, tn * 2 * tp));
    const double ts_bytes = 3.0 * tn * 2;
    arms.push_back({"tilesum shipped", ts_bytes, [=](int i, hipStream_t q) {
        launch_bf16_add(ta + (size_t)(i % tp) * tn, tb + (size_t)(i % tp) * tn, tn, q); }, {}});
    for (int grid : {65536, 32768, 16384}) {
        for (int nt = 0; nt < 2; ++nt) {
            arms.push_back({"tilesum v2 grid=" + std::to_string(grid) + (nt ? " nt" : ""), ts_bytes,
                            [=](int i, hipStream_t q) {
                                uint4* d = (uint4*)(ta + (size_t)(i % tp) * tn);
                                const uint4* sr = (const uint4*)(tb + (size_t)(i % tp) * tn);
                                if (nt) hipLaunchKernelGGL((k_add_v2<true, 1>), dim3(grid), dim3(256), 0, q, d, sr, (uint64_t)tn / 8);
                                else hipLaunchKernelGGL((k_add_v2<false, 1>), dim3(grid), dim3(256), 0, q, d, sr, (uint64_t)tn / 8);
                            }, {}});
        }
    }
    arms.push_back({"copy 256MiB grid=65536", 2.0 * tn * 2, [=](int i, hipStream_t q) {
        hipLaunchKernelGGL(k_copy, dim3(65536), dim3(256), 0, q, (uint4*)(ta + (size_t)(i % tp) * tn),
                           (const uint4*)(tb + (size_t)(i % tp) * tn), (uint64_t)tn / 8); }, {}});
    arms.push_back({"copy 256MiB grid=2048", 2.0 * tn * 2, [=](int i, hipStream_t q) {
        hipLaunchKernelGGL(k_copy, dim3(2048), dim3(256), 0, q, (uint4*)(ta + (size_t)(i % tp) * tn),
                           (const uint4*)(tb + (size_t)(i % tp) * tn), (uint64_t)tn / 8); }, {}});

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r) {
        for (auto& a : arms) {
            for (int i = 0; i < 3; ++i) a.run(i, st);
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < reps; ++i) a.run(i, st);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            a.us.push_back(ms * 1000.0f / reps);
        }
    }
    std::printf("%-40s %10s %10s %8s\n", "arm", "median_us", "min_us", "GB/s");
    for (auto& a : arms) {
        std::sort(a.us.begin(), a.us.end());
        const double med = a.us[a.us.size() / 2];
        std::printf("%-40s %10.2f %10.2f %8.0f\n", a.name.c_str(), med, a.us[0], a.bytes / (med * 1e-6) / 1e9);
    }
    return 0;
}
