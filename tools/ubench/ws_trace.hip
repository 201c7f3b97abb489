// ws_trace.hip — timeline of the pipelined hierarchical step (k_hier_ws) on one
// GPU (W = 1, 64 ranks x 327,680 bf16, config 2): average time per launch of
// k_hier_ws vs k_hier_ll over 32 rotating bucket sets, then one traced launch
// (ALLRED_WS_TRACE stamps, 100 MHz) summarised per tile slot over the
// workgroups that own 3 tiles.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../include \
//         -I../../tenstorrentallreduce_amd/csrc ws_trace.hip -o ws_trace
#ifndef NO_TRACE
#define ALLRED_WS_TRACE 1
#endif
#include "../../tenstorrentallreduce_amd/csrc/kernels.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

int main(int argc, char** argv) {
    using namespace tsa;
    const int P = 64, SETS = 32, REPS = argc > 1 ? std::atoi(argv[1]) : 200;
    const unsigned cap = argc > 2 ? (unsigned)std::atoi(argv[2]) : 0;
    const size_t n = 327680, stride = n + 64, ntiles = n / 256;
    std::vector<uint16_t*> sets(SETS);
    for (auto& s : sets) {
        CK(hipMalloc(&s, (size_t)P * stride * 2));
        CK(hipMemset(s, 0x3f, (size_t)P * stride * 2));
    }
    uint8_t* order;
    CK(hipMalloc(&order, 64));
    std::vector<uint8_t> ord(64);
    for (int i = 0; i < 64; ++i) ord[i] = (uint8_t)i;
    CK(hipMemcpy(order, ord.data(), 64, hipMemcpyHostToDevice));
    const uint64_t box_words = ntiles * 128;
    uint64_t* ll;   // 2 parities x [inbox][box]
    CK(hipExtMallocWithFlags((void**)&ll, 2 * 2 * box_words * 8, hipDeviceMallocUncached));
    CK(hipMemset(ll, 0, 2 * 2 * box_words * 8));
    uint32_t* status;
    CK(hipMalloc(&status, 4));
    CK(hipMemset(status, 0, 4));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    uint32_t epoch = 0;
    auto run = [&](int form, int i) {
        ++epoch;
        uint64_t* l[1] = {ll + (epoch & 1) * 2 * box_words};
        int rc = 0;
        if (form == 1) {
            rc = launch_hier_ll(sets[i % SETS], stride, order, l, 1, 0, n, box_words, epoch, status, cap, st);
        } else if (form == 2) {
            rc = launch_hier_ws(sets[i % SETS], stride, order, l, 1, 0, n, box_words, epoch, status, cap, st);
        } else {   // diagnostic modes of k_hier_ws (W = 1)
            LLPtrs lp{};
            lp.ll[0] = l[0];
            const unsigned grid = (unsigned)std::min<size_t>(ntiles, cap && cap < 512 ? cap : 512);
            if (form == 3)
                hipLaunchKernelGGL(k_hier_ws<1>, dim3(grid), dim3(kWsBlock), 0, st, sets[i % SETS], stride, order, lp, 1,
                                   0, ntiles, ntiles, box_words, epoch, status);
            else if (form == 7)
                hipLaunchKernelGGL(k_hier_ws<6>, dim3(grid), dim3(kWsBlock), 0, st, sets[i % SETS], stride, order, lp, 1,
                                   0, ntiles, ntiles, box_words, epoch, status);
            else if (form == 8)
                hipLaunchKernelGGL(k_hier_ws<5>, dim3(grid), dim3(kWsBlock), 0, st, sets[i % SETS], stride, order, lp, 1,
                                   0, ntiles, ntiles, box_words, epoch, status);
            else if (form == 6)
                hipLaunchKernelGGL(k_hier_ws<4>, dim3(grid), dim3(kWsBlock), 0, st, sets[i % SETS], stride, order, lp, 1,
                                   0, ntiles, ntiles, box_words, epoch, status);
            else if (form == 5)
                hipLaunchKernelGGL(k_hier_ws<3>, dim3(grid), dim3(kWsBlock), 0, st, sets[i % SETS], stride, order, lp, 1,
                                   0, ntiles, ntiles, box_words, epoch, status);
            else
                hipLaunchKernelGGL(k_hier_ws<2>, dim3(grid), dim3(kWsBlock), 0, st, sets[i % SETS], stride, order, lp, 1,
                                   0, ntiles, ntiles, box_words, epoch, status);
        }
        if (rc) { std::printf("launch rc %d\n", rc); std::exit(1); }
    };
    const char* names_f[9] = {"", "k_hier_ll", "k_hier_ws", "ws<1> data only", "ws<2> data only lag 1",
                              "ws<3> lag 1 + 2 spinning waves", "ws<4> lag 1 + 2 sleeping waves, s_wakeup", "ws<6> helpers sleep 3 us, no LDS",
                              "ws<5> helpers leave after tile 0"};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int round = 0; round < 3; ++round) {
        for (int form : {4, 7}) {
            for (int i = 0; i < 20; ++i) run(form, i);
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < REPS; ++i) run(form, i);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::printf("{\"form\": \"%s\", \"cap\": %u, \"us\": %.3f}\n", names_f[form], cap,
                        ms * 1e3 / REPS);
        }
    }
#ifndef ALLRED_WS_TRACE
    return 0;
#else
    // one traced launch
    std::vector<uint64_t> tr(1024 * 16);
    const int traced = argc > 3 ? std::atoi(argv[3]) : 2;
    run(traced, 0);
    CK(hipStreamSynchronize(st));
    CK(hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(g_ws_trace), tr.size() * 8));
    uint32_t stv;
    CK(hipMemcpy(&stv, status, 4, hipMemcpyDeviceToHost));
    const unsigned grid = (unsigned)std::min<size_t>(ntiles, cap && cap < 512 ? cap : 512);
    uint64_t t0 = ~0ull;
    for (unsigned b = 0; b < grid; ++b) t0 = std::min(t0, tr[b * 16 + 0]);
    const char* names[16] = {"start", "L0 in", "L1 in", "L2 in", "res0 seen", "res1 seen", "res2 seen", "data end",
                             "res0 LDS", "res1 LDS", "res2 LDS", "push0", "push1", "push2", "poll0 done", "own0 seen"};
    std::printf("status %u, grid %u; us after the first workgroup start, over workgroups with >= 3 tiles:\n", stv, grid);
    for (int s = 0; s < 16; ++s) {
        std::vector<double> v;
        for (unsigned b = 0; b < grid; ++b) {
            const int mine = (int)((ntiles - 1 - b) / grid + 1);
            if (mine < 3) continue;
            v.push_back((double)(tr[b * 16 + s] - t0) / 100.0);
        }
        if (v.empty()) continue;
        std::sort(v.begin(), v.end());
        std::printf("  %-10s min %6.2f  med %6.2f  max %6.2f\n", names[s], v.front(), v[v.size() / 2], v.back());
    }
    return 0;
#endif
}
