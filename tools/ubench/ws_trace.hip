// ws_trace.hip — timeline of the pipelined hierarchical step (k_hier_ws) on one
// GPU (W = 1, 64 ranks x 327,680 bf16, config 2): average time per launch of
// k_hier_ws vs k_hier_ll over 32 rotating bucket sets, then one traced launch
// (ALLRED_WS_TRACE stamps, 100 MHz) summarised per tile slot over the
// workgroups that own 3 tiles.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../include \
//         -I../../tenstorrentallreduce_amd/csrc ws_trace.hip -o ws_trace -L../../tenstorrentallreduce_amd/lib -lallred
#ifndef NO_TRACE
#define ALLRED_WS_TRACE 1
#endif
#include "../../tenstorrentallreduce_amd/csrc/kernels.hip"
#include "../../tenstorrentallreduce_amd/csrc/peer_kernels.hip"

// this probe still bounds its own waits by poll count (the product waits by the clock)
constexpr uint64_t kPeerSpinLimit = 1ull << 22;

// k_hier_ws: the round-1 pipelined specialised-wave form of the hierarchical
// step (removed from the product library: 27-38 us vs 18 for k_hier_ll at W = 1,
// DESIGN.md §5); kept here with its launcher for this study.
namespace tsa {
namespace {
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
                if (spin > kPeerSpinLimit) { atomicOr(status, ALLRED_PEER_TIMEOUT); break; }
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
}  // namespace

int launch_hier_ws(uint16_t* ranks, uint64_t stride, const uint8_t* order, uint64_t* const* ll, int nranks, int me,
                   size_t n, uint64_t box_words, uint32_t epoch, uint32_t* status, unsigned max_grid,
                   void* stream) {
    const uint64_t nv = n / 8, ntiles = nv / 32;
    if (nranks < 1 || nranks > kLLMaxGpus || nv % 32 || ntiles % nranks || stride % 8 || !aligned16(ranks) ||
        ntiles * 128 > box_words)
        return ALLRED_ERR_ARG;
    LLPtrs lp{};
    for (int q = 0; q < nranks; ++q) lp.ll[q] = ll[q];
    const unsigned cap = max_grid && max_grid < 512 ? max_grid : 512;
    const unsigned grid = (unsigned)(ntiles < cap ? ntiles : cap);
    hipLaunchKernelGGL(k_hier_ws<0>, dim3(grid), dim3(kWsBlock), 0, (hipStream_t)stream, ranks, stride, order, lp, nranks,
                       me, ntiles, ntiles / nranks, box_words, epoch, status);
    return hip_status((int)hipGetLastError());
}
}  // namespace tsa

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
