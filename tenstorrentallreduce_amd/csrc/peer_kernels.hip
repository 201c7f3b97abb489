// peer_kernels.hip — CDNA4 (gfx950) kernels of the multi-GPU transports over
// IPC-mapped peer windows (peer.cpp): the allred_mem_2D program across GPUs
// (one-shot reduce-scatter / all-gather, allred_mem_2D/kernels/*), the Swing /
// RecDub BO and LO program of dist.cpp with RCCL replaced by direct xGMI reads
// of the partners' windows, the hierarchical step (64 local ranks per GPU) and
// the LL (data + epoch word) push forms for small buckets.
// Every cross-GPU wait is bounded (device.hpp peer_give_up): a dead or slow
// peer sets ALLRED_PEER_TIMEOUT in the status word instead of hanging.
#include <map>
#include <mutex>
#include <utility>

#include "device.hpp"

namespace tsa {
namespace {

// ---------------------------------------------------------------------------
// Peer-mapped one-shot allreduce (allred_mem_2D over xGMI): every GPU's window
// is IPC-mapped into every other GPU; flags live in fine-grained (uncached)
// memory and are written / polled with system-scope atomics.  Kernel
// boundaries on the stream carry the system-scope release / acquire of the
// window bytes (HIP dispatch packets fence at system scope).
// ---------------------------------------------------------------------------

struct PeerPtrs {
    uint16_t* win[ALLRED_MAX_NODES];     // window of rank q (this parity), as mapped here
    uint32_t* flags[ALLRED_MAX_NODES];   // flag array of rank q, as mapped here
};

// tune peer_fence = 1 (the `fence` argument of the flag protocols: k_peer_oneshot's
// peer_signal_wait, k_peer_sched's sched_signal / sched_wait, k_peer_sched_push's
// push_signal): a system-scope release fence before every flag store that
// publishes data written before it, and an acquire fence after every flag wait.
// The default (0) relies on the ordering argument of DESIGN.md §5 instead: the
// data go to uncached (MTYPE UC) memory, so a store acknowledged to s_waitcnt
// vmcnt(0) is in the target's HBM before the workgroup barrier that precedes
// the flag.  Same bits either way; the fenced form is the one a node that
// breaks the argument still runs correctly.  The LL kernels take no fence: an
// LL word is its own flag (data and epoch in one 8-byte store), so there is no
// earlier store to order before it (measured: fences around their pushes and
// polls cost 10x, 16 -> 161 us a step at W = 1, for no ordering they need).
__device__ __forceinline__ void peer_release(uint32_t fence) {
    if (fence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}
__device__ __forceinline__ void peer_acquire(uint32_t fence) {
    if (fence) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// one workgroup: tell every peer "rank `me` reached `epoch`", then wait for all.
// Bounded: on timeout bit 0 of *status is set and the kernel returns.
__global__ void k_peer_barrier(PeerPtrs pp, int nranks, int me, uint32_t epoch, uint32_t* status) {
    const int t = threadIdx.x;
    if (t < nranks)
        __hip_atomic_store(pp.flags[t] + me, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (t < nranks) {
        uint32_t* mine = pp.flags[me] + t;
        uint64_t t0 = 0;
        for (uint64_t spin = 0;; ++spin) {
            if (__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= epoch) break;
            if (peer_give_up(spin, t0, status)) break;   // ~ seconds: a peer never arrived
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// kSchedU vectors per thread in flight per loop trip of the copy / add loops
// that read peers' windows over xGMI: a remote read's latency is paid once per
// kSchedU vectors instead of once per vector
constexpr int kSchedU = 4;

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
    const uint64_t G = gthreads();
    for (uint64_t v = gtid(); v < blk_vec; v += kSchedU * G) {
        uint4 y[kSchedU];
#pragma unroll
        for (int u = 0; u < kSchedU; ++u)
            if (v + u * G < blk_vec) y[u] = ld_nt(reinterpret_cast<const uint4*>(pp.win[q]) + off + v + u * G);
#pragma unroll
        for (int u = 0; u < kSchedU; ++u)
            if (v + u * G < blk_vec) st_nt(reinterpret_cast<uint4*>(bucket) + off + v + u * G, y[u]);
    }
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
                                        uint32_t* status, uint32_t fence) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    peer_release(fence);
    __syncthreads();
    const int t = threadIdx.x;
    if (t < nranks)
        __hip_atomic_store(pp.flags[t] + slot_base + me, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (t < nranks) {
        uint32_t* mine = pp.flags[me] + slot_base + t;
        uint64_t t0 = 0;
        for (uint64_t spin = 0;; ++spin) {
            if (__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= epoch) break;
            if (peer_give_up(spin, t0, status)) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
    peer_acquire(fence);
}

__global__ __launch_bounds__(kBlock) void k_peer_oneshot(PeerPtrs pp, int nranks, int me, uint16_t* __restrict__ bucket,
                                                         uint64_t blk_vec, uint64_t chunk, uint32_t epoch,
                                                         uint32_t* status, uint32_t fence) {
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
    peer_signal_wait(pp, nranks, me, base0, epoch, status, fence);
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
    peer_signal_wait(pp, nranks, me, base1, epoch, status, fence);
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
    peer_release(pr.fence);
    __syncthreads();
    const int t = threadIdx.x;
    if (t < pr.S)
        __hip_atomic_store(pp.flags[pr.peer[c][t]] + slot + me, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ inline void sched_wait(const PeerPtrs& pp, int me, uint32_t slot, int q0, int q1, uint32_t value,
                                  uint32_t* status, uint32_t fence) {
    const int t = threadIdx.x;
    const int q = t == 0 ? q0 : (t == 1 ? q1 : -1);
    if (q >= 0) {
        uint32_t* f = pp.flags[me] + slot + q;
        uint64_t t0 = 0;
        for (uint64_t spin = 0;; ++spin) {
            if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= value) break;
            if (peer_give_up(spin, t0, status)) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
    peer_acquire(fence);
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
            sched_wait(pp, me, slot, p, -1, base + 1 + k, status, pr.fence);
            const uint4* theirs = reinterpret_cast<const uint4*>(pp.win[p]);
            const bool last = k == S - 1;
            for (uint64_t m = pr.recv[c][k]; m; m &= m - 1) {
                const int b = __builtin_ctzll(m);
                const uint64_t end = cb + b * blk + hi;
                for (uint64_t v = cb + b * blk + lo + tid; v < end; v += kSchedU * kBlock) {
                    uint4 x[kSchedU], y[kSchedU];
#pragma unroll
                    for (int u = 0; u < kSchedU; ++u)
                        if (v + u * kBlock < end) {
                            x[u] = ld_nt(mine + v + u * kBlock);
                            y[u] = ld_nt(theirs + v + u * kBlock);
                        }
#pragma unroll
                    for (int u = 0; u < kSchedU; ++u)
                        if (v + u * kBlock < end) {
                            const uint4 o = add8(x[u], y[u]);
                            st_nt(mine + v + u * kBlock, o);
                            if (last) st_nt(bk + v + u * kBlock, o);
                        }
                }
            }
            sched_signal(pp, pr, c, me, slot, base + 2 + k);
        }
        for (int t = 0; t < S; ++t) {  // all-gather, steps in reverse
            const int i = S - 1 - t, pos = S + t;
            const int p = pr.peer[c][i];
            sched_wait(pp, me, slot, p, -1, base + 1 + pos, status, pr.fence);
            const uint4* theirs = reinterpret_cast<const uint4*>(pp.win[p]);
            const bool keep = t < S - 1;  // later partners read these blocks from my window
            for (uint64_t m = pr.send[c][i]; m; m &= m - 1) {
                const int b = __builtin_ctzll(m);
                const uint64_t end = cb + b * blk + hi;
                for (uint64_t v = cb + b * blk + lo + tid; v < end; v += kSchedU * kBlock) {
                    uint4 y[kSchedU];
#pragma unroll
                    for (int u = 0; u < kSchedU; ++u)
                        if (v + u * kBlock < end) y[u] = ld_nt(theirs + v + u * kBlock);
#pragma unroll
                    for (int u = 0; u < kSchedU; ++u)
                        if (v + u * kBlock < end) {
                            if (keep) st_nt(mine + v + u * kBlock, y[u]);
                            st_nt(bk + v + u * kBlock, y[u]);
                        }
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
        sched_wait(pp, me, slot, p, (k >= 1 && !last) ? pr.peer[c][k - 1] : -1, base + 1 + k, status, pr.fence);
        const uint4* a = mine + (k & 1) * half_vec;
        const uint4* b = reinterpret_cast<const uint4*>(pp.win[p]) + (k & 1) * half_vec;
        uint4* dst = last ? bk : mine + ((k + 1) & 1) * half_vec;
        for (uint64_t v = lo + tid; v < hi; v += kSchedU * kBlock) {
            uint4 x[kSchedU], y[kSchedU];
#pragma unroll
            for (int u = 0; u < kSchedU; ++u)
                if (v + u * kBlock < hi) {
                    x[u] = ld_nt(a + v + u * kBlock);
                    y[u] = ld_nt(b + v + u * kBlock);
                }
#pragma unroll
            for (int u = 0; u < kSchedU; ++u)
                if (v + u * kBlock < hi) st_nt(dst + v + u * kBlock, add8(x[u], y[u]));
        }
        if (!last) sched_signal(pp, pr, c, me, slot, base + 2 + k);
    }
}

// ---- scheduled form, push variant (BO) --------------------------------------
// k_peer_sched's program with the data moved by the SENDER: remote writes are
// posted (no read round trip over xGMI), so large buckets may stream faster.
//   RS step k: wait until partner p finished step k-1 (its staging window free,
//     progress slot as in the pull form); write my blocks send[k] into p's
//     staging window; raise p's data slot; wait for p's data slot in mine; add
//     my staging blocks recv[k] into my window (and, at the last step, bucket);
//     progress k+1.
//   AG step i: wait for p's progress; write my owned blocks recv[i] into p's
//     MAIN window (p's blocks send_p[i] = my recv[i]: its stale partials there
//     are read by nobody after its RS step i); raise p's data slot; wait for
//     mine; copy my window's blocks send[i] into the bucket.
// Same adds in the same order as the pull form: the same bits.
struct PeerStage {
    uint16_t* st[ALLRED_MAX_NODES];   // GPU q's staging window, as mapped here
};

__device__ inline void push_signal(const PeerPtrs& pp, int p, int me, uint32_t slot, uint32_t value, uint32_t fence) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's pushes have completed
    peer_release(fence);
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(pp.flags[p] + kPeerSchedPushOff + slot + me, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(kBlock) void k_peer_sched_push(PeerPtrs pp, PeerStage ps, PeerProg pr, int me,
                                                            uint16_t* __restrict__ bucket, uint32_t base,
                                                            uint32_t* status) {
    const int C = pr.C, S = pr.S, N = pr.N;
    const int g = blockIdx.x, c = g % C, Gc = gridDim.x / C, j = g / C;
    const uint32_t gs = (uint32_t)g * 64u;                 // this workgroup's slots (progress / pushed data)
    const uint32_t slot = kPeerSchedFlagOff + gs;
    uint4* bk = reinterpret_cast<uint4*>(bucket);
    uint4* mine = reinterpret_cast<uint4*>(pp.win[me]);
    const uint4* stage = reinterpret_cast<const uint4*>(ps.st[me]);
    const uint64_t cb = pr.base[c];
    const int tid = threadIdx.x;
    const uint64_t blk = pr.len[c] / N;
    const uint64_t chunk = (blk + Gc - 1) / Gc;
    const uint64_t lo = (uint64_t)j * chunk, hi = lo + chunk < blk ? lo + chunk : blk;
    // my sub-slice of every block in `mask`: src -> dst (kSchedU vectors in flight per thread)
    auto move = [&](uint64_t mask, const uint4* src, uint4* dst) {
        for (uint64_t m = mask; m; m &= m - 1) {
            const int b = __builtin_ctzll(m);
            const uint64_t end = cb + b * blk + hi;
            for (uint64_t v = cb + b * blk + lo + tid; v < end; v += kSchedU * kBlock) {
                uint4 y[kSchedU];
#pragma unroll
                for (int u = 0; u < kSchedU; ++u)
                    if (v + u * kBlock < end) y[u] = ld_nt(src + v + u * kBlock);
#pragma unroll
                for (int u = 0; u < kSchedU; ++u)
                    if (v + u * kBlock < end) st_nt(dst + v + u * kBlock, y[u]);
            }
        }
    };
    for (int b = 0; b < N; ++b)
        for (uint64_t v = cb + b * blk + lo + tid; v < cb + b * blk + hi; v += kBlock) st_nt(mine + v, ld_nt(bk + v));
    sched_signal(pp, pr, c, me, slot, base + 1);
    for (int k = 0; k < S; ++k) {  // reduce-scatter
        const int p = pr.peer[c][k];
        sched_wait(pp, me, slot, p, -1, base + 1 + k, status, pr.fence);                 // p's staging is free
        move(pr.send[c][k], mine, reinterpret_cast<uint4*>(ps.st[p]));         // my blocks -> p's staging
        push_signal(pp, p, me, gs, base + 1 + k, pr.fence);
        sched_wait(pp, me, kPeerSchedPushOff + gs, p, -1, base + 1 + k, status, pr.fence);   // p's blocks are in mine
        const bool last = k == S - 1;
        for (uint64_t m = pr.recv[c][k]; m; m &= m - 1) {
            const int b = __builtin_ctzll(m);
            const uint64_t end = cb + b * blk + hi;
            for (uint64_t v = cb + b * blk + lo + tid; v < end; v += kSchedU * kBlock) {
                uint4 x[kSchedU], y[kSchedU];
#pragma unroll
                for (int u = 0; u < kSchedU; ++u)
                    if (v + u * kBlock < end) {
                        x[u] = ld_nt(mine + v + u * kBlock);
                        y[u] = ld_nt(stage + v + u * kBlock);
                    }
#pragma unroll
                for (int u = 0; u < kSchedU; ++u)
                    if (v + u * kBlock < end) {
                        const uint4 o = add8(x[u], y[u]);
                        st_nt(mine + v + u * kBlock, o);
                        if (last) st_nt(bk + v + u * kBlock, o);
                    }
            }
        }
        sched_signal(pp, pr, c, me, slot, base + 2 + k);
    }
    for (int t = 0; t < S; ++t) {  // all-gather, steps in reverse
        const int i = S - 1 - t, pos = S + t;
        const int p = pr.peer[c][i];
        sched_wait(pp, me, slot, p, -1, base + 1 + pos, status, pr.fence);               // p is past its RS step i
        move(pr.recv[c][i], mine, reinterpret_cast<uint4*>(pp.win[p]));        // my owned blocks -> p's window
        push_signal(pp, p, me, gs, base + 1 + pos, pr.fence);
        sched_wait(pp, me, kPeerSchedPushOff + gs, p, -1, base + 1 + pos, status, pr.fence);
        move(pr.send[c][i], mine, bk);                                          // p's blocks, now in mine -> bucket
        if (t < S - 1) sched_signal(pp, pr, c, me, slot, base + 2 + pos);
    }
}

// ---- hierarchical one-kernel forms: 64 local ranks per GPU, LL (push) hand-offs
// The whole hierarchical step (local tree of the 64 virtual ranks -> mem_2D
// across the W GPUs -> broadcast back to the 64 ranks) as ONE persistent
// launch (k_hier_ws), or pipelined two buckets deep (k_hier_x2); the same bits
// as tree_reduce + the mem_2D exchange + broadcast (fp32 owner first then
// ascending, one rounding).  Tile = 256 elements (512 B per rank row);
// owner(t) = t / (tiles / W), the block ownership of allred_mem_2D.  Every
// cross-GPU transfer is a PUSH of self-validating 8-byte words (data + the
// call's epoch, RCCL's "LL" idea): the producer's relaxed system-scope stores
// go straight into the consumer's uncached LL area and the consumer polls its
// OWN memory until every word carries the epoch.  No flag follows the data and
// no remote load is ever waited for, so each hand-off costs one one-way xGMI
// trip.  Three roles per tile:
//   A (every tile of the GPU): the local tree -> partial -> owner o's inbox
//     slot [t - o*tpo][me].
//   R (the tiles this GPU owns): poll the W slots, fp32 sum owner first then
//     ascending, one rounding -> every GPU's result box [t].
//   B (every tile): poll the own result box [t], store to the 64 rank rows.
// A never waits, R waits only for A, B only for R; the grid is resident (2
// workgroups per CU), so every wait is reached and satisfied.  Epochs grow by
// one per call and the LL areas alternate by call parity, so a word of an
// earlier call never carries the awaited epoch.  (Retired forms and their
// numbers, profiles/README.md: a per-tile flag form, 19.9 us at W = 1, and a
// pipelined LL form, 17.8 us, in round 5; in round 6 k_hier_ll — A, R, B as
// three phases of every workgroup, 16.2 us — and the one-deep pipeline k_hier_x,
// 15.1-15.3 us, both behind k_hier_ws and k_hier_x2 in every measurement.)
constexpr int kLLMaxGpus = 8;
struct LLPtrs {
    uint64_t* ll[kLLMaxGpus];   // GPU q's LL area, this parity: [inbox: tiles x 128 words][result box: same]
};

// LL slot layout: 32 consecutive slots (16 data bytes each) form a group of 128
// words, word k of slot i of the group at k * 32 + i.  Lanes serving consecutive
// slots therefore write (and poll) 256 contiguous bytes per instruction — whole
// 128-byte lines over xGMI — instead of one 8-byte word every 32 bytes.
constexpr int kLLGroup = 32;
__device__ __forceinline__ uint64_t* ll_slot(uint64_t* base, uint64_t s) {
    return base + (s / kLLGroup) * (4 * kLLGroup) + s % kLLGroup;
}
__device__ __forceinline__ const uint64_t* ll_slot(const uint64_t* base, uint64_t s) {
    return base + (s / kLLGroup) * (4 * kLLGroup) + s % kLLGroup;
}

__device__ __forceinline__ void ll_put(uint64_t* dst, uint4 v, uint32_t e) {
    const uint64_t hi = (uint64_t)e << 32;
    __hip_atomic_store(dst + 0 * kLLGroup, hi | v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(dst + 1 * kLLGroup, hi | v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(dst + 2 * kLLGroup, hi | v.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(dst + 3 * kLLGroup, hi | v.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// poll 4 LL words until all carry epoch e (bounded: status bit 0 on timeout)
__device__ __forceinline__ uint4 ll_get(const uint64_t* src, uint32_t e, uint32_t* status) {
    uint64_t w0, w1, w2, w3;
    uint64_t t0 = 0;
    for (uint64_t spin = 0;; ++spin) {
        w0 = __hip_atomic_load(src + 0 * kLLGroup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        w1 = __hip_atomic_load(src + 1 * kLLGroup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        w2 = __hip_atomic_load(src + 2 * kLLGroup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        w3 = __hip_atomic_load(src + 3 * kLLGroup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((uint32_t)(w0 >> 32) == e && (uint32_t)(w1 >> 32) == e && (uint32_t)(w2 >> 32) == e &&
            (uint32_t)(w3 >> 32) == e)
            break;
        if (peer_give_up(spin, t0, status)) break;
        __builtin_amdgcn_s_sleep(1);
    }
    return make_uint4((uint32_t)w0, (uint32_t)w1, (uint32_t)w2, (uint32_t)w3);
}

// ---- the hierarchical forms' hand-off words (round 5) -------------------------
// A tile's 512-byte partial or result crosses as 96 self-validating 8-byte
// words: column c's 16 bytes as three words, bytes 0-5 / 6-11 / 12-15 of the
// column in bits 0..47 and the call's 16-bit epoch in bits 48..63 — 1.5x the
// data bytes instead of the 2x of the 4 + 4 LL word above.  Word k of column c
// sits at k * 32 + c of the tile's slot (kHSlot words), so the 32 lanes of a
// tile write or poll 256 contiguous bytes per instruction, each lane only its
// own column (no cross-lane traffic; a 7 + 1 byte packing, 1.16x, needed two
// columns per word and ran 0.6-0.8 us slower a step at W = 1 on the shuffles
// and scattered polls, profiles/README.md).  One 8-byte store is the unit of
// visibility, as for the LL words: a word carries its own epoch, no flag
// follows it.  The 16-bit epoch repeats every 65535 calls: the host clears a
// parity's area, between two barriers of the peer set, before a bucket whose
// slots could still hold a word of an older same-parity call with the same
// epoch (peer.cpp hier_area_prepare; every call rewrites all of its own slots,
// so only a bucket larger than the recent ones can meet such a word).
__device__ __forceinline__ uint32_t h_epoch(uint32_t e) { return e % 65535u + 1u; }
constexpr uint64_t kH48 = 0x0000FFFFFFFFFFFFull;
// word k of a column
__device__ __forceinline__ uint64_t h_pack(uint4 v, int k, uint32_t e16) {
    const uint64_t lo = v.x | ((uint64_t)v.y << 32), hi = v.z | ((uint64_t)v.w << 32);
    const uint64_t d = k == 0 ? (lo & kH48) : k == 1 ? ((lo >> 48) | ((hi & 0xFFFFFFFFull) << 16)) : (hi >> 32);
    return d | ((uint64_t)e16 << 48);
}
// the column from its three words
__device__ __forceinline__ uint4 h_unpack(const uint64_t (&wd)[3]) {
    const uint64_t lo = (wd[0] & kH48) | (wd[1] << 48);
    const uint64_t hi = ((wd[1] >> 16) & 0xFFFFFFFFull) | (wd[2] << 32);
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}
// the three words of column c of the tile at `tile`: one poll, no wait
__device__ __forceinline__ void h_load(const uint64_t* tile, int c, uint64_t (&wd)[3]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) wd[k] = __hip_atomic_load(tile + 32 * k + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool h_fresh(const uint64_t (&wd)[3], uint32_t e16) {
    return (uint32_t)(wd[0] >> 48) == e16 && (uint32_t)(wd[1] >> 48) == e16 && (uint32_t)(wd[2] >> 48) == e16;
}
// poll until all three words carry e16 (bounded: status bit 0 on timeout), then the column
__device__ __forceinline__ uint4 h_get(const uint64_t* tile, int c, uint32_t e16, uint32_t* status) {
    uint64_t wd[3];
    uint64_t t0 = 0;
    for (uint64_t spin = 0;; ++spin) {
        h_load(tile, c, wd);
        if (h_fresh(wd, e16)) break;
        if (peer_give_up(spin, t0, status)) break;
        __builtin_amdgcn_s_sleep(1);
    }
    return h_unpack(wd);
}
__device__ __forceinline__ uint4 h_take(const uint64_t (&wd)[3], const uint64_t* tile, int c, uint32_t e16,
                                        uint32_t* status) {
    return h_fresh(wd, e16) ? h_unpack(wd) : h_get(tile, c, e16, status);
}
// column c (v) -> its three words in the tile slot at `tile`
__device__ __forceinline__ void h_put(uint64_t* tile, int c, uint4 v, uint32_t e16) {
#pragma unroll
    for (int k = 0; k < 3; ++k)
        __hip_atomic_store(tile + 32 * k + c, h_pack(v, k, e16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the owner's sum of one column of a tile: y[q] = GPU q's partial; fp32, owner
// first then ascending, one rounding (allred_mem_2D semantics, k_peer_oneshot's bits)
__device__ __forceinline__ uint4 owner_sum(const uint4 (&y)[kLLMaxGpus], int W, int me) {
    uint4 s0 = y[0];
#pragma unroll
    for (int src = 0; src < kLLMaxGpus; ++src)
        if (src == me) s0 = y[src];
    float a[8] = {lo_f(s0.x), hi_f(s0.x), lo_f(s0.y), hi_f(s0.y), lo_f(s0.z), hi_f(s0.z), lo_f(s0.w), hi_f(s0.w)};
#pragma unroll
    for (int qq = 0; qq < kLLMaxGpus; ++qq) {
        if (qq >= W || qq == me) continue;
        a[0] += lo_f(y[qq].x); a[1] += hi_f(y[qq].x);
        a[2] += lo_f(y[qq].y); a[3] += hi_f(y[qq].y);
        a[4] += lo_f(y[qq].z); a[5] += hi_f(y[qq].z);
        a[6] += lo_f(y[qq].w); a[7] += hi_f(y[qq].w);
    }
    return make_uint4(pack_rne(a[0], a[1]), pack_rne(a[2], a[3]), pack_rne(a[4], a[5]), pack_rne(a[6], a[7]));
}

// The workgroup's tiles of the one-launch forms: blk + kG of the reducing grid G
// (identical on every GPU).  A reduces them in a different order (tile_a):
// within each batch of 8, the tiles other GPUs own first, its own tiles last —
// the owned ones form the run k0 <= k < k1.  Every GPU reduces the tiles it does
// not own first, so an owner finds the remote partials of its tiles already
// arrived, and the result leaves after one xGMI trip (natural order: remote
// partials of the last tiles arrive one trip after the owner's own, then the
// result needs a second).  At W = 1 nothing moves.
struct HierTiles {
    uint64_t blk, G, tpo;
    int mine, k0, k1;
    __device__ HierTiles(uint64_t b, uint64_t g, uint64_t ntiles, uint64_t tiles_per_owner, int me)
        : blk(b), G(g), tpo(tiles_per_owner) {
        mine = b < ntiles ? (int)((ntiles - 1 - b) / g + 1) : 0;
        const uint32_t tpo32 = (uint32_t)tiles_per_owner;
        k0 = count_below((uint32_t)me * tpo32);
        k1 = count_below((uint32_t)(me + 1) * tpo32);
    }
    __device__ int count_below(uint32_t t0) const {   // the workgroup's tiles below tile index t0 (< 2^20 tiles)
        return t0 <= blk ? 0 : (int)min((uint32_t)mine, (t0 - (uint32_t)blk + (uint32_t)G - 1) / (uint32_t)G);
    }
    __device__ uint64_t tile_of(int k) const { return blk + (uint64_t)k * G; }
    __device__ uint64_t tile_a(int j) const {
        const int lo = j & ~7, hi = lo + 8 < mine ? lo + 8 : mine;
        const int a0 = k0 < lo ? lo : (k0 > hi ? hi : k0), a1 = k1 < lo ? lo : (k1 > hi ? hi : k1);
        const int p = j - lo, below = a0 - lo, above = hi - a1;
        const int k = p < below ? lo + p : (p < below + above ? a1 + (p - below) : a0 + (p - below - above));
        return tile_of(k);
    }
    __device__ int owner_of(uint64_t t) const { return (int)(t / tpo); }
};

__device__ __forceinline__ uint4 shfl4(uint4 v, int src) {
    return make_uint4((uint32_t)__shfl((int)v.x, src), (uint32_t)__shfl((int)v.y, src), (uint32_t)__shfl((int)v.z, src),
                      (uint32_t)__shfl((int)v.w, src));
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    return (uint64_t)(uint32_t)__shfl((int)(uint32_t)v, src) | ((uint64_t)(uint32_t)__shfl((int)(v >> 32), src) << 32);
}

// k_hier_ws: the hierarchical step in one launch with its two HBM phases on
// different waves of one workgroup, so every CU reads and writes at once (a
// workgroup that reads all its tiles, then writes them — round 4's k_hier_ll —
// makes the chip read, then write: 16.2 us at W = 1 against 14.2 for the fused
// one-GPU pass, which interleaves a tile's stores with later tiles' loads).
// A workgroup has 2 * NQ waves and no barrier after its start; the
// tile's 32 columns (16 bytes each) split into NQ = 32 / CW groups of CW:
//   wave q < NQ (A) reduces columns CW q .. CW q + CW - 1 of the workgroup's
//     tiles on its own: LDS-DMA of those columns of the 64 rank rows into its
//     own two buffers (one tile ahead), CW leaves per lane (lane = leaf group g
//     x column c) and the tree's last levels across lanes (xor CW .. 32 — the
//     tree and operand order of k_hier_x2 and tree_reduce, 8 leaves a lane).  A
//     partial another GPU owns is pushed to its inbox (the 6 + 2-byte words,
//     one per lane); an owned one goes to an LDS slot for wave q + NQ (the
//     first kWsRing owned tiles; later ones through the own inbox), so at W = 1
//     nothing crosses global memory but the rank rows.
//   wave q + NQ (B) writes those columns of the tiles' 64 rank rows: for a tile
//     it owns, the own partial (LDS or inbox) and the W - 1 others polled from
//     its inbox, summed (owner first, fp32, one rounding), the result pushed
//     to every other GPU's box; for another GPU's tile the result polled from
//     its own box.  Two cursors (next owned, next other tile, both polled in a
//     round, whichever arrived is finished): an owned tile waits only for A
//     (which never waits), another only for its owner's owned tile, so no wait
//     is circular.  Bounded like every peer wait (status bit 0).
// CW = 16 (halves: 4 waves, 256-byte row segments) is the default: 14.5-14.7 us a
// step at W = 1 against 14.8-15.0 for quarters (8 waves, 128-byte segments) and
// 16.2 for whole tiles (2 waves: too few in flight); profiles/r05_hier_ws_step_w1.json.
// Every workgroup must be resident (the B waves wait across GPUs): 2 per CU (the
// A buffers' 64 KiB of LDS), max_grid when processes share the GPU.
constexpr int kWsRing = 16;
// AHEAD 1: tile j+1's loads issued before tile j's tree; 2: also tile j+2's, into tile j's buffer
// right after its tree (k_tree_lds_lag's schedule).  CW: columns (16-byte vectors) of a tile per
// reducing wave — 8 (a quarter: 8 waves per workgroup, 128-byte row segments, 8 leaves per
// lane), 16 (a half: 4 waves, 256-byte segments, 16 leaves) or 32 (the whole tile: 2 waves,
// 512-byte segments, 32 leaves)
template <int AHEAD, int CW>
__global__ __launch_bounds__(128 * (32 / CW), (CW == 8 ? 4 : CW == 16 ? 2 : 1)) void k_hier_ws(
    uint16_t* __restrict__ ranks, uint64_t stride, const uint8_t* __restrict__ order, LLPtrs lp, int W, int me,
    uint64_t ntiles, uint64_t tiles_per_owner, uint64_t box_words, uint32_t epoch, uint32_t* status) {
    constexpr int TV = 32, NQ = TV / CW, GR = 64 / CW, LPL = CW, OPS = CW;
    constexpr int NWR = (3 * CW + 63) / 64;   // word rounds: a tile's 3 CW hand-off words of this wave's columns
    static_assert(CW == 8 || CW == 16 || CW == 32, "a quarter, a half or the whole tile per reducing wave");
    __shared__ __attribute__((aligned(16))) uint4 buf[NQ][2][64 * CW];    // A wave q: two tiles of its columns
    __shared__ __attribute__((aligned(16))) uint4 res[NQ][kWsRing][CW];   // A -> B: owned partials
    __shared__ uint32_t prod[NQ];                                          // owned partials published per wave
    // the wave index as a scalar: the A / B split is a uniform branch (one role's code only per wave)
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = w % NQ;
    const int cc = lane % CW, g = lane / CW;
    const uint32_t e8 = h_epoch(epoch);
    const HierTiles ht(blockIdx.x, gridDim.x, ntiles, tiles_per_owner, me);
    const int mine = ht.mine;
    if (threadIdx.x < NQ) prod[threadIdx.x] = 0;
    __syncthreads();
    // hand-off word i = lane + 64 r of this wave's columns: word i / CW of column CW q + i % CW
    // (column i % CW = cc: every lane packs its own column)
    auto wvalid = [&](int r) { return lane + 64 * r < 3 * CW; };
    auto wkey = [&](int r) { return (lane + 64 * r) / CW; };
    auto woff = [&](int r) { return (uint64_t)(32 * wkey(r) + CW * q + cc); };
    if (w < NQ) {
        // ---- A: the leaf bytes CW g .. CW g + CW - 1 of the tree order (loaded ahead of the tiles')
        uint32_t ob[CW / 4];
        if constexpr (CW == 8) {
            u32x2 ov;
            asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(ov) : "v"(order + CW * g) : "memory");
            ob[0] = ov.x;
            ob[1] = ov.y;
        } else {
#pragma unroll
            for (int h = 0; h < CW / 16; ++h) {
                u32x4 ov;
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(ov) : "v"(order + CW * g + 16 * h) : "memory");
                ob[4 * h + 0] = ov.x;
                ob[4 * h + 1] = ov.y;
                ob[4 * h + 2] = ov.z;
                ob[4 * h + 3] = ov.w;
            }
        }
        const uint32_t wbase = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&buf[q][0][0]);
        auto issue = [&](uint64_t t, int b) {   // rows GR k + g, column CW q + cc: GR rows x 16 CW bytes per op
#pragma unroll
            for (int k = 0; k < OPS; ++k)
                lds_dma16(reinterpret_cast<const uint4*>(ranks + (uint64_t)(GR * k + g) * stride) + t * TV + CW * q + cc,
                          wbase + (uint32_t)(b * 64 * CW * 16 + k * 1024));
        };
        if (mine > 0) issue(ht.tile_a(0), 0);
        if (AHEAD == 2 && mine > 1) issue(ht.tile_a(1), 1);
        bool pushed = false;   // the previous tile's partial went out as global stores (NWR ops)
        int ko = 0;            // owned tiles so far
        for (int j = 0; j < mine; ++j) {
            // after L(j): AHEAD 1 the previous tile's stores; AHEAD 2 those and L(j+1)
            if (AHEAD == 2 && j + 1 < mine) {
                if (pushed) wait_vm<OPS + NWR>(); else wait_vm<OPS>();
            } else {
                if (pushed) wait_vm<NWR>(); else wait_vm<0>();
            }
#pragma unroll
            for (int i = 0; i < CW / 4; ++i) asm volatile("" : "+v"(ob[i]));   // no use may move above the first wait
            if (AHEAD == 1 && j + 1 < mine) issue(ht.tile_a(j + 1), (j + 1) & 1);
            const uint4* tile = buf[q][j & 1];
            uint4 x[LPL];
#pragma unroll
            for (int i = 0; i < LPL; ++i) {
                const uint32_t leaf = (ob[i / 4] >> (8 * (i & 3))) & 255u;
                x[i] = tile[(int)leaf * CW + cc];
            }
#pragma unroll
            for (int s2 = 1; s2 < LPL; s2 *= 2)
#pragma unroll
                for (int i = 0; i < LPL; i += 2 * s2) x[i] = add8(x[i], x[i + s2]);
#pragma unroll
            for (int m = CW; m < 64; m *= 2) x[0] = add8(x[0], shfl_xor4(x[0], m));
            const uint4 pr = CW == 32 ? x[0] : shfl4(x[0], cc);   // leaf group 0's sum: k_hier_x2's operand order
            const uint64_t t = ht.tile_a(j);
            const int o = ht.owner_of(t);
            if (o == me && ko < kWsRing) {
                if (g == 0) res[q][ko][cc] = pr;
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot before the count
                if (lane == 0) __hip_atomic_store(&prod[q], (uint32_t)(ko + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                pushed = false;
            } else {
                uint64_t* const slot = lp.ll[o] + ((t - (uint64_t)o * ht.tpo) * W + me) * kHSlot;
#pragma unroll
                for (int r = 0; r < NWR; ++r)
                    if (wvalid(r))
                        __hip_atomic_store(slot + woff(r), h_pack(pr, wkey(r), e8), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
                pushed = true;
            }
            if (o == me) ++ko;
            if (AHEAD == 2 && j + 2 < mine) issue(ht.tile_a(j + 2), j & 1);   // this wave has read tile j
        }
        return;
    }
    // ---- B: columns CW q .. CW q + CW - 1 of the tiles' rank rows
    uint64_t* const my_ll = lp.ll[me];
    auto owned = [&](int j) { return ht.owner_of(ht.tile_a(j)) == me; };
    auto next = [&](int j, bool own) {
        while (j < mine && owned(j) != own) ++j;
        return j;
    };
    auto rows_out = [&](uint64_t t, uint4 v) {   // rows GR k + g, column CW q + cc
#pragma unroll
        for (int k = 0; k < OPS; ++k)
            st_nt(reinterpret_cast<uint4*>(ranks + (uint64_t)(GR * k + g) * stride) + t * TV + CW * q + cc, v);
    };
    auto poll = [&](const uint64_t* slot, uint64_t (&wd)[NWR]) {
#pragma unroll
        for (int r = 0; r < NWR; ++r)
            wd[r] = wvalid(r) ? __hip_atomic_load(slot + woff(r), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0;
    };
    auto fresh = [&](const uint64_t (&wd)[NWR]) {
        bool f = true;
#pragma unroll
        for (int r = 0; r < NWR; ++r) f = f && (!wvalid(r) || (uint32_t)(wd[r] >> 48) == e8);
        return f;
    };
    // the column of this lane from its three words: word k sits in round (k CW) / 64, lane (k CW) % 64 + cc
    auto gather = [&](const uint64_t (&wd)[NWR]) {
        const uint64_t a[3] = {shfl64(wd[0], cc), shfl64(wd[CW / 64], (CW % 64) + cc),
                               shfl64(wd[(2 * CW) / 64], ((2 * CW) % 64) + cc)};
        return h_unpack(a);
    };
    int jo = next(0, true), jx = next(0, false), ko = 0;
    uint64_t spin = 0, t0 = 0;
    while (jo < mine || jx < mine) {
        const uint64_t to = ht.tile_a(jo < mine ? jo : 0), tx = ht.tile_a(jx < mine ? jx : 0);
        const uint64_t li = to - (uint64_t)me * tiles_per_owner;
        const bool own_lds = ko < kWsRing;
        // one round: every word both cursors need, in flight at once
        uint64_t wr[kLLMaxGpus][NWR] = {}, wb[NWR] = {};
        if (jo < mine) {
#pragma unroll
            for (int src = 0; src < kLLMaxGpus; ++src)
                if (src < W && (src != me || !own_lds)) poll(my_ll + (li * W + src) * kHSlot, wr[src]);
        }
        if (jx < mine) poll(my_ll + box_words + tx * kHSlot, wb);
        bool moved = false;
        if (jo < mine) {
            bool f = !own_lds || __hip_atomic_load(&prod[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > (uint32_t)ko;
#pragma unroll
            for (int src = 0; src < kLLMaxGpus; ++src)
                if (src < W && (src != me || !own_lds)) f = f && fresh(wr[src]);
            if (__all(f)) {
                asm volatile("" ::: "memory");   // the slot read stays behind the count read
                uint4 y[kLLMaxGpus];
#pragma unroll
                for (int src = 0; src < kLLMaxGpus; ++src) {
                    if (src >= W) y[src] = make_uint4(0, 0, 0, 0);
                    else if (src == me && own_lds) y[src] = res[q][ko][cc];
                    else y[src] = gather(wr[src]);
                }
                const uint4 val = owner_sum(y, W, me);
#pragma unroll
                for (int dst = 0; dst < kLLMaxGpus; ++dst)
                    if (dst < W && dst != me) {
                        uint64_t* const box = lp.ll[dst] + box_words + to * kHSlot;
#pragma unroll
                        for (int r = 0; r < NWR; ++r)
                            if (wvalid(r))
                                __hip_atomic_store(box + woff(r), h_pack(val, wkey(r), e8), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                rows_out(to, val);
                ++ko;
                jo = next(jo + 1, true);
                moved = true;
            }
        }
        if (jx < mine) {
            if (__all(fresh(wb))) {
                rows_out(tx, gather(wb));
                jx = next(jx + 1, false);
                moved = true;
            }
        }
        if (moved) {
            spin = 0;   // progress: the next wait gets a bound of its own (t0 re-armed), like h_get's
        } else {
            if (peer_give_up(spin++, t0, status)) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
}

// ---- hierarchical step, two-deep bucket pipeline ----------------------------
// k_hier_x2: launch i starts bucket i (cur: tree -> partial pushed to the
// tile's owner), sums the owned tiles of bucket i-1 (mid: its W partials were
// pushed during launch i-1 -> the result is pushed to every GPU) and writes
// bucket i-2 (old: its results were pushed during launch i-1).  Every poll of
// launch i waits for pushes of launch i-1, never for one of its own launch, so
// a GPU that starts its launch late (launch jitter, a slower peer) costs the
// others nothing as long as it is less than a launch behind.  Within one
// bucket the read phase (tree -> partial) must finish on every GPU before its
// write phase (result -> 64 rank rows) can start; across buckets there is no
// such dependency, so a launch streams cur's tiles in while old's tiles go out,
// interleaved op by op as in k_tree_lds_lag.  Order in a launch:
//   L(cur 0), L(cur 1) issued (HBM busy from the start)
//   loop j:  A(cur j) [tree, partial -> owner] | S(old j - 1) stores
//            interleaved with L(cur j+2); in A(cur 0), between tile 0's tree
//            and its partial push, old's results of this workgroup's tiles
//            polled into LDS (behind a workgroup barrier, see below); before
//            the last iteration's row stores, mid's owned sums (polls of its W
//            partials, sum, result pushed to every GPU's box), so their xGMI
//            trips overlap those stores
//   fin:     (the flush launch, cur null) mid's results — pushed by the owned
//            sums of every GPU's flush launch — polled, mid's rows written
// Hand-offs per tile are ordered by the workgroup that serves the tile on every
// GPU (the same index): GPU g polls old = bucket i-2's result of tile t before
// it pushes bucket i's partial of t, and the owner reads bucket i's partials of
// t (launch i+1) before it pushes bucket i's result of t, so LL parity k & 1
// (inbox and box) is reused only after its previous reader is done.
// Any number of tiles per workgroup: with CH old's results are staged in LDS
// chunks of kHierXChunk tiles (lanes (j, c) of the whole workgroup serve tile j
// of a chunk), two chunks resident — chunk k + 1 is polled when the row stores
// of chunk k begin, into the slot chunk k - 1 left, before cur's partial of any
// of its tiles is pushed (the order above holds per tile) — and mid's owned
// sums run chunk by chunk; the launcher picks CH above kHierXChunk tiles per
// workgroup (a capped grid: processes sharing a GPU), since the bookkeeping
// costs 0.15-0.3 us at one chunk (profiles/r04_hier_x_chunk_ab.txt).
// Same bits as k_hier_ws and the launch form.  (Round-4/5 placements measured
// and retired with their tune keys in round 6, profiles/README.md: the owned
// sums at the start / the end of a launch, the result polls at the start, a
// tile's row stores in its own iteration.)
constexpr int kHierXChunk = 8;

template <bool CH>
__global__ __launch_bounds__(kBlock) void k_hier_x2(uint16_t* __restrict__ cur, uint16_t* __restrict__ old,
                                                    uint16_t* __restrict__ fin, uint64_t stride,
                                                    const uint8_t* __restrict__ order, LLPtrs lc, LLPtrs lm, LLPtrs lo,
                                                    int W, int me, uint64_t ntiles, uint64_t tiles_per_owner,
                                                    uint64_t box_words, uint32_t ecur, uint32_t emid, uint32_t eold,
                                                    int has_mid, uint32_t* status) {
    const uint32_t e8c = h_epoch(ecur), e8m = h_epoch(emid), e8o = h_epoch(eold);
    // late polls (old's results in A(cur 0)); a flush launch (no A phase) polls at its start
    const bool lp = cur != nullptr;
    constexpr int P = 64, NW = 4, TV = 32, RPI = 2, RPW = P / NW, OPS = RPW / RPI, LPL = OPS, LAG = 1;
    __shared__ __attribute__((aligned(16))) uint4 buf[2][P * TV];
    __shared__ __attribute__((aligned(16))) uint4 part[2][NW * TV];
    __shared__ __attribute__((aligned(16))) uint4 res[CH ? 2 : 1][kHierXChunk][TV];   // two chunks of results
    __shared__ __attribute__((aligned(16))) uint8_t ord_lds[ALLRED_MAX_NODES];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane % TV, q = lane / TV;
    const uint32_t wbase = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&buf[0][0] + (uint32_t)(RPW * w * TV * 16));
    const uint64_t row_off = (uint64_t)(RPW * w + q) * stride;   // + RPI * k * stride for op k
    const uint64_t G = gridDim.x;
    const int mine = blockIdx.x < ntiles ? (int)((ntiles - 1 - blockIdx.x) / G + 1) : 0;
    const int nch = CH ? (mine + kHierXChunk - 1) / kHierXChunk : (mine > 0 ? 1 : 0);
    auto tile_of = [&](int j) { return blockIdx.x + (uint64_t)j * G; };
    auto owner_of = [&](uint64_t t) { return (int)(t / tiles_per_owner); };
    auto issue = [&](uint64_t t, int b) {
#pragma unroll
        for (int k = 0; k < OPS; ++k)
            lds_dma16(reinterpret_cast<const uint4*>(cur + row_off + (uint64_t)(RPI * k) * stride) + t * TV + c,
                      wbase + (uint32_t)(b * P * TV * 16 + RPI * k * TV * 16));
    };
    // rows of tile j of bucket `dst` from its chunk's slot (lanes of wave w, half q: rows RPW w + q + RPI k)
    auto store_rows = [&](uint16_t* dst, int j) {
        const uint4 rv = CH ? res[(j / kHierXChunk) & 1][j % kHierXChunk][c] : res[0][j][c];
#pragma unroll
        for (int k = 0; k < OPS; ++k)
            st_nt(reinterpret_cast<uint4*>(dst + row_off + (uint64_t)(RPI * k) * stride) + tile_of(j) * TV + c, rv);
    };
    uint32_t ob = 0;
    if (w == 0) ob = order_byte_load(order, lane);
    if (cur && mine > 0) issue(tile_of(0), 0);
    if (cur && mine > 1) issue(tile_of(1), 1);
    if (w == 0) {   // the order byte only (the tiles' loads stay in flight)
        wait_any((cur && mine > 0 ? OPS : 0) + (cur && mine > 1 ? OPS : 0));
        asm volatile("" : "+v"(ob));   // no use of ob may move above the wait
        ord_lds[lane] = (uint8_t)ob;
    }
    // ---- lane (jr, c) (32 jr + c) serves tile jr of a chunk of this workgroup, column c
    const int jr = threadIdx.x / TV;
    auto act_in = [&](int ch) { return ch * kHierXChunk + jr < mine; };
    auto rmid_in = [&](int ch) { return has_mid && act_in(ch) && owner_of(tile_of(ch * kHierXChunk + jr)) == me; };
    // mid's owned sums of chunk ch: polls of its W partials, owner sum, pushed to every GPU's box
    auto owned_sums = [&](int ch) {
        if (!rmid_in(ch)) return;
        const uint64_t tr = tile_of(ch * kHierXChunk + jr);
        const uint64_t lr = tr - (uint64_t)me * tiles_per_owner;
        uint4 y[kLLMaxGpus];
        uint64_t wr[kLLMaxGpus][3];
#pragma unroll
        for (int src = 0; src < kLLMaxGpus; ++src)
            if (src < W) h_load(lm.ll[me] + (lr * W + src) * kHSlot, c, wr[src]);
#pragma unroll
        for (int src = 0; src < kLLMaxGpus; ++src)
            if (src < W) y[src] = h_take(wr[src], lm.ll[me] + (lr * W + src) * kHSlot, c, e8m, status);
        const uint4 o = owner_sum(y, W, me);
#pragma unroll
        for (int dst = 0; dst < kLLMaxGpus; ++dst)
            if (dst < W) h_put(lm.ll[dst] + box_words + tr * kHSlot, c, o, e8m);
    };
    // old's results of chunk ch -> its slot
    auto poll_old = [&](int ch) {
        if (!act_in(ch)) return;
        uint4& slot = res[CH ? ch & 1 : 0][jr][c];
        const uint64_t* at = lo.ll[me] + box_words + tile_of(ch * kHierXChunk + jr) * kHSlot;
        uint64_t wd[3];
        h_load(at, c, wd);
        slot = h_take(wd, at, c, e8o, status);
    };
    if (old && !lp) {   // the flush launch: old's results at the start (no A phase to hide them behind)
        poll_old(0);
        if (CH && nch > 1) poll_old(1);
    }
    lds_barrier();   // order bytes (and a flush launch's results) in LDS
    for (int j = 0; j < mine; ++j) {
        if (cur) {   // ---- A(cur j)
            // after L(j): the last row store interleaved behind it (old's tile j-2-LAG), this wave's
            // partial word of tile j-1, L(j+1), the row stores of iteration j-1 (tile j-1-LAG)
            wait_any((j >= 2 + LAG && old ? 1 : 0) + (j + 1 < mine ? OPS : 0) + (j - 1 >= LAG && old ? OPS : 0) +
                     (j >= 1 && w < 3 ? 1 : 0));
            lds_barrier();   // tile j is in LDS
            const uint4* tile = buf[j & 1];
            const uint8_t* ord = ord_lds + RPW * w + LPL * q;
            uint4 x[LPL];
#pragma unroll
            for (int i = 0; i < LPL; ++i) x[i] = tile[(int)ord[i] * TV + c];
#pragma unroll
            for (int s2 = 1; s2 < LPL; s2 *= 2)
#pragma unroll
                for (int i = 0; i < LPL; i += 2 * s2) x[i] = add8(x[i], x[i + s2]);
            const uint4 pw = add8(x[0], shfl_xor4(x[0], 32));
            if (q == 0) part[j & 1][w * TV + c] = pw;
            lds_barrier();   // partials in; every wave has read tile j out of buf[j & 1]
            // old's results of chunks 0 (and 1), ahead of this launch's first partial push (the
            // order above holds per tile); first read by iteration 1's stores, behind its A barrier
            if (j == 0 && old) {
                poll_old(0);
                if (CH && nch > 1) poll_old(1);
                // every wave's polls have read their slots before ANY wave pushes a word of this
                // launch's partials: a tile's partial words come from all four waves, and the
                // owner's inbox slot they overwrite is free only once old's result of that tile
                // exists (the owner read the slot's previous partial first).  vmcnt(0): relaxed
                // atomics to different addresses are not ordered; the barrier: the other waves
                // (only the lanes of a chunk's tiles poll).  Costs little the polls' own wait did
                // not (they were issued behind L(1)); profiles/r04_hier_latepoll_ab.txt
                wait_vm<0>();
                lds_barrier();
            }
            // the partial -> its owner's inbox: wave w < 3 writing word w of every column (one
            // store instruction; wave 3 none)
            if (q == 0) {
                const uint64_t t = tile_of(j);
                const int o = owner_of(t);
                const uint4* pp = part[j & 1];
                const uint4 pr = add8(add8(pp[0 * TV + c], pp[1 * TV + c]), add8(pp[2 * TV + c], pp[3 * TV + c]));
                const uint64_t slot = (t - (uint64_t)o * tiles_per_owner) * W + me;
                if (w < 3)
                    __hip_atomic_store(lc.ll[o] + slot * kHSlot + 32 * w + c, h_pack(pr, w, e8c), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        // mid's owned sums ahead of the last iteration's row stores, so their polls and pushes
        // overlap those stores instead of queueing behind every store of the launch
        if (j == mine - 1)
            for (int ch = 0; ch < nch; ++ch) owned_sums(ch);
        // ---- cur's tile j+2 in, old's tile j - LAG out, interleaved op by op
        const int sj = j - LAG;   // the tile whose rows this iteration stores
        if (CH && old && sj >= kHierXChunk && sj % kHierXChunk == 0) {
            // chunk sj / 8 begins: every wave is past the reads of chunk sj / 8 - 1 (A's
            // barrier, or this one in a flush launch), whose slot takes chunk sj / 8 + 1.
            // Its tiles' partials of cur are pushed in later iterations (sj + 8 > j)
            if (!cur) lds_barrier();
            poll_old(sj / kHierXChunk + 1);
        }
        const uint64_t tl = tile_of(j + 2), ts = tile_of(sj);
        const uint32_t bl = wbase + (uint32_t)((j & 1) * P * TV * 16);
        const bool st = old && sj >= 0;
        const uint4 rv = st ? (CH ? res[(sj / kHierXChunk) & 1][sj % kHierXChunk][c] : res[0][sj][c]) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < OPS; ++k) {
            if (cur && j + 2 < mine)
                lds_dma16(reinterpret_cast<const uint4*>(cur + row_off + (uint64_t)(RPI * k) * stride) + tl * TV + c,
                          bl + (uint32_t)(RPI * k * TV * 16));
            if (st) st_nt(reinterpret_cast<uint4*>(old + row_off + (uint64_t)(RPI * k) * stride) + ts * TV + c, rv);
        }
    }
    if (old && mine > 0) {   // old's last tile
        // a flush launch has no other barrier behind its chunk's poll, nor a one-tile workgroup
        // behind its late polls
        if (!cur || mine == 1) lds_barrier();
        store_rows(old, mine - 1);
    }
    if (fin) {   // ---- the flush launch: mid's results (every GPU summed its owned tiles above)
        for (int ch = 0; ch < nch; ++ch) {
            __syncthreads();   // every wave has read the slot's previous results
            if (act_in(ch))
                res[CH ? ch & 1 : 0][jr][c] = h_get(lm.ll[me] + box_words + tile_of(ch * kHierXChunk + jr) * kHSlot, c, e8m, status);
            lds_barrier();
            for (int j = ch * kHierXChunk; j < mine && j < (ch + 1) * kHierXChunk; ++j) store_rows(fin, j);
        }
    }
}

// ---------------------------------------------------------------------------
// k_peer_mem_ll: allred_mem_2D across GPUs for small buckets with LL hand-offs
// (the flat counterpart of the hierarchical forms).  A: every vector is pushed as four
// data+epoch words to its block owner's inbox; R: the owner polls the W
// copies of each of its vectors (all loads in flight at once), sums them in
// fp32 owner first then ascending, one rounding (allred_mem_2D semantics, the
// bits of k_peer_oneshot), and pushes the result into every GPU's box; B:
// every GPU polls its box and writes its bucket.  Two one-way trips, no flag,
// no remote read.  A never waits and the grid is resident (<= 128 groups), so
// every wait of R and B is reached.  LL slots of the call's parity (ll_slot
// groups): [inbox: slot q * bv + u = vector u of my block from GPU q], then,
// from the next whole group, [box: slot v = vector v of the bucket].
// ---------------------------------------------------------------------------
__host__ __device__ constexpr uint64_t ll_padded(uint64_t slots) { return (slots + 31) / 32 * 32; }

__global__ __launch_bounds__(kBlock) void k_peer_mem_ll(LLPtrs lp, int W, int me, uint16_t* __restrict__ bucket,
                                                        uint64_t nv, uint64_t bv, uint32_t epoch, uint32_t* status) {
    const uint64_t gt = gtid(), GT = gthreads();
    uint4* bk = reinterpret_cast<uint4*>(bucket);
    uint64_t* const my_ll = lp.ll[me];
    const uint64_t box = ll_padded(nv) * 4;   // words
    for (uint64_t v = gt; v < nv; v += GT) {   // A
        const int o = (int)(v / bv);
        // the owner's area by an unrolled select over the (scalar) kernarg pointers: a
        // per-lane index into lp.ll would be a vector load waiting behind every store
        uint64_t* dst = lp.ll[0];
#pragma unroll
        for (int q = 1; q < kLLMaxGpus; ++q)
            if (o == q) dst = lp.ll[q];
        ll_put(ll_slot(dst, (uint64_t)me * bv + (v - (uint64_t)o * bv)), ld_nt(bk + v), epoch);
    }
    for (uint64_t u = gt; u < bv; u += GT) {   // R: my block
        uint4 y[kLLMaxGpus];
        uint64_t t0 = 0;
        for (uint64_t spin = 0;; ++spin) {
            uint64_t wv[kLLMaxGpus][4];
#pragma unroll
            for (int q = 0; q < kLLMaxGpus; ++q) {
                const uint64_t* slot = ll_slot(my_ll, (uint64_t)(q < W ? q : 0) * bv + u);
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    wv[q][e] = q < W ? __hip_atomic_load(slot + e * kLLGroup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                     : (uint64_t)epoch << 32;
            }
            uint32_t bad = 0;
#pragma unroll
            for (int q = 0; q < kLLMaxGpus; ++q) {
#pragma unroll
                for (int e = 0; e < 4; ++e) bad |= (uint32_t)(wv[q][e] >> 32) ^ epoch;
                y[q] = make_uint4((uint32_t)wv[q][0], (uint32_t)wv[q][1], (uint32_t)wv[q][2], (uint32_t)wv[q][3]);
            }
            if (bad == 0) break;
            if (peer_give_up(spin, t0, status)) break;
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
        for (int q = 0; q < W; ++q) ll_put(ll_slot(lp.ll[q] + box, v), r, epoch);
    }
    for (uint64_t v = gt; v < nv; v += GT) st_nt(bk + v, ll_get(ll_slot(my_ll + box, v), epoch, status));   // B
}

// ---------------------------------------------------------------------------
// k_peer_lo_ll: the LO program of allred_peer_dist_allreduce (one channel)
// for small buckets with LL hand-offs: step k, every lane pushes its 16 bytes
// as four self-validating 8-byte words (4 data bytes + the call's epoch) into
// partner p_k's step-k slot, then polls its OWN step-k slot until the four
// words of p_k carry the epoch, and adds (one bf16 rounding, the same add as
// every LO form).  Per step one one-way xGMI trip instead of k_peer_sched's
// progress flag + remote read round trip; no window, no flag area.  Slot of
// step k, vector v: k * ll_padded(nv) + v (ll_slot groups) in the LL area of
// the call's parity; call k+2 may reuse a parity because finishing call k+1
// needs every rank to have started it (the partners of all steps reach every
// rank of the schedule).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_peer_lo_ll(LLPtrs lp, PeerProg pr, int me, uint16_t* __restrict__ bucket,
                                                       uint64_t nv, uint32_t epoch, uint32_t* status) {
    const uint64_t v = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (v >= nv) return;
    uint4* bk = reinterpret_cast<uint4*>(bucket);
    uint4 cur = ld_nt(bk + v);
    const uint64_t* mine = lp.ll[me];
    const uint64_t per_step = ll_padded(nv);   // slots
    for (int k = 0; k < pr.S; ++k) {
        const int p = pr.peer[0][k];
        ll_put(ll_slot(lp.ll[p], (uint64_t)k * per_step + v), cur, epoch);
        cur = add8(cur, ll_get(ll_slot(mine, (uint64_t)k * per_step + v), epoch, status));
    }
    st_nt(bk + v, cur);
}

int peer_last_error() { return hip_status((int)hipGetLastError()); }

// Workgroups of `func` (block threads) resident on the current device at once: the grid cap of
// the hierarchical forms, whose workgroups wait for each other across GPUs (every one must be
// resident).  512 on a whole MI355X (2 per CU x 256 CUs: 73.7 KiB of LDS each); fewer on a
// partitioned GPU, where a 512-workgroup grid would wait for workgroups that cannot start.
// Cached per (device, kernel); 0 when the runtime cannot say (the caller keeps its cap).
unsigned resident_limit(const void* func, int block) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    static std::mutex mu;
    static std::map<std::pair<int, const void*>, unsigned> cache;
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair(dev, func);
    const auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int cus = 0, per = 0;
    unsigned lim = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, func, block, 0) == hipSuccess && cus > 0 && per > 0)
        lim = (unsigned)cus * (unsigned)per;
    cache.emplace(key, lim);
    return lim;
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
    int rc = launch_copy_ranks(bucket, 0, wins[me], 0, 1, n, stream);
    if (rc != ALLRED_OK) return rc;
    // 2. everyone's window is written
    hipLaunchKernelGGL(k_peer_barrier, dim3(1), dim3(64), 0, st, pp, nranks, me, epoch, status);
    // 3. reduce my block from every window
    hipLaunchKernelGGL(k_peer_rs, dim3(grid_all(bv)), dim3(kBlock), 0, st, pp, nranks, me, bucket, bv);
    // 4. every block is reduced
    hipLaunchKernelGGL(k_peer_barrier, dim3(1), dim3(64), 0, st, pp, nranks, me, epoch + 1, status);
    // 5. gather the other blocks
    hipLaunchKernelGGL(k_peer_ag, dim3(grid_all(bv), nranks), dim3(kBlock), 0, st, pp, me, bucket, bv);
    return peer_last_error();
}

int launch_peer_barrier(uint32_t* const* flags, int nranks, int me, uint32_t epoch, uint32_t* status, void* stream) {
    if (nranks > ALLRED_MAX_NODES) return ALLRED_ERR_ARG;
    PeerPtrs pp{};
    for (int q = 0; q < nranks; ++q) pp.flags[q] = flags[q];
    hipLaunchKernelGGL(k_peer_barrier, dim3(1), dim3(64), 0, (hipStream_t)stream, pp, nranks, me, epoch, status);
    return peer_last_error();
}

int launch_peer_sched(uint16_t* const* wins, uint32_t* const* flags, int me, uint16_t* bucket, const PeerProg& prog,
                      uint64_t half_vec, uint32_t base_epoch, uint32_t* status, unsigned max_groups, void* stream) {
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
    // workgroup g waits for workgroup g of its partners: every GPU's grid must be resident
    // at once (max_groups < kPeerSchedMaxGroups when processes share one GPU)
    uint64_t cap = max_groups && max_groups < kPeerSchedMaxGroups ? max_groups : kPeerSchedMaxGroups;
    const uint64_t res = resident_limit(reinterpret_cast<const void*>(&k_peer_sched), kBlock);   // all resident
    if (res && cap > res) cap = res;
    const uint64_t gmax = cap / prog.C > 0 ? cap / prog.C : 1;
    if (gc > gmax) gc = gmax;
    if (gc < 1) gc = 1;
    PeerProg pf = prog;
    pf.fence = (int)tune(Tune::peer_fence);
    hipLaunchKernelGGL(k_peer_sched, dim3((unsigned)(gc * prog.C)), dim3(kBlock), 0, (hipStream_t)stream, pp, pf, me,
                       bucket, half_vec, base_epoch, status);
    return peer_last_error();
}

int launch_peer_sched_push(uint16_t* const* wins, uint16_t* const* stages, uint32_t* const* flags, int me,
                           uint16_t* bucket, const PeerProg& prog, uint32_t base_epoch, uint32_t* status,
                           unsigned max_groups, void* stream) {
    if (!aligned16(bucket) || prog.lo || prog.N > ALLRED_MAX_NODES || prog.C < 1 || prog.C > kPeerMaxChannels ||
        prog.S > kPeerMaxSteps)
        return ALLRED_ERR_ARG;
    PeerPtrs pp{};
    PeerStage ps{};
    for (int q = 0; q < prog.N; ++q) {
        pp.win[q] = wins[q];
        pp.flags[q] = flags[q];
        ps.st[q] = stages[q];
    }
    uint64_t per = 0;
    for (int c = 0; c < prog.C; ++c) per = prog.len[c] / prog.N > per ? prog.len[c] / prog.N : per;
    uint64_t gc = (per + kBlock - 1) / kBlock;
    uint64_t cap = max_groups && max_groups < kPeerSchedMaxGroups ? max_groups : kPeerSchedMaxGroups;
    const uint64_t res = resident_limit(reinterpret_cast<const void*>(&k_peer_sched_push), kBlock);   // all resident
    if (res && cap > res) cap = res;
    const uint64_t gmax = cap / prog.C > 0 ? cap / prog.C : 1;
    if (gc > gmax) gc = gmax;
    if (gc < 1) gc = 1;
    PeerProg pf = prog;
    pf.fence = (int)tune(Tune::peer_fence);
    hipLaunchKernelGGL(k_peer_sched_push, dim3((unsigned)(gc * prog.C)), dim3(kBlock), 0, (hipStream_t)stream, pp, ps,
                       pf, me, bucket, base_epoch, status);
    return peer_last_error();
}

int launch_peer_mem_ll(uint64_t* const* ll, int nranks, int me, uint16_t* bucket, size_t n, uint64_t area_words,
                       uint32_t epoch, uint32_t* status, unsigned max_groups, void* stream) {
    const uint64_t nv = n / 8;
    if (n % (8 * (size_t)nranks) || !aligned16(bucket) || nranks > kLLMaxGpus || 8 * ll_padded(nv) > area_words)
        return ALLRED_ERR_ARG;
    LLPtrs lp{};
    for (int q = 0; q < nranks; ++q) lp.ll[q] = ll[q];
    uint64_t groups = (nv + kBlock - 1) / kBlock;
    uint64_t cap = max_groups && max_groups < kPeerFusedMaxGroups ? max_groups : kPeerFusedMaxGroups;
    const uint64_t res = resident_limit(reinterpret_cast<const void*>(&k_peer_mem_ll), kBlock);   // all resident
    if (res && cap > res) cap = res;
    if (groups > cap) groups = cap;   // resident: every wait is reached
    hipLaunchKernelGGL(k_peer_mem_ll, dim3((unsigned)groups), dim3(kBlock), 0, (hipStream_t)stream, lp, nranks, me,
                       bucket, nv, nv / nranks, epoch, status);
    return peer_last_error();
}

int launch_peer_lo_ll(uint64_t* const* ll, int nranks, int me, uint16_t* bucket, const PeerProg& prog, size_t n,
                      uint64_t area_words, uint32_t epoch, uint32_t* status, void* stream) {
    const uint64_t nv = n / 8;
    if (n % 8 || !aligned16(bucket) || nranks > kLLMaxGpus || !prog.lo || prog.C != 1 ||
        ll_padded(nv) * 4 * (uint64_t)prog.S > area_words)
        return ALLRED_ERR_ARG;
    LLPtrs lp{};
    for (int q = 0; q < nranks; ++q) lp.ll[q] = ll[q];
    hipLaunchKernelGGL(k_peer_lo_ll, dim3((unsigned)((nv + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       (hipStream_t)stream, lp, prog, me, bucket, nv, epoch, status);
    return peer_last_error();
}

int launch_hier_ws(uint16_t* ranks, uint64_t stride, const uint8_t* order, uint64_t* const* ll, int nranks, int me,
                   size_t n, uint64_t box_words, uint32_t epoch, uint32_t* status, unsigned max_grid,
                   void* stream) {
    const uint64_t nv = n / 8, ntiles = nv / 32;
    if (nranks < 1 || nranks > kLLMaxGpus || nv % 32 || ntiles % nranks || stride % 8 || !aligned16(ranks) ||
        ntiles * kHSlot > box_words)
        return ALLRED_ERR_ARG;
    LLPtrs lp{};
    for (int q = 0; q < nranks; ++q) lp.ll[q] = ll[q];
    const bool a2 = tune(Tune::hier_ws_ahead) == 2;
    const int cw = tune(Tune::hier_ws_cols) >= 32 ? 32 : tune(Tune::hier_ws_cols) >= 16 ? 16 : 8;
    decltype(&k_hier_ws<1, 8>) kern = cw == 32 ? (a2 ? k_hier_ws<2, 32> : k_hier_ws<1, 32>)
                                      : cw == 16 ? (a2 ? k_hier_ws<2, 16> : k_hier_ws<1, 16>)
                                                 : (a2 ? k_hier_ws<2, 8> : k_hier_ws<1, 8>);
    // 2 per CU: the whole grid resident (max_grid < 512 when processes share the GPU; fewer
    // where the device holds fewer at once)
    unsigned cap = max_grid && max_grid < 512 ? max_grid : 512;
    const unsigned res = resident_limit(reinterpret_cast<const void*>(kern), 128 * (32 / cw));
    if (res && cap > res) cap = res;
    const unsigned grid = (unsigned)(ntiles < cap ? ntiles : cap);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(128 * (32 / cw)), 0, (hipStream_t)stream, ranks, stride, order, lp, nranks, me,
                       ntiles, ntiles / nranks, box_words, epoch, status);
    static const char* const names[2][3] = {{"k_hier_ws<1, 8>", "k_hier_ws<1, 16>", "k_hier_ws<1, 32>"},
                                            {"k_hier_ws<2, 8>", "k_hier_ws<2, 16>", "k_hier_ws<2, 32>"}};
    note_launch(reinterpret_cast<const void*>(kern), names[a2 ? 1 : 0][cw == 8 ? 0 : cw == 16 ? 1 : 2], grid,
                128 * (32 / cw));
    return peer_last_error();
}

int launch_hier_x2(uint16_t* cur, uint16_t* old, uint16_t* fin, uint64_t stride, const uint8_t* order,
                   uint64_t* const* llc, uint64_t* const* llm, uint64_t* const* llo, int nranks, int me, size_t n,
                   uint64_t box_words, uint32_t ecur, uint32_t emid, uint32_t eold, uint32_t* status,
                   unsigned max_grid, void* stream) {
    const uint64_t nv = n / 8, ntiles = nv / 32;
    if (nranks < 1 || nranks > kLLMaxGpus || nv % 32 || ntiles % nranks || stride % 8 || ntiles * kHSlot > box_words ||
        (!cur && !old && !fin) || (cur && !llc) || (old && !llo) || (fin && (cur || !llm)) ||
        (cur && !aligned16(cur)) || (old && !aligned16(old)) || (fin && !aligned16(fin)))
        return ALLRED_ERR_ARG;
    // 2 per CU: the whole grid resident (max_grid < 512 when processes share the GPU; fewer
    // where the device holds fewer at once — the chunked form's LDS, the larger, decides)
    unsigned cap = max_grid && max_grid < 512 ? max_grid : 512;
    const unsigned res = resident_limit(reinterpret_cast<const void*>(&k_hier_x2<true>), kBlock);
    if (res && cap > res) cap = res;
    const unsigned grid = (unsigned)(ntiles < cap ? ntiles : cap);
    LLPtrs lc{}, lm{}, lo{};
    for (int q = 0; q < nranks; ++q) {
        lc.ll[q] = llc ? llc[q] : nullptr;
        lm.ll[q] = llm ? llm[q] : nullptr;
        lo.ll[q] = llo ? llo[q] : nullptr;
    }
    // the chunked form only where a workgroup has more than one chunk of tiles
    const bool ch = (ntiles + grid - 1) / grid > (uint64_t)kHierXChunk;
    decltype(&k_hier_x2<false>) kern = ch ? k_hier_x2<true> : k_hier_x2<false>;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, cur, old, fin, stride, order, lc, lm, lo, nranks, me, ntiles, ntiles / nranks,
                       box_words, ecur, emid, eold, llm ? 1 : 0, status);
    if (cur) note_launch(reinterpret_cast<const void*>(kern), ch ? "k_hier_x2<chunked>" : "k_hier_x2", grid, kBlock);
    return peer_last_error();
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
    const uint64_t res = resident_limit(reinterpret_cast<const void*>(&k_peer_oneshot), kBlock);   // all resident
    if (res && groups > res) groups = res;
    if (groups < 1) groups = 1;
    const uint64_t chunk = (bv + groups - 1) / groups;
    hipLaunchKernelGGL(k_peer_oneshot, dim3((unsigned)groups), dim3(kBlock), 0, (hipStream_t)stream, pp, nranks, me,
                       bucket, bv, chunk, epoch, status, (uint32_t)tune(Tune::peer_fence));
    return peer_last_error();
}

}  // namespace tsa
