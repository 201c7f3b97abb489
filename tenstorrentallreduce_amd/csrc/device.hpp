// device.hpp — CDNA4 (gfx950) device helpers shared by the engine's kernels
// (kernels.hip: virtual-rank plans; peer_kernels.hip: across GPUs) and by the
// micro-benchmarks under tools/ubench/.
//
// bf16 arithmetic: unpack to fp32 (<< 16), add in fp32, pack back with the
// gfx950 v_cvt_pk_bf16_f32 (round to nearest even) — one rounding per add, the
// Tensix add_tiles + pack_tile<true> of allred_BO_2D/kernels/compute_kernel.cpp:53-60
// with fp32_dest_acc_en = false (allred_helper.cpp:331-335).
// Memory: 16-byte (8 x bf16) accesses per lane, nontemporal where a byte is
// touched once per pass; LDS-DMA (global_load_lds_dwordx4) issued from inline
// asm with exact s_waitcnt vmcnt(n) accounting.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

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

// one mem_2D accumulation step: fp32 (rounded once at the end, the default) or
// ACC16, the reference's bf16 dest register (fp32_dest_acc_en = false,
// allred_helper.cpp:331-335): every add rounded to bf16, nearest even
template <bool ACC16>
__device__ __forceinline__ float acc_add(float a, float y) {
    const float s = a + y;
    return ACC16 ? lo_f(pack_rne(s, 0.0f)) : s;
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
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
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
// Exact vmcnt waits.  CDNA3/4 count VMEM loads, LDS-DMA loads and stores on
// one in-order counter, so "wait until this tile's loads have landed" is
// s_waitcnt vmcnt(n) with n = the ops issued after them; the pipelined kernels
// keep later loads and earlier stores in flight that way.
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

// the 64-byte tree order, one byte per lane of wave 0, loaded by inline asm: the
// compiler would follow its own load with vmcnt(0) before staging it, so the
// tiles' LDS-DMA loads (invisible to it) would wait behind the order's round
// trip; here they go out right behind it and only the byte is waited for
__device__ __forceinline__ uint32_t order_byte_load(const uint8_t* order, int lane) {
    uint32_t b;
    asm volatile("global_load_ubyte %0, %1, off" : "=v"(b) : "v"(order + lane) : "memory");
    return b;
}

// workgroup barrier without the release fence of __syncthreads (which waits
// vmcnt(0)); LDS traffic is ordered by the lgkmcnt wait
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// bounded waits of the peer kernels: a wait gives up after kPeerWaitTicks of
// the 100 MHz s_memrealtime clock (4 s, far above any legitimate skew between
// ranks; a poll count is no clock — polls of uncached memory took ~50-200 ns,
// so round 3's 2^22-poll bound expired in well under a second when several
// ranks' grids time-sliced one GPU).  The clock is read every 64 polls.  On
// timeout bit 0 of *status is set; every later wait of the launch sees that
// bit (checked with the clock) and gives up at once, so a dead or slow peer
// ends the launch within seconds instead of paying the bound once per wait.
constexpr uint64_t kPeerWaitTicks = 400000000ull;

__device__ __forceinline__ bool peer_give_up(uint64_t spin, uint64_t& t0, uint32_t* status) {
    if (spin & 63u) return false;
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (spin == 0) {
        t0 = now;
        return false;
    }
    if (now - t0 > kPeerWaitTicks ||
        (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ALLRED_PEER_TIMEOUT)) {
        atomicOr(status, ALLRED_PEER_TIMEOUT);
        return true;
    }
    return false;
}

}  // namespace
}  // namespace tsa
