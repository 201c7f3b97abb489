/*
 * allred_oracle.c — CPU ORACLE (test infrastructure only; see allred_oracle.h).
 *
 * Plain-C restatement of the reference allreduce.  Every function cites the
 * reference file:line it restates.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use this file, as the checker / CPU baseline;
 * the product never links it.
 */
#define _GNU_SOURCE
#include "allred_oracle.h"

#include <errno.h>
#include <linux/futex.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

/* ===================================================================== */
/* bf16                                                                   */
/* ===================================================================== */
static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

float or_bf16_to_float(uint16_t h) { return u2f((uint32_t)h << 16); }

uint16_t or_bf16_rne(float f) {
    uint32_t u = f2u(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x0040u); /* quiet NaN */
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

/* tt-metal bfloat16(float) of the v0.5x era: keep the upper 16 bits. */
uint16_t or_bf16_trunc(float f) { return (uint16_t)(f2u(f) >> 16); }

/* Tensix add_tiles (allred_BO_2D/kernels/compute_kernel.cpp:55, HiFi4,
 * fp32_dest_acc_en=false, allred_helper.cpp:331-335): one bf16 result per add.
 * Rounding restated as fp32 add then round-to-nearest-even. */
uint16_t or_bf16_add(uint16_t a, uint16_t b) {
    volatile float s = or_bf16_to_float(a) + or_bf16_to_float(b);
    return or_bf16_rne(s);
}

/* ===================================================================== */
/* mt19937 + libstdc++ uniform_real_distribution<float>                   */
/* (tt-metal create_random_vector_of_bfloat16, called at                  */
/*  allred_helper.cpp:283-284; tt-metal is not vendored: restated from    */
/*  its published algorithm and pinned by tests/golden/inputs_ref.json)  */
/* ===================================================================== */
typedef struct { uint32_t mt[624]; int idx; } mt19937;

static void mt_seed(mt19937* g, uint32_t seed) {
    g->mt[0] = seed;
    for (int i = 1; i < 624; ++i)
        g->mt[i] = 1812433253u * (g->mt[i - 1] ^ (g->mt[i - 1] >> 30)) + (uint32_t)i;
    g->idx = 624;
}

static uint32_t mt_next(mt19937* g) {
    if (g->idx >= 624) {
        for (int i = 0; i < 624; ++i) {
            uint32_t y = (g->mt[i] & 0x80000000u) | (g->mt[(i + 1) % 624] & 0x7fffffffu);
            uint32_t v = g->mt[(i + 397) % 624] ^ (y >> 1);
            if (y & 1u) v ^= 0x9908b0dfu;
            g->mt[i] = v;
        }
        g->idx = 0;
    }
    uint32_t y = g->mt[g->idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

/* std::generate_canonical<float, 24> (libstdc++ random.tcc) then
 * uniform_real_distribution<float>(0, b): canon * (b - 0) + 0, in float. */
static float uniform_float(mt19937* g, float b) {
    volatile float sum = (float)mt_next(g);
    volatile float canon = sum / 4294967296.0f;
    if (canon >= 1.0f) canon = nextafterf(1.0f, 0.0f);
    volatile float prod = canon * b;
    return prod + 0.0f;
}

void or_random_bf16_vector(size_t num_bytes, int rand_max, int seed, int round_mode, uint32_t* out) {
    mt19937 g;
    mt_seed(&g, (uint32_t)seed);
    size_t words = num_bytes / 4;
    for (size_t i = 0; i < words; ++i) {
        float f1 = uniform_float(&g, (float)rand_max);
        float f2 = uniform_float(&g, (float)rand_max);
        uint16_t h1 = round_mode ? or_bf16_rne(f1) : or_bf16_trunc(f1);
        uint16_t h2 = round_mode ? or_bf16_rne(f2) : or_bf16_trunc(f2);
        out[i] = (uint32_t)h1 | ((uint32_t)h2 << 16);
    }
}

void or_constant_bf16_vector(size_t num_bytes, float value, uint32_t* out) {
    uint16_t h = or_bf16_trunc(value);
    size_t words = num_bytes / 4;
    for (size_t i = 0; i < words; ++i) out[i] = (uint32_t)h | ((uint32_t)h << 16);
}

/* ===================================================================== */
/* schedule                                                               */
/* ===================================================================== */
/* allred_helper.cpp:122-133 */
int or_highest_power_of_two(int v) {
    int p = 1;
    while (p < 8 && 2 * p <= v) p *= 2;
    return p;
}

/* allred_helper.cpp:136-142 : per-step NoC choice from (x, y) parity */
uint32_t or_step_directions(int x, int y) {
    static const uint32_t tbl[2][2] = {{0x33u, 0x19u}, {0x26u, 0x0cu}}; /* [x%2][y%2] */
    return tbl[x & 1][y & 1];
}

int or_steps(int total) {
    int s = 0;
    while ((1 << s) < total) ++s;
    return s;
}

/* Swing distance rho(k) = (1 - (-2)^(k+1)) / 3 : 1, -1, 3, -5, 11, ... */
static int swing_rho(int k) {
    int p = 1;
    for (int i = 0; i <= k; ++i) p *= -2;
    return (1 - p) / 3;
}

/* allred_helper.cpp:166-191. Even steps move inside the row (direction from
 * node parity, wrap by one row length); odd steps move between rows
 * (direction from row parity, wrap modulo total). */
int or_partner_swing(int node, int step, int side, int total) {
    int row = node / side;
    int d = swing_rho(step / 2);
    int p;
    if (step % 2 == 0) {
        p = (node % 2 == 0) ? node + d : node - d;
        if (p < 0 || p / side < row) p += side;
        else if (p / side > row) p -= side;
    } else {
        p = (row % 2 == 0) ? node + side * d : node - side * d;
        if (p < 0) p += total;
        else if (p >= total) p -= total;
    }
    return p;
}

/* allred_helper.cpp:145-163 with the caller's bookkeeping of
 * allred_BO_2D.cpp:98-127: horizontal on even steps, depth doubles after
 * every vertical step. */
int or_partner_recdub(int node, int step, int side, int* sends_se) {
    int depth = 1 << (step / 2);
    int horizontal = (step % 2 == 0);
    int row = node / side, col = node % side;
    int pos = horizontal ? col : row;
    int se = (pos % (2 * depth)) < depth;
    if (sends_se) *sends_se = se;
    int q = pos + (se ? depth : -depth);
    return horizontal ? row * side + q : q * side + col;
}

/* scratch_work/all_red_swing_1D/all_red_swing_1D.cpp:32-36 */
int or_partner_swing_1d(int node, int step, int total) {
    int d = swing_rho(step);
    int p = (node % 2 == 0) ? node + d : node - d;
    return (p + total) % total;
}

/* scratch_work/recdub_multicore_1D/recdub_multicore_1D.cpp:165-175 */
int or_partner_recdub_1d(int node, int step, int* sends_se) {
    int depth = 1 << step;
    int se = (node % (2 * depth)) < depth;
    if (sends_se) *sends_se = se;
    return se ? node + depth : node - depth;
}

/* algo: 0 RecDub 2D, 1 Swing 2D, 2 RecDub 1D, 3 Swing 1D */
static int partner_of(int swing, int node, int step, int side, int total) {
    switch (swing) {
        case 1: return or_partner_swing(node, step, side, total);
        case 2: return or_partner_recdub_1d(node, step, NULL);
        case 3: return or_partner_swing_1d(node, step, total);
        default: return or_partner_recdub(node, step, side, NULL);
    }
}

/* allred_BO_2D.cpp:220-270 restated without recursion: the set of nodes
 * reachable from `node` by partner hops taken at strictly increasing steps
 * >= `from_step` (the recursion ORs exactly that set; the node itself is
 * included here because the caller ORs it in, allred_BO_2D.cpp:111-124). */
static uint64_t reach(int swing, int node, int from_step, int side, int total, int steps, int* bad) {
    uint64_t set = 1ull << node;
    for (int s = from_step; s < steps; ++s) {
        uint64_t add = 0;
        for (int v = 0; v < total; ++v) {
            if (!((set >> v) & 1ull)) continue;
            int p = partner_of(swing, v, s, side, total);
            if (p < 0 || p >= total) { *bad = 1; continue; }
            add |= 1ull << p;
        }
        set |= add;
    }
    return set;
}

int or_build_schedule(int swing, int side, int total, or_schedule* s) {
    memset(s, 0, sizeof(*s));
    if (swing >= 2) side = total;
    s->swing = swing; s->side = side; s->total = total; s->steps = or_steps(total);
    if (total < 1 || total > OR_MAX_NODES || side < 1 || (total & (total - 1))) return -1;
    int bad = 0;
    for (int r = 0; r < total; ++r) {
        uint32_t dirs = 0;
        for (int k = 0; k < s->steps; ++k) {
            int se = 0;
            int p = swing == 1 ? or_partner_swing(r, k, side, total)
                    : swing == 2 ? or_partner_recdub_1d(r, k, &se)
                    : swing == 3 ? or_partner_swing_1d(r, k, total)
                                 : or_partner_recdub(r, k, side, &se);
            s->partner[r][k] = p;
            if ((swing == 0 || swing == 2) && se) dirs |= 1u << k;
            if (p < 0 || p >= total) { bad = 1; continue; }
            s->send[r][k] = reach(swing, p, k + 1, side, total, s->steps, &bad);
            s->recv[r][k] = reach(swing, r, k + 1, side, total, s->steps, &bad);
        }
        s->dirs[r] = swing == 1 ? (or_step_directions(r % side, r / side) & ((1u << s->steps) - 1u))
                     : swing == 3 ? 0u : dirs;
    }
    return bad ? -1 : 0;
}

/* allred_helper.cpp:224-234 */
int or_normalize_tiles(int tiles, int total_nodes, int large_buffer) {
    if (tiles < 1) tiles = 1;
    if (large_buffer) return tiles * total_nodes;
    if (tiles < 64) {
        int p = 1;
        while (p < tiles) p <<= 1;
        return p;
    }
    return ((tiles + 63) / 64) * 64;
}

/* ===================================================================== */
/* data-path simulations                                                  */
/* ===================================================================== */
/* Reduce-scatter (dataflow_kernel.cpp:152-213 + compute_kernel.cpp:35-67):
 * each step, every rank receives its partner's blocks named by its recv mask
 * into a recv buffer and adds recv into local tile by tile.  All-gather
 * (dataflow_kernel.cpp:219-267): steps in reverse, each rank writes the
 * blocks of its recv mask into the partner's local buffer. */
int or_allreduce_bo(const or_schedule* s, uint16_t** ranks, size_t n) {
    int N = s->total;
    if (n % (size_t)N) return -1;
    size_t blk = n / (size_t)N;
    uint16_t** recv = (uint16_t**)calloc((size_t)N, sizeof(uint16_t*));
    for (int r = 0; r < N; ++r) recv[r] = (uint16_t*)malloc(n * 2);
    for (int k = 0; k < s->steps; ++k) {
        /* send phase: partner p writes its local blocks of recv mask(r) into recv[r] */
        for (int r = 0; r < N; ++r) {
            int p = s->partner[r][k];
            for (int b = 0; b < N; ++b)
                if ((s->recv[r][k] >> b) & 1ull)
                    memcpy(recv[r] + b * blk, ranks[p] + b * blk, blk * 2);
        }
        /* compute phase */
        for (int r = 0; r < N; ++r)
            for (int b = 0; b < N; ++b)
                if ((s->recv[r][k] >> b) & 1ull)
                    for (size_t e = b * blk; e < (b + 1) * blk; ++e)
                        ranks[r][e] = or_bf16_add(ranks[r][e], recv[r][e]);
    }
    for (int k = s->steps - 1; k >= 0; --k) {
        /* write phase into a snapshot so the step is simultaneous */
        for (int r = 0; r < N; ++r) memcpy(recv[r], ranks[r], n * 2);
        for (int r = 0; r < N; ++r) {
            int p = s->partner[r][k];
            for (int b = 0; b < N; ++b)
                if ((s->recv[r][k] >> b) & 1ull)
                    memcpy(ranks[p] + b * blk, recv[r] + b * blk, blk * 2);
        }
    }
    for (int r = 0; r < N; ++r) free(recv[r]);
    free(recv);
    return 0;
}

/* LO: every step exchanges the full vector (shouldSendBlock with
 * bandwidth_optimal = 0, dataflow_kernel.cpp:19-29; LOO kernel
 * allred_LOO_2D/kernels/dataflow_kernel.cpp:133-170) and adds it. */
int or_allreduce_lo(const or_schedule* s, uint16_t** ranks, size_t n) {
    int N = s->total;
    uint16_t** recv = (uint16_t**)calloc((size_t)N, sizeof(uint16_t*));
    for (int r = 0; r < N; ++r) recv[r] = (uint16_t*)malloc(n * 2);
    for (int k = 0; k < s->steps; ++k) {
        for (int r = 0; r < N; ++r) memcpy(recv[r], ranks[s->partner[r][k]], n * 2);
        for (int r = 0; r < N; ++r)
            for (size_t e = 0; e < n; ++e) ranks[r][e] = or_bf16_add(ranks[r][e], recv[r][e]);
    }
    for (int r = 0; r < N; ++r) free(recv[r]);
    free(recv);
    return 0;
}

/* mem_2D (allred_mem_2D/kernels/dataflow_kernel.cpp:133-188,
 * compute_kernel.cpp:43-72): block b is reduced by rank b from the common
 * buffer.  Intended semantics: seed with the OWN block, then add
 * the other ranks' copies of block b in rank order; the accumulation is kept
 * in fp32 and rounded once (the MI355X design).  Then every
 * rank reads the whole reduced vector back. */
/* acc16 = 1: the reference's own accumulation register instead — the Tensix
 * dest holds bf16 (fp32_dest_acc_en = false, allred_helper.cpp:331-335), so
 * every binary_dest_reuse_tiles add (allred_mem_2D/kernels/compute_kernel.cpp:51-60)
 * rounds the running sum to bf16 (nearest even here, like every other add). */
int or_allreduce_mem_acc(int N, uint16_t** ranks, size_t n, int acc16) {
    if (n % (size_t)N) return -1;
    size_t blk = n / (size_t)N;
    uint16_t* dst = (uint16_t*)malloc(n * 2);
    for (int b = 0; b < N; ++b)
        for (size_t e = b * blk; e < (b + 1) * blk; ++e) {
            volatile float acc = or_bf16_to_float(ranks[b][e]);
            for (int r = 0; r < N; ++r) {
                if (r == b) continue;
                acc = acc + or_bf16_to_float(ranks[r][e]);
                if (acc16) acc = or_bf16_to_float(or_bf16_rne(acc));
            }
            dst[e] = or_bf16_rne(acc);
        }
    for (int r = 0; r < N; ++r) memcpy(ranks[r], dst, n * 2);
    free(dst);
    return 0;
}

int or_allreduce_mem(int N, uint16_t** ranks, size_t n) { return or_allreduce_mem_acc(N, ranks, n, 0); }

/* ===================================================================== */
/* validation (allred_helper.cpp:18-120)                                  */
/* ===================================================================== */
long or_validate(const uint32_t* result, const uint32_t* src0, const uint32_t* src1, size_t num_els,
                 float error, uint32_t total_nodes, int trgt_mode, float* max_err_out) {
    long bad = 0;
    float max_err = 0.0f;
    float mult = (float)(total_nodes / 2); /* integer division, as :43 */
    for (size_t i = 0; i < num_els * 2; ++i) {
        size_t w = i / 2;
        int hi = (int)(i & 1);
        uint16_t r = (uint16_t)(hi ? result[w] >> 16 : result[w] & 0xffffu);
        uint16_t a = (uint16_t)(hi ? src0[w] >> 16 : src0[w] & 0xffffu);
        uint16_t b = (uint16_t)(hi ? src1[w] >> 16 : src1[w] & 0xffffu);
        volatile float sum = or_bf16_to_float(a) + or_bf16_to_float(b);
        volatile float t = sum * mult;
        uint16_t tb = trgt_mode ? or_bf16_rne(t) : or_bf16_trunc(t);
        float diff = fabsf(or_bf16_to_float(r) - or_bf16_to_float(tb));
        if (diff > error) {
            ++bad;
            if (diff > max_err) max_err = diff;
        }
    }
    if (max_err_out) *max_err_out = max_err;
    return bad;
}

/* ===================================================================== */
/* loopback multi-process restatement                                     */
/* ===================================================================== */
static long futex(volatile uint32_t* addr, int op, uint32_t val) {
    return syscall(SYS_futex, (uint32_t*)addr, op, val, NULL, NULL, 0);
}

static void sem_inc(volatile uint32_t* w) {
    __atomic_add_fetch(w, 1u, __ATOMIC_RELEASE);
    futex(w, FUTEX_WAKE, 0x7fffffff);
}

static void sem_wait_min(volatile uint32_t* w, uint32_t v) {
    for (int spin = 0;; ++spin) {
        uint32_t cur = __atomic_load_n(w, __ATOMIC_ACQUIRE);
        if (cur >= v) return;
        if (spin < 64) continue;
        futex(w, FUTEX_WAIT, cur);
    }
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* per-rank control block in shared memory, one cache line per word group */
typedef struct {
    volatile uint32_t sem0[8];   /* per-step handshake (semaphore_0[i % 6]) */
    volatile uint32_t sem1;      /* RS data-ready counter (semaphore_1[0]) */
    volatile uint32_t sem_ag;    /* AG completion counter (semaphore_1[i % 2]) */
    uint32_t pad[6];
    double t_start, t_end;
} rank_ctl;

typedef struct {
    volatile uint32_t arrive;
    volatile uint32_t gen;
} shm_barrier;

static void barrier_wait(shm_barrier* b, uint32_t n) {
    uint32_t g = __atomic_load_n(&b->gen, __ATOMIC_ACQUIRE);
    if (__atomic_add_fetch(&b->arrive, 1u, __ATOMIC_ACQ_REL) == n) {
        __atomic_store_n(&b->arrive, 0u, __ATOMIC_RELAXED);
        __atomic_add_fetch(&b->gen, 1u, __ATOMIC_RELEASE);
        futex(&b->gen, FUTEX_WAKE, 0x7fffffff);
        return;
    }
    while (__atomic_load_n(&b->gen, __ATOMIC_ACQUIRE) == g) futex(&b->gen, FUTEX_WAIT, g);
}

static void add_range(uint16_t* dst, const uint16_t* src, size_t n) {
    for (size_t e = 0; e < n; ++e) dst[e] = or_bf16_add(dst[e], src[e]);
}

/* One rank of the BO / LO dataflow (allred_BO_2D/kernels/dataflow_kernel.cpp
 * and allred_LOO_2D/kernels/dataflow_kernel.cpp), sender and monitor roles
 * folded into one process; the compute kernel's add is done as each
 * data-ready signal arrives. */
static void rank_bo_lo(int r, const or_schedule* s, int bo, size_t n, uint16_t* local_all,
                       uint16_t* recv_all, rank_ctl* ctl, uint32_t rep) {
    int N = s->total;
    size_t tile = 1024;
    size_t blk = bo ? n / (size_t)N : 0;
    size_t nt = n / tile;
    uint16_t* local = local_all + (size_t)r * n;
    uint16_t* recv = recv_all + (size_t)r * n;
    /* sync granularity, dataflow_kernel.cpp:134-144 / LOO :114-125 */
    size_t unit, units, per_sync;
    if (bo) { unit = blk; units = (size_t)N; per_sync = (size_t)N >= 32 ? (size_t)N / 32 : 1; }
    else {
        unit = tile; units = nt;
        size_t syncs = nt >= 64 ? 32 : (nt > 2 ? nt / 2 : nt);
        per_sync = nt / syncs;
    }
    size_t windows = (units + per_sync - 1) / per_sync;
    uint32_t sem1_base = rep * (uint32_t)(s->steps * windows);
    uint32_t hs = rep * (bo ? 2u : 1u);
    for (int k = 0; k < s->steps; ++k) {
        int p = s->partner[r][k];
        rank_ctl* pc = ctl + p;
        uint16_t* precv = recv_all + (size_t)p * n;
        uint64_t smask = bo ? s->send[r][k] : ~0ull;
        uint64_t rmask = bo ? s->recv[r][k] : ~0ull;
        sem_inc(&pc->sem0[k % 6]);
        sem_wait_min(&ctl[r].sem0[k % 6], hs + 1);
        for (size_t w = 0; w < windows; ++w) {
            for (size_t u = w * per_sync; u < (w + 1) * per_sync && u < units; ++u)
                if (!bo || ((smask >> u) & 1ull)) memcpy(precv + u * unit, local + u * unit, unit * 2);
            sem_inc(&pc->sem1);
        }
        for (size_t w = 0; w < windows; ++w) {
            sem_wait_min(&ctl[r].sem1, sem1_base + (uint32_t)(k * windows + w + 1));
            for (size_t u = w * per_sync; u < (w + 1) * per_sync && u < units; ++u)
                if (!bo || ((rmask >> u) & 1ull)) add_range(local + u * unit, recv + u * unit, unit);
        }
    }
    if (!bo) return;
    for (int k = s->steps - 1; k >= 0; --k) {
        int p = s->partner[r][k];
        rank_ctl* pc = ctl + p;
        uint16_t* plocal = local_all + (size_t)p * n;
        sem_inc(&pc->sem0[k % 6]);
        sem_wait_min(&ctl[r].sem0[k % 6], hs + 2);
        for (int b = 0; b < N; ++b)
            if ((s->recv[r][k] >> b) & 1ull) memcpy(plocal + b * blk, local + b * blk, blk * 2);
        sem_inc(&pc->sem_ag);
        sem_wait_min(&ctl[r].sem_ag, rep * (uint32_t)s->steps + (uint32_t)(s->steps - k));
    }
}

/* sync_nodes (allred_mem_2D/kernels/dataflow_kernel.cpp:201-230): a
 * dissemination barrier over the schedule's partners. */
static void sync_nodes(int r, const or_schedule* s, rank_ctl* ctl, uint32_t count) {
    for (int k = 0; k < s->steps; ++k) {
        sem_inc(&ctl[s->partner[r][k]].sem0[k % 6]);
        sem_wait_min(&ctl[r].sem0[k % 6], count);
    }
}

static void rank_mem(int r, const or_schedule* s, size_t n, uint16_t* local_all, uint16_t* common,
                     uint16_t* dst, rank_ctl* ctl, uint32_t* sync_count) {
    int N = s->total;
    size_t blk = n / (size_t)N;
    uint16_t* local = local_all + (size_t)r * n;
    memcpy(common + (size_t)r * n, local, n * 2);
    sync_nodes(r, s, ctl, ++*sync_count);
    for (size_t e = (size_t)r * blk; e < (size_t)(r + 1) * blk; ++e) {
        volatile float acc = or_bf16_to_float(common[(size_t)r * n + e]);
        for (int q = 0; q < N; ++q)
            if (q != r) acc = acc + or_bf16_to_float(common[(size_t)q * n + e]);
        dst[e] = or_bf16_rne(acc);
    }
    sync_nodes(r, s, ctl, ++*sync_count);
    memcpy(local, dst, n * 2);
}

long or_loopback_run(const or_loopback_args* a, double* seconds) { return or_loopback_run_stamps(a, seconds, NULL); }

long or_loopback_run_stamps(const or_loopback_args* a, double* seconds, double* stamps) {
    int side = or_highest_power_of_two(a->side);
    int N = a->total > 0 ? a->total : side * side;
    int mem = a->variant == 2;
    int bo = mem ? 1 : a->bo;
    or_schedule s;
    if (or_build_schedule(a->swing, side, N, &s) != 0) return -2;
    int NT = or_normalize_tiles(a->tiles_arg, N, bo);
    size_t n = (size_t)NT * 1024;
    if (bo && n % (size_t)N) return -3;
    size_t bytes = n * 2;
    /* inputs (allred_helper.cpp:277-285) */
    uint32_t* src0 = (uint32_t*)malloc(bytes);
    uint32_t* src1 = (uint32_t*)malloc(bytes);
    if (a->seed < 0) {
        or_constant_bf16_vector(bytes, 1.0f, src0);
        memcpy(src1, src0, bytes);
    } else {
        or_random_bf16_vector(bytes, 100, a->seed, a->round_mode, src0);
        or_random_bf16_vector(bytes, 100, a->seed + 1, a->round_mode, src1);
    }
    int reps = a->reps < 1 ? 1 : a->reps;
    size_t shm_bytes = 4096 + (size_t)N * sizeof(rank_ctl) + 2 * (size_t)N * bytes + bytes + 8 * (size_t)reps +
                       16 * (size_t)reps * (size_t)N;
    uint8_t* shm = (uint8_t*)mmap(NULL, shm_bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (shm == MAP_FAILED) { free(src0); free(src1); return -4; }
    memset(shm, 0, 4096 + (size_t)N * sizeof(rank_ctl));
    shm_barrier* bar = (shm_barrier*)shm;
    rank_ctl* ctl = (rank_ctl*)(shm + 4096);
    uint16_t* local_all = (uint16_t*)(shm + 4096 + (size_t)N * sizeof(rank_ctl));
    uint16_t* recv_all = local_all + (size_t)N * n;   /* recv buffers, or the common buffer for mem */
    uint16_t* dst = recv_all + (size_t)N * n;
    double* times = (double*)(dst + n);
    double* rank_stamps = times + reps;   /* [reps][N][2] absolute CLOCK_MONOTONIC seconds */
    pid_t* pids = (pid_t*)calloc((size_t)N, sizeof(pid_t));
    for (int r = 0; r < N; ++r) {
        pid_t pid = fork();
        if (pid == 0) {
            uint32_t sync_count = 0;
            /* even x loads src_1, odd x loads src_0 (allred_BO_2D.cpp:79-85) */
            const uint32_t* src = ((r % side) % 2 == 0) ? src1 : src0;
            for (int rep = 0; rep < reps; ++rep) {
                memcpy(local_all + (size_t)r * n, src, bytes);
                barrier_wait(bar, (uint32_t)N);
                ctl[r].t_start = now_s();
                if (mem) rank_mem(r, &s, n, local_all, recv_all, dst, ctl, &sync_count);
                else rank_bo_lo(r, &s, bo, n, local_all, recv_all, ctl, (uint32_t)rep);
                ctl[r].t_end = now_s();
                rank_stamps[((size_t)rep * N + r) * 2] = ctl[r].t_start;
                rank_stamps[((size_t)rep * N + r) * 2 + 1] = ctl[r].t_end;
                barrier_wait(bar, (uint32_t)N);
                if (r == 0) {
                    double t0 = 1e300, t1 = 0;
                    for (int q = 0; q < N; ++q) {
                        if (ctl[q].t_start < t0) t0 = ctl[q].t_start;
                        if (ctl[q].t_end > t1) t1 = ctl[q].t_end;
                    }
                    times[rep] = t1 - t0;
                }
                barrier_wait(bar, (uint32_t)N);
            }
            _exit(0);
        }
        pids[r] = pid;
    }
    int ok = 1;
    for (int r = 0; r < N; ++r) {
        int st = 0;
        if (waitpid(pids[r], &st, 0) < 0 || !WIFEXITED(st) || WEXITSTATUS(st) != 0) ok = 0;
    }
    (void)ok;
    long bad = 0;
    if (seconds)
        for (int rep = 0; rep < reps; ++rep) seconds[rep] = times[rep];
    if (stamps) {
        double t0 = 1e300;
        for (int r = 0; r < N; ++r)
            if (rank_stamps[(size_t)r * 2] < t0) t0 = rank_stamps[(size_t)r * 2];
        for (size_t i = 0; i < (size_t)reps * N * 2; ++i) stamps[i] = rank_stamps[i] - t0;
    }
    int pc = (a->print_core >= 0 && a->print_core < N) ? a->print_core : 0;
    bad = or_validate((const uint32_t*)(local_all + (size_t)pc * n), src0, src1, bytes / 4, (float)a->error,
                      (uint32_t)N, a->round_mode, NULL);
    munmap(shm, shm_bytes);
    free(pids);
    free(src0);
    free(src1);
    return ok ? bad : -5;
}
