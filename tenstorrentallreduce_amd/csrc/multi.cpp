// multi.cpp — allred_run across the GPUs of one node (args->gpus = G): the
// reference's argv (allred_BO_2D.cpp:7-29, allred_helper.cpp:205-220) with its
// ranks spread over G GPUs, one host thread per GPU.
//
// Two parts (include/allred.h, "allred_run across GPUs"):
//   the PLAN (allred_multi_plan_build): pure host computation — how the
//     (side, total) ranks split over the GPUs, the exchange every GPU runs,
//     which ranks are validated; no HIP call, so the CPU suite inspects it;
//   an EXCHANGE BACKEND executing it: RCCL (one communicator per GPU,
//     bounded waits), the peer windows of the G threads mapped into each
//     other (optionally every group on one GPU: the orchestration rehearsed on
//     hardware), or the host twin (host memory, allred_dist_allreduce_host
//     with an in-memory exchange; no HIP call at all).
// Everything between the two — input generation (allred_helper.cpp:277-285),
// the G threads and their barriers, per-GPU H2D / D2H slices, the timed region (Finish before the
// read-back where groups share a GPU)
// (EnqueueWriteBuffer | EnqueueProgram + Finish | EnqueueReadBuffer,
// allred_helper.hpp:84-96), the status agreement, validation
// (validate_result_vector, allred_helper.cpp:18-120) — is shared, so the host
// twin's CPU tests cover the same orchestration the GPU backends run.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "internal.hpp"

using namespace tsa;

namespace {

// (side, total) grids the reference's 2D functions accept for `c` ranks: SURVEY §8(e)
// (2,2), (2,4), (4,8) and the squares / rectangles above
int grid_side(int c) {
    switch (c) {
        case 1: return 1;
        case 2: case 4: return 2;
        case 8: case 16: return 4;
        default: return 8;
    }
}

// workgroup slots the groups sharing one GPU divide among their grids (default 256
// of the 512 the chip holds at two per CU); ALLRED_SHARE_SLOTS overrides (probes)
unsigned share_slots() {
    const char* s = std::getenv("ALLRED_SHARE_SLOTS");
    const int v = s && *s ? std::atoi(s) : 256;
    return (unsigned)std::min(512, std::max(8, v));
}

struct HostBarrier {   // the G threads meet before the warm-up and before the timed region
    std::mutex mu;
    std::condition_variable cv;
    int n, waiting = 0, gen = 0;
    explicit HostBarrier(int count) : n(count) {}
    void wait() {
        std::unique_lock<std::mutex> l(mu);
        const int g = gen;
        if (++waiting == n) {
            waiting = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(l, [&] { return gen != g; });
        }
    }
};

// ---------------------------------------------------------------------------
// Backends.  One Group per GPU; every method but open_all / close_all runs on
// the group's own thread.
// ---------------------------------------------------------------------------
struct Group {
    int g = 0, dev = 0;
    uint16_t *buf = nullptr, *tmp = nullptr;   // the GPU's L rank rows (timed / warm-up copy)
    void* ws = nullptr;
    hipStream_t hs = nullptr;
    hipEvent_t ev[4] = {};
    std::chrono::steady_clock::time_point t[4];
    std::vector<uint16_t> hbuf, htmp, hws;     // host backend memory
    float dev_ms = 0, e2e_ms = 0;
};

class Backend {
   public:
    Backend(const allred_multi_plan& p, const allred_multi_opts& o) : plan(p), opts(o) {}
    virtual ~Backend() = default;
    virtual int open_all(const std::vector<int>& devs) = 0;
    virtual int open(Group& gr) = 0;
    virtual int put(Group& gr, uint16_t* dst, const uint16_t* h_src, size_t bytes) = 0;
    virtual int get(Group& gr, uint16_t* h_dst, const uint16_t* src, size_t bytes) = 0;
    virtual int reduce(Group& gr, uint16_t* rows) = 0;
    virtual int mark(Group& gr, int i) = 0;
    virtual int drain(Group& gr) = 0;           // bounded wait for the group's work
    virtual int times(Group& gr) = 0;
    virtual void close(Group& gr) = 0;
    virtual void close_all() = 0;
    virtual void* host_alloc(size_t bytes) = 0;
    virtual void host_free(void* p) = 0;
    virtual void fail() { cancel.store(1); }    // another thread failed: waits give up
    std::atomic<int> cancel{0};

   protected:
    const allred_multi_plan& plan;
    const allred_multi_opts& opts;
    size_t rows_bytes() const { return (size_t)plan.local_ranks * plan.elems * 2; }
};

// ---- HIP device memory, streams, events: shared by the RCCL and peer backends ----
class DeviceBackend : public Backend {
   public:
    using Backend::Backend;
    int open(Group& gr) override {
        if (hipSetDevice(gr.dev) != hipSuccess) return ALLRED_ERR_HIP;
        if (hipStreamCreateWithFlags(&gr.hs, hipStreamNonBlocking) != hipSuccess) return ALLRED_ERR_HIP;
        if (hipMalloc((void**)&gr.buf, rows_bytes()) != hipSuccess) return ALLRED_ERR_NOMEM;
        if (hipMalloc((void**)&gr.tmp, rows_bytes()) != hipSuccess) return ALLRED_ERR_NOMEM;
        if (hipMalloc(&gr.ws, allred_dist_workspace_bytes(&plan.desc) + 16) != hipSuccess) return ALLRED_ERR_NOMEM;
        for (auto& e : gr.ev)
            if (hipEventCreate(&e) != hipSuccess) return ALLRED_ERR_HIP;
        return ALLRED_OK;
    }
    int put(Group& gr, uint16_t* dst, const uint16_t* h_src, size_t bytes) override {
        return hipMemcpyAsync(dst, h_src, bytes, hipMemcpyHostToDevice, gr.hs) == hipSuccess ? ALLRED_OK : ALLRED_ERR_HIP;
    }
    int get(Group& gr, uint16_t* h_dst, const uint16_t* src, size_t bytes) override {
        return hipMemcpyAsync(h_dst, src, bytes, hipMemcpyDeviceToHost, gr.hs) == hipSuccess ? ALLRED_OK : ALLRED_ERR_HIP;
    }
    int mark(Group& gr, int i) override { return hipEventRecord(gr.ev[i], gr.hs) == hipSuccess ? ALLRED_OK : ALLRED_ERR_HIP; }
    int times(Group& gr) override {
        if (hipEventElapsedTime(&gr.dev_ms, gr.ev[1], gr.ev[2]) != hipSuccess) return ALLRED_ERR_HIP;
        if (hipEventElapsedTime(&gr.e2e_ms, gr.ev[0], gr.ev[3]) != hipSuccess) return ALLRED_ERR_HIP;
        return ALLRED_OK;
    }
    void close(Group& gr) override {
        (void)hipSetDevice(gr.dev);
        for (auto& e : gr.ev)
            if (e) (void)hipEventDestroy(e);
        if (gr.ws) (void)hipFree(gr.ws);
        if (gr.tmp) (void)hipFree(gr.tmp);
        if (gr.buf) (void)hipFree(gr.buf);
        if (gr.hs) (void)hipStreamDestroy(gr.hs);
    }
    void* host_alloc(size_t bytes) override {
        void* p = nullptr;
        return hipHostMalloc(&p, bytes, hipHostMallocPortable) == hipSuccess ? p : nullptr;
    }
    void host_free(void* p) override { (void)hipHostFree(p); }

   protected:
    // G == 1 mem_2D: every rank on this GPU, the fused mem_2D pass (no exchange)
    int reduce_local(Group& gr, uint16_t* rows) {
        return launch_mem_fused(rows, plan.elems, plan.elems, plan.local_ranks, plan.desc.mem_accum == ALLRED_ACC_BF16,
                                gr.hs);
    }
};

class RcclBackend : public DeviceBackend {
   public:
    using DeviceBackend::DeviceBackend;
    int open_all(const std::vector<int>& devs) override {
        // RCCL refuses two ranks on one GPU: sharing a device is the peer / host backends' rehearsal
        if (opts.share_device && devs.size() > 1) return ALLRED_ERR_UNSUPPORTED;
        comms.assign(devs.size(), nullptr);
        int st = allred_comm_init_all((int)devs.size(), devs.data(), comms.data());
        for (allred_comm* c : comms) {
            comm_set_cancel(c, &cancel);
            if (c && opts.timeout_ms > 0) allred_comm_set_timeout(c, opts.timeout_ms);
        }
        return st;
    }
    int reduce(Group& gr, uint16_t* rows) override {
        if (plan.mode == ALLRED_MULTI_LOCAL) return reduce_local(gr, rows);
        return allred_dist_allreduce(comms[(size_t)gr.g], &plan.desc, rows, gr.ws, gr.hs);
    }
    // bounded (ALLRED_RCCL_TIMEOUT_MS): a GPU whose partner never arrives, or
    // whose peer thread failed (cancel), aborts its communicator and returns
    int drain(Group& gr) override { return allred_comm_wait(comms[(size_t)gr.g], gr.hs); }
    void close_all() override {
        for (allred_comm* c : comms) allred_comm_destroy(c);
        comms.clear();
    }

   private:
    std::vector<allred_comm*> comms;
};

class PeerBackend : public DeviceBackend {
   public:
    using DeviceBackend::DeviceBackend;
    int open_all(const std::vector<int>& devs) override {
        const int G = (int)devs.size();
        peers.assign((size_t)G, nullptr);
        // LO programs need elems <= max_elems / 2 (allred_peer_dist_allreduce)
        uint64_t max_elems = plan.elems * (plan.variant == ALLRED_LO ? 2 : 1);
        for (int g = 0; g < G; ++g) {
            int st = allred_peer_create(G, g, devs[(size_t)g], max_elems, &peers[(size_t)g]);
            if (st != ALLRED_OK) return st;
            // groups sharing one GPU wait for each other inside their kernels: every
            // group's grid must be resident at once (allred_peer_set_max_groups).  The
            // groups share half the chip's 512 two-per-CU slots (ALLRED_SHARE_SLOTS):
            // the other groups' copy kernels and next launches find room without
            // taking the last slot a waiting grid needs
            if (opts.share_device && G > 1) allred_peer_set_max_groups(peers[(size_t)g], share_slots() / (unsigned)G);
        }
        return allred_peer_connect_all(G, peers.data());
    }
    int reduce(Group& gr, uint16_t* rows) override {
        if (plan.mode == ALLRED_MULTI_LOCAL) return reduce_local(gr, rows);
        return allred_peer_dist_allreduce(peers[(size_t)gr.g], &plan.desc, rows, gr.ws, gr.hs);
    }
    // the peer kernels' spins are bounded: a dead partner sets the timeout bit instead of hanging
    int drain(Group& gr) override { return allred_peer_check(peers[(size_t)gr.g], gr.hs); }
    void close_all() override {
        for (allred_peer* p : peers) allred_peer_destroy(p);
        peers.clear();
    }

   private:
    std::vector<allred_peer*> peers;
};

// ---- the host twin: host memory, in-memory exchange, no HIP call ----------
// A pairwise rendezvous per exchange (the allred_exchange_fn contract: both
// sides send every send segment and receive every recv segment in list
// order): post my send list, wait for the partner's, copy it into my receive
// segments, mark it taken, wait until mine was taken.  Every wait has the
// deadline; a failed thread (cancel) wakes and fails every waiter.
struct HostExchange {
    int G = 0, timeout_ms = 4000;
    std::mutex mu;
    std::condition_variable cv;
    struct Box {
        const allred_seg* segs = nullptr;
        int nseg = 0;
        uint64_t posted = 0, taken = 0;
    };
    std::vector<Box> box;        // [src * G + dst]
    std::vector<uint64_t> seq;   // exchanges src started with dst
    std::atomic<int>* cancel = nullptr;
};
struct HostCtx {
    HostExchange* x;
    int me;
};

int host_exchange(void* ctx, int peer, int nsend, const allred_seg* send, int nrecv, const allred_seg* recv) {
    auto* hc = static_cast<HostCtx*>(ctx);
    HostExchange& x = *hc->x;
    const int me = hc->me, G = x.G;
    if (peer < 0 || peer >= G || peer == me) return 1;
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(x.timeout_ms);
    auto stopped = [&] { return x.cancel->load() != 0; };
    auto give_up = [&] {
        x.cancel->store(1);
        x.cv.notify_all();
        return 1;
    };
    std::unique_lock<std::mutex> l(x.mu);
    HostExchange::Box& out = x.box[(size_t)me * G + peer];
    HostExchange::Box& in = x.box[(size_t)peer * G + me];
    const uint64_t k = ++x.seq[(size_t)me * G + peer];
    out.segs = send;
    out.nseg = nsend;
    out.posted = k;
    x.cv.notify_all();
    if (!x.cv.wait_until(l, deadline, [&] { return in.posted >= k || stopped(); }) || stopped()) return give_up();
    const allred_seg* src = in.segs;
    const int ns = in.nseg;
    l.unlock();
    uint64_t have = 0, want = 0;
    for (int i = 0; i < ns; ++i) have += src[i].bytes;
    for (int i = 0; i < nrecv; ++i) want += recv[i].bytes;
    bool ok = have == want;
    // the partner's send list concatenated into my receive list (segment bounds may differ)
    int i = 0, j = 0;
    uint64_t si = 0, ro = 0;
    while (ok && i < ns && j < nrecv) {
        const uint64_t m = std::min(src[i].bytes - si, recv[j].bytes - ro);
        std::memcpy(static_cast<uint8_t*>(recv[j].ptr) + ro, static_cast<const uint8_t*>(src[i].ptr) + si, m);
        si += m;
        ro += m;
        if (si == src[i].bytes) { ++i; si = 0; }
        if (ro == recv[j].bytes) { ++j; ro = 0; }
    }
    l.lock();
    if (!ok) return give_up();
    in.taken = k;
    x.cv.notify_all();
    if (!x.cv.wait_until(l, deadline, [&] { return out.taken >= k || stopped(); }) || stopped()) return give_up();
    return 0;
}

// mem_2D with every rank in one memory (G == 1): block b = owner b's copy, then
// every other rank ascending, fp32 rounded once or bf16 per add — k_mem's order
void host_mem_local(uint16_t* rows, size_t n, int total, bool acc16) {
    const size_t blk = n / (size_t)total;
    std::vector<uint16_t> res(n);
    for (size_t e = 0; e < n; ++e) {
        const int own = (int)(e / blk);
        float a = bf16_to_float(rows[(size_t)own * n + e]);
        for (int r = 0; r < total; ++r) {
            if (r == own) continue;
            a += bf16_to_float(rows[(size_t)r * n + e]);
            if (acc16) a = bf16_to_float(bf16_from_float_rne(a));
        }
        res[e] = bf16_from_float_rne(a);
    }
    for (int r = 0; r < total; ++r) std::memcpy(rows + (size_t)r * n, res.data(), n * 2);
}

class HostBackend : public Backend {
   public:
    using Backend::Backend;
    int open_all(const std::vector<int>& devs) override {
        x.G = (int)devs.size();
        x.timeout_ms = opts.timeout_ms > 0 ? opts.timeout_ms : 60000;   // CPU twins of big buckets are slow
        x.box.assign((size_t)x.G * x.G, HostExchange::Box{});
        x.seq.assign((size_t)x.G * x.G, 0);
        x.cancel = &cancel;
        return ALLRED_OK;
    }
    int open(Group& gr) override {
        const size_t rows = (size_t)plan.local_ranks * plan.elems;
        gr.hbuf.assign(rows, 0);
        gr.htmp.assign(rows, 0);
        gr.hws.assign(2 * (size_t)plan.elems, 0);   // allred_dist_allreduce_host scratch: staging + partial
        gr.buf = gr.hbuf.data();
        gr.tmp = gr.htmp.data();
        gr.ws = gr.hws.data();
        return ALLRED_OK;
    }
    int put(Group&, uint16_t* dst, const uint16_t* h_src, size_t bytes) override {
        std::memcpy(dst, h_src, bytes);
        return ALLRED_OK;
    }
    int get(Group&, uint16_t* h_dst, const uint16_t* src, size_t bytes) override {
        std::memcpy(h_dst, src, bytes);
        return ALLRED_OK;
    }
    int reduce(Group& gr, uint16_t* rows) override {
        if (plan.mode == ALLRED_MULTI_LOCAL) {
            host_mem_local(rows, plan.elems, plan.local_ranks, plan.desc.mem_accum == ALLRED_ACC_BF16);
            return ALLRED_OK;
        }
        HostCtx ctx{&x, gr.g};
        return allred_dist_allreduce_host(&plan.desc, gr.g, rows, static_cast<uint16_t*>(gr.ws), host_exchange, &ctx);
    }
    int mark(Group& gr, int i) override {
        gr.t[i] = std::chrono::steady_clock::now();
        return ALLRED_OK;
    }
    int drain(Group&) override { return cancel.load() ? ALLRED_ERR_TRANSPORT : ALLRED_OK; }
    int times(Group& gr) override {
        gr.dev_ms = std::chrono::duration<float, std::milli>(gr.t[2] - gr.t[1]).count();
        gr.e2e_ms = std::chrono::duration<float, std::milli>(gr.t[3] - gr.t[0]).count();
        return ALLRED_OK;
    }
    void close(Group&) override {}
    void close_all() override {}
    void* host_alloc(size_t bytes) override { return std::malloc(bytes); }
    void host_free(void* p) override { std::free(p); }
    void fail() override {
        cancel.store(1);
        std::lock_guard<std::mutex> l(x.mu);
        x.cv.notify_all();
    }

   private:
    HostExchange x;
};

int env_transport(int* out) {
    const char* t = std::getenv("ALLRED_TRANSPORT");
    if (!t || !*t || std::strcmp(t, "rccl") == 0) *out = ALLRED_TRANSPORT_RCCL;
    else if (std::strcmp(t, "peer") == 0) *out = ALLRED_TRANSPORT_PEER;
    else if (std::strcmp(t, "host") == 0) *out = ALLRED_TRANSPORT_HOST;
    else return ALLRED_ERR_ARG;
    return ALLRED_OK;
}

}  // namespace

extern "C" {

int allred_multi_plan_build(const allred_args* a, int check_all, allred_multi_plan* P) {
    if (!a || !P) return ALLRED_ERR_ARG;
    std::memset(P, 0, sizeof(*P));
    const int G = a->gpus, N = a->total_nodes;
    if (G < 1 || G > ALLRED_MAX_NODES || (G & (G - 1)) || N < 1 || N > ALLRED_MAX_NODES || N % G) return ALLRED_ERR_ARG;
    if (a->print_core < 0 || a->print_core >= N || a->num_tiles < 1) return ALLRED_ERR_ARG;
    const int L = N / G;
    const size_t n = (size_t)a->num_tiles * 1024;
    const int variant = a->variant == ALLRED_MEM ? ALLRED_MEM
                        : (a->variant == ALLRED_BO && a->bandwidth_optimal) ? ALLRED_BO : ALLRED_LO;
    const int algo = a->swing ? ALLRED_SWING : ALLRED_RECDUB;
    // mem_2D sums every RANK's copy in rank order: one rank per GPU, or every rank on one
    if (variant == ALLRED_MEM && L > 1 && G > 1) return ALLRED_ERR_UNSUPPORTED;
    P->gpus = G;
    P->local_ranks = L;
    P->total_nodes = N;
    P->variant = variant;
    P->print_core = a->print_core;
    P->elems = n;
    allred_dist_desc& d = P->desc;
    d.algo = algo;
    d.variant = variant;
    d.elems = n;
    d.channels = 0;
    d.mem_accum = a->mem_accum;
    d.local_algo = algo;
    if (L == 1) {   // one rank per GPU: the reference's own grid across the GPUs
        d.side_length = a->side_length;
        d.total_nodes = N;
        d.local_ranks = 1;
        d.local_side = 1;
    } else {        // L ranks per GPU: their sub-grid (rows of the reference's grid if they form one)
        d.side_length = grid_side(G);
        d.total_nodes = G;
        d.local_ranks = L;
        allred_schedule ls;
        d.local_side = (L % a->side_length == 0 && build_schedule(algo, a->side_length, L, &ls, nullptr) == ALLRED_OK)
                           ? a->side_length : grid_side(L);
    }
    if (variant == ALLRED_MEM && G == 1) {   // every rank on one GPU: the fused mem_2D pass, no exchange
        if (n % (8 * (size_t)N)) return ALLRED_ERR_ARG;
        P->mode = ALLRED_MULTI_LOCAL;
        d.local_ranks = L;
    } else {
        allred_schedule s;
        int st = dist_check_desc(&d, &s);
        if (st != ALLRED_OK) return st;
        if (L > 1 && (st = build_schedule(algo, d.local_side, L, &s, nullptr)) != ALLRED_OK) return st;
        P->mode = L == 1 ? ALLRED_MULTI_FLAT : ALLRED_MULTI_HIER;
    }
    P->validated_mask = 1ull << a->print_core;
    for (int r = 0; r < N; ++r)
        if (check_all || r % L == 0) P->validated_mask |= 1ull << r;
    return ALLRED_OK;
}

int allred_run_multi(const allred_args* a, const allred_multi_opts* o, int verbose, allred_report* R,
                     const uint16_t* in_all, uint16_t* out_all) {
    if (!a || !o || !R) return ALLRED_ERR_ARG;
    if (o->transport < ALLRED_TRANSPORT_RCCL || o->transport > ALLRED_TRANSPORT_HOST || o->timeout_ms < 0)
        return ALLRED_ERR_ARG;
    std::memset(R, 0, sizeof(*R));
    R->mismatches = -1;
    allred_multi_plan plan;
    // everything checkable without a GPU first (no HIP call before the plan holds)
    int st = allred_multi_plan_build(a, std::getenv("ALLRED_CHECK_ALL") != nullptr, &plan);
    if (st != ALLRED_OK) return st;
    const int G = plan.gpus, L = plan.local_ranks, N = plan.total_nodes;
    const size_t n = (size_t)plan.elems, bytes = n * 2;
    R->bytes_per_rank = bytes;
    R->total_nodes = N;
    if (o->share_device && o->transport == ALLRED_TRANSPORT_RCCL && G > 1) return ALLRED_ERR_UNSUPPORTED;
    // the peer windows sum mem_2D in fp32 only (allred_peer_dist_allreduce): refused here,
    // before any GPU memory is allocated, not in every group's warm-up
    if (o->transport == ALLRED_TRANSPORT_PEER && plan.variant == ALLRED_MEM && plan.mode != ALLRED_MULTI_LOCAL &&
        plan.desc.mem_accum == ALLRED_ACC_BF16)
        return ALLRED_ERR_UNSUPPORTED;
    const int dev0 = a->device > 0 ? a->device : 0;
    std::vector<int> devs((size_t)G);
    for (int g = 0; g < G; ++g) devs[(size_t)g] = o->share_device ? dev0 : dev0 + g;
    if (o->transport != ALLRED_TRANSPORT_HOST) {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess) return ALLRED_ERR_HIP;
        if (devs.back() >= ndev) return ALLRED_ERR_ARG;
    }
    std::unique_ptr<Backend> be;
    if (o->transport == ALLRED_TRANSPORT_RCCL) be.reset(new RcclBackend(plan, *o));
    else if (o->transport == ALLRED_TRANSPORT_PEER) be.reset(new PeerBackend(plan, *o));
    else be.reset(new HostBackend(plan, *o));

    std::vector<uint32_t> src0(bytes / 4), src1(bytes / 4);
    if (a->seed < 0) {
        allred_constant_bf16_vector(bytes, 1.0f, src0.data());
        src1 = src0;
    } else {
        allred_random_bf16_vector(bytes, 100, a->seed, a->round_mode, src0.data());
        allred_random_bf16_vector(bytes, 100, a->seed + 1, a->round_mode, src1.data());
    }
    const size_t all_bytes = (size_t)N * bytes;
    auto* h_in = static_cast<uint16_t*>(be->host_alloc(all_bytes));
    auto* h_out = static_cast<uint16_t*>(be->host_alloc(all_bytes));
    if (!h_in || !h_out) {
        if (h_in) be->host_free(h_in);
        if (h_out) be->host_free(h_out);
        return ALLRED_ERR_NOMEM;
    }
    if (in_all) {   // the caller's own rank vectors
        std::memcpy(h_in, in_all, all_bytes);
    } else {        // even x loads src_1, odd x loads src_0 (allred_BO_2D.cpp:79-85)
        for (int r = 0; r < N; ++r)
            std::memcpy(h_in + (size_t)r * n, ((r % a->side_length) % 2 == 0) ? src1.data() : src0.data(), bytes);
    }
    std::memset(h_out, 0, all_bytes);

    std::vector<Group> grs((size_t)G);
    st = be->open_all(devs);
    if (st == ALLRED_OK) {
        HostBarrier bar(G);
        // one verdict slot per thread and round: a thread already in round 2 must not
        // change what a slower thread still reads for round 1
        std::vector<int> ok(2 * (size_t)G, 0);
        std::vector<int> status((size_t)G, ALLRED_OK);
        std::vector<std::thread> th;
        const size_t mine = (size_t)L * bytes;
        // every thread reaches bar.wait() of round 1, and of round 2 iff round 1 agreed
        // everywhere (every thread reads the same round-1 slots), so none waits forever
        auto agree = [&](int g, int s, int round) {
            int* v = ok.data() + (size_t)round * G;
            v[g] = s == ALLRED_OK;
            if (s != ALLRED_OK) be->fail();
            bar.wait();
            bool all = true;
            for (int q = 0; q < G; ++q) all = all && v[q];
            return all;
        };
        // ALLRED_MULTI_TRACE=1: every thread's host-side phases on stderr (ms since the start)
        const bool trace = std::getenv("ALLRED_MULTI_TRACE") && std::atoi(std::getenv("ALLRED_MULTI_TRACE")) != 0;
        const auto t_start = std::chrono::steady_clock::now();
        std::mutex trace_mu;
        auto mark = [&](int g, const char* what, int s) {
            if (!trace) return;
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
            std::lock_guard<std::mutex> l(trace_mu);
            std::fprintf(stderr, "multi-trace g%d %-12s %9.3f ms status %d\n", g, what, ms, s);
        };
        for (int g = 0; g < G; ++g) {
            grs[(size_t)g].g = g;
            grs[(size_t)g].dev = devs[(size_t)g];
            th.emplace_back([&, g] {
                Group& gr = grs[(size_t)g];
                int& s = status[(size_t)g];
                const uint16_t* in = h_in + (size_t)g * L * n;
                // every call runs only while this thread is healthy; the first failure
                // raises the shared cancel at once (the peers' waits give up instead of
                // running into their deadlines) and this thread skips its own exchanges
                auto step = [&](auto&& call) {
                    if (s != ALLRED_OK) return;
                    s = call();
                    if (s != ALLRED_OK) be->fail();
                };
                // every way out of a failed thread: one more cancel-aware drain, so work
                // it already queued (RCCL kernels waiting for aborted peers) is aborted
                // before close() frees the memory it points at (a hipFree syncs the device)
                bool opened = false;
                auto leave = [&] {
                    if (s != ALLRED_OK && opened) (void)be->drain(gr);
                };
                step([&] { return be->open(gr); });
                opened = s == ALLRED_OK;
                mark(g, "open", s);
                // warm-up on a scratch copy (connection setup, code-object loads stay untimed)
                step([&] { return be->put(gr, gr.tmp, in, mine); });
                mark(g, "put", s);
                // every thread agrees before any exchange: one failed setup ends all
                if (!agree(g, s, 0)) {
                    if (s == ALLRED_OK) s = ALLRED_ERR_TRANSPORT;   // another GPU failed to set up
                    return leave();
                }
                mark(g, "agree1", s);
                if (a->run_kernel) step([&] { return be->reduce(gr, gr.tmp); });
                // fault injection (tests): GPU multi_fault - 33 fails its warm-up; every
                // thread must skip the timed region and return
                if (tune(Tune::multi_fault) == 33 + g) step([] { return (int)ALLRED_ERR_TRANSPORT; });
                mark(g, "warm-launch", s);
                step([&] { return be->drain(gr); });
                mark(g, "warm-drain", s);
                // ... and again after the warm-up (a GPU whose warm-up failed must not
                // leave the others alone in the timed exchanges)
                if (!agree(g, s, 1)) {
                    if (s == ALLRED_OK) s = ALLRED_ERR_TRANSPORT;
                    return leave();
                }
                // timed: H2D | allreduce | D2H (the reference's EnqueueWriteBuffer,
                // EnqueueProgram + Finish, EnqueueReadBuffer; allred_helper.hpp:84-96)
                mark(g, "agree2", s);
                step([&] { return be->mark(gr, 0); });
                step([&] { return be->put(gr, gr.buf, in, mine); });
                step([&] { return be->mark(gr, 1); });
                // fault injection (tests): GPU multi_fault - 1 fails its timed allreduce before any
                // exchange, while its peers are inside theirs: it never joins them, they are
                // cancelled, and every thread still returns
                if (a->run_kernel && tune(Tune::multi_fault) == g + 1) step([] { return (int)ALLRED_ERR_TRANSPORT; });
                mark(g, "timed-put", s);
                if (a->run_kernel) step([&] { return be->reduce(gr, gr.buf); });
                mark(g, "timed-launch", s);
                step([&] { return be->mark(gr, 2); });
                // groups sharing one GPU: Finish before the read-back, as the reference's helper
                // does — a D2H copy queued behind a waiting allreduce can hold the copy engine
                // that another group's H2D (which its allreduce waits for) is queued behind
                // (they share its SDMA engines: profiles/r04_multi_share_trace.txt).  A GPU of
                // its own queues the D2H right behind its allreduce (stream order), no host wait
                if (o->share_device) step([&] { return be->drain(gr); });
                mark(g, "timed-finish", s);
                step([&] { return be->get(gr, h_out + (size_t)g * L * n, gr.buf, mine); });
                step([&] { return be->mark(gr, 3); });
                step([&] { return be->drain(gr); });
                mark(g, "timed-drain", s);
                step([&] { return be->times(gr); });
                leave();
            });
        }
        for (auto& x : th) x.join();
        for (int g = 0; g < G && st == ALLRED_OK; ++g) st = status[(size_t)g];
        // after a failure the communicators / peer windows go first: an aborted
        // communicator's kernels have left their waits before any group's memory is freed
        if (st != ALLRED_OK) be->close_all();
        // the groups' memory, events and streams released once every thread is done: a
        // hipFree synchronises the device, which groups sharing one GPU must not do while
        // another group still has work queued behind it
        for (Group& gr : grs) be->close(gr);
        // a thread that failed first reports its own status, not the others' TRANSPORT
        for (int g = 0; g < G; ++g)
            if (status[(size_t)g] != ALLRED_OK && status[(size_t)g] != ALLRED_ERR_TRANSPORT) {
                st = status[(size_t)g];
                break;
            }
    }
    be->close_all();
    if (st == ALLRED_OK) {
        float dmax = 0, emax = 0;
        for (const Group& gr : grs) {
            dmax = std::max(dmax, gr.dev_ms);
            emax = std::max(emax, gr.e2e_ms);
        }
        R->device_seconds = dmax * 1e-3;
        R->e2e_seconds = emax * 1e-3;
        R->launches = -1;   // RCCL groups and add kernels per GPU: allred_dist_program_stats
        if (const char* log = std::getenv("ALLRED_PROFILE_LOG")) {   // one zone per rank: its GPU's interval
            std::vector<uint64_t> zs((size_t)N, 0), ze((size_t)N, 0);
            for (int r = 0; r < N; ++r) ze[(size_t)r] = (uint64_t)(grs[(size_t)(r / L)].dev_ms * 1e5);
            st = write_profile_log(log, N, a->side_length, zs.data(), ze.data());
        }
    }
    if (st == ALLRED_OK && in_all) {   // arbitrary data: no closed-form check, the caller compares
        if (out_all) std::memcpy(out_all, h_out, all_bytes);
    } else if (st == ALLRED_OK) {
        // print_core exactly as the reference (verbose report), then every other
        // validated rank (every GPU's first; ALLRED_CHECK_ALL: all) silently into the count
        float maxe = 0;
        R->mismatches = allred_validate_result_vector(
            reinterpret_cast<const uint32_t*>(h_out + (size_t)a->print_core * n), src0.data(), src1.data(), bytes / 4,
            (float)a->error, (uint32_t)N, verbose, &maxe);
        R->max_error = maxe;
        for (int r = 0; r < N; ++r) {
            if (r == a->print_core || !((plan.validated_mask >> r) & 1ull)) continue;
            float m = 0;
            R->mismatches += allred_validate_result_vector(reinterpret_cast<const uint32_t*>(h_out + (size_t)r * n),
                                                           src0.data(), src1.data(), bytes / 4, (float)a->error,
                                                           (uint32_t)N, 0, &m);
            R->max_error = std::max(R->max_error, m);
        }
        if (out_all) std::memcpy(out_all, h_out, all_bytes);
    }
    be->host_free(h_in);
    be->host_free(h_out);
    return st;
}

}  // extern "C"

// allred_run with args->gpus > 0: the backend from the environment
int tsa::run_multi_gpu(const allred_args* a, int verbose, allred_report* R) {
    allred_multi_opts o{};
    if (env_transport(&o.transport) != ALLRED_OK) return ALLRED_ERR_ARG;
    const char* share = std::getenv("ALLRED_SHARE_GPU");
    o.share_device = share && *share && std::strcmp(share, "0") != 0;
    if (const char* t = std::getenv("ALLRED_RCCL_TIMEOUT_MS")) o.timeout_ms = std::max(0, std::atoi(t));
    return allred_run_multi(a, &o, verbose, R, nullptr, nullptr);
}
