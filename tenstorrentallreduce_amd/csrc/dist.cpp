// dist.cpp — multi-GPU allreduce: one process per GPU, RCCL point-to-point.
//
// The per-rank step program is the reference's per-core dataflow program
// (allred_BO_2D/kernels/dataflow_kernel.cpp) with the NoC replaced by xGMI:
//   reduce-scatter step k (:152-213): send the blocks of send_mask_k to the
//     partner, receive recv_mask_k's blocks into a staging buffer, add them
//     into the local bucket (compute_kernel.cpp:35-67);
//   all-gather step k, reverse order (:219-267): send the blocks of
//     recv_mask_k, receive the partner's owned blocks straight into the bucket;
//   LO (shouldSendBlock with bandwidth_optimal = 0, :19-29): full-vector
//     exchange + add every step.
// A step's blocks go out as one ncclSend/ncclRecv per contiguous run of set
// bits, inside one ncclGroupStart/End, on the caller's stream; the add is the
// HIP kernel of kernels.hip on the same stream.  The identical program also
// runs on host memory with a caller-supplied exchange (allred_dist_allreduce_host)
// so CPU tests (gloo) cover every step of it.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "internal.hpp"

using namespace tsa;

struct allred_comm {
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0, device = 0;
};

namespace {

struct Seg {
    size_t off, len;  // elements
};

struct Step {
    int peer = -1;
    std::vector<Seg> send;          // from the bucket
    std::vector<Seg> recv;          // into staging (add) or into the bucket (AG)
    bool recv_to_bucket = false;
    bool add = false;               // bucket[recv segs] += staging[recv segs]
};

void runs(uint64_t mask, int total, size_t blk, std::vector<Seg>* out) {
    int b = 0;
    while (b < total) {
        if (!((mask >> b) & 1ull)) { ++b; continue; }
        int e = b;
        while (e < total && ((mask >> e) & 1ull)) ++e;
        out->push_back(Seg{(size_t)b * blk, (size_t)(e - b) * blk});
        b = e;
    }
}

// the rank's program; chunks > 1 splits every step's segments into pieces so
// the add of one piece can overlap the transfer of the next
std::vector<Step> program(const allred_schedule& s, int rank, int variant, size_t n) {
    std::vector<Step> prog;
    const int N = s.total;
    const size_t blk = n / (size_t)N;
    if (variant == ALLRED_LO) {
        for (int k = 0; k < s.steps; ++k) {
            Step st;
            st.peer = s.partner[rank][k];
            st.send.push_back(Seg{0, n});
            st.recv.push_back(Seg{0, n});
            st.add = true;
            prog.push_back(st);
        }
        return prog;
    }
    for (int k = 0; k < s.steps; ++k) {
        Step st;
        st.peer = s.partner[rank][k];
        runs(s.send[rank][k], N, blk, &st.send);
        runs(s.recv[rank][k], N, blk, &st.recv);
        st.add = true;
        prog.push_back(st);
    }
    for (int k = s.steps - 1; k >= 0; --k) {
        Step st;
        st.peer = s.partner[rank][k];
        runs(s.recv[rank][k], N, blk, &st.send);
        runs(s.send[rank][k], N, blk, &st.recv);
        st.recv_to_bucket = true;
        prog.push_back(st);
    }
    return prog;
}

int check_desc(const allred_dist_desc* d, allred_schedule* s) {
    if (!d) return ALLRED_ERR_ARG;
    if (d->variant != ALLRED_BO && d->variant != ALLRED_LO) return ALLRED_ERR_UNSUPPORTED;
    const size_t n = (size_t)d->elems;
    if (n == 0 || n % 8) return ALLRED_ERR_ARG;
    if (d->variant == ALLRED_BO && n % (8 * (size_t)d->total_nodes)) return ALLRED_ERR_ARG;
    if (d->local_ranks > 1 && (d->local_ranks & (d->local_ranks - 1))) return ALLRED_ERR_ARG;
    return build_schedule(d->algo, d->side_length, d->total_nodes, s, nullptr);
}

size_t partial_bytes(const allred_dist_desc* d) { return d->local_ranks > 1 ? (size_t)d->elems * 2 : 0; }

// ---------------- host twin helpers ----------------
void host_add(uint16_t* dst, const uint16_t* src, size_t n) {
    for (size_t i = 0; i < n; ++i)
        dst[i] = bf16_from_float_rne(bf16_to_float(dst[i]) + bf16_to_float(src[i]));
}

// tree reduce over L local ranks in schedule tree order, bf16 rounding per level
void host_tree_reduce(const uint16_t* ranks, size_t stride, size_t n, const allred_schedule& s, uint16_t* out) {
    const int L = s.total;
    std::vector<uint16_t> v((size_t)L);
    for (size_t e = 0; e < n; ++e) {
        for (int i = 0; i < L; ++i) v[i] = ranks[(size_t)s.tree_order[0][i] * stride + e];
        for (int w = 1; w < L; w *= 2)
            for (int i = 0; i < L; i += 2 * w)
                v[i] = bf16_from_float_rne(bf16_to_float(v[i]) + bf16_to_float(v[i + w]));
        out[e] = v[0];
    }
}

// device copy of tree_order[0] of a (algo, side, total) schedule, cached for the process
std::mutex g_order_mu;
std::map<std::tuple<int, int, int, int>, uint8_t*> g_orders;

int device_order(int algo, int side, int total, const uint8_t** out) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(g_order_mu);
    auto key = std::make_tuple(dev, algo, side, total);
    auto it = g_orders.find(key);
    if (it == g_orders.end()) {
        allred_schedule s;
        int st = build_schedule(algo, side, total, &s, nullptr);
        if (st != ALLRED_OK) return st;
        uint8_t* p = nullptr;
        if (hipMalloc((void**)&p, ALLRED_MAX_NODES) != hipSuccess) return ALLRED_ERR_NOMEM;
        if (hipMemcpy(p, s.tree_order[0], ALLRED_MAX_NODES, hipMemcpyHostToDevice) != hipSuccess) return ALLRED_ERR_HIP;
        it = g_orders.emplace(key, p).first;
    }
    *out = it->second;
    return ALLRED_OK;
}

}  // namespace

extern "C" {

int allred_tree_reduce(const uint16_t* ranks, uint64_t stride, size_t n, int algo, int side, int total,
                       uint16_t* out, void* stream) {
    if (!ranks || !out || stride < n) return ALLRED_ERR_ARG;
    const uint8_t* order = nullptr;
    int st = device_order(algo, side, total, &order);
    if (st != ALLRED_OK) return st;
    return launch_tree_reduce(ranks, stride, n, total, order, out, stream);
}

int allred_broadcast(uint16_t* ranks, uint64_t stride, size_t n, int total, const uint16_t* src, void* stream) {
    if (!ranks || !src || stride < n || total < 1) return ALLRED_ERR_ARG;
    return launch_broadcast(ranks, stride, n, total, src, stream);
}

int allred_comm_get_unique_id(uint8_t* id) {
    if (!id) return ALLRED_ERR_ARG;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return ALLRED_ERR_RCCL;
    std::memcpy(id, &u, sizeof(u));
    return ALLRED_OK;
}

int allred_comm_init(const uint8_t* id, int nranks, int rank, int device, allred_comm** out) {
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return ALLRED_ERR_ARG;
    *out = nullptr;
    if (device >= 0 && hipSetDevice(device) != hipSuccess) return ALLRED_ERR_HIP;
    auto* c = new allred_comm();
    c->nranks = nranks;
    c->rank = rank;
    (void)hipGetDevice(&c->device);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    if (ncclCommInitRank(&c->comm, nranks, u, rank) != ncclSuccess) {
        delete c;
        return ALLRED_ERR_RCCL;
    }
    *out = c;
    return ALLRED_OK;
}

int allred_comm_destroy(allred_comm* c) {
    if (!c) return ALLRED_OK;
    if (c->comm) ncclCommDestroy(c->comm);
    delete c;
    return ALLRED_OK;
}

size_t allred_dist_workspace_bytes(const allred_dist_desc* d) {
    if (!d) return 0;
    return (size_t)d->elems * 2 + partial_bytes(d);
}

int allred_dist_allreduce(allred_comm* c, const allred_dist_desc* d, uint16_t* buf, void* workspace,
                          void* stream) {
    if (!c || !buf || !workspace) return ALLRED_ERR_ARG;
    allred_schedule s;
    int st = check_desc(d, &s);
    if (st != ALLRED_OK) return st;
    if (d->total_nodes != c->nranks) return ALLRED_ERR_ARG;
    hipStream_t hs = (hipStream_t)stream;
    const size_t n = (size_t)d->elems;
    uint16_t* staging = static_cast<uint16_t*>(workspace);
    uint16_t* bucket = buf;
    if (d->local_ranks > 1) {
        bucket = staging + n;  // the GPU's partial
        st = allred_tree_reduce(buf, n, n, d->local_algo, d->local_side, d->local_ranks, bucket, stream);
        if (st != ALLRED_OK) return st;
    }
    const std::vector<Step> prog = program(s, c->rank, d->variant, n);
    const size_t blk = n / (size_t)s.total;
    for (const Step& step : prog) {
        if (ncclGroupStart() != ncclSuccess) return ALLRED_ERR_RCCL;
        for (const Seg& g : step.send)
            if (ncclSend(bucket + g.off, g.len * 2, ncclUint8, step.peer, c->comm, hs) != ncclSuccess)
                return ALLRED_ERR_RCCL;
        for (const Seg& g : step.recv)
            if (ncclRecv((step.recv_to_bucket ? bucket : staging) + g.off, g.len * 2, ncclUint8, step.peer, c->comm,
                         hs) != ncclSuccess)
                return ALLRED_ERR_RCCL;
        if (ncclGroupEnd() != ncclSuccess) return ALLRED_ERR_RCCL;
        if (step.add) {
            if (d->variant == ALLRED_LO) {
                st = launch_bf16_add(bucket, staging, n, stream);
            } else {
                uint8_t blocks[ALLRED_MAX_NODES];
                int nb = 0;
                for (const Seg& g : step.recv)
                    for (size_t b = g.off / blk; b < (g.off + g.len) / blk; ++b) blocks[nb++] = (uint8_t)b;
                st = launch_bf16_add_blocks(bucket, staging, blocks, nb, blk, stream);
            }
            if (st != ALLRED_OK) return st;
        }
    }
    if (d->local_ranks > 1) st = launch_broadcast(buf, n, n, d->local_ranks, bucket, stream);
    return st;
}

int allred_dist_allreduce_host(const allred_dist_desc* d, int rank, uint16_t* buf, uint16_t* scratch,
                               allred_exchange_fn exchange, void* ctx) {
    if (!buf || !scratch || !exchange) return ALLRED_ERR_ARG;
    allred_schedule s;
    int st = check_desc(d, &s);
    if (st != ALLRED_OK) return st;
    if (rank < 0 || rank >= d->total_nodes) return ALLRED_ERR_ARG;
    const size_t n = (size_t)d->elems;
    uint16_t* bucket = buf;
    if (d->local_ranks > 1) {
        allred_schedule ls;
        st = build_schedule(d->local_algo, d->local_side, d->local_ranks, &ls, nullptr);
        if (st != ALLRED_OK) return st;
        bucket = scratch + n;
        host_tree_reduce(buf, n, n, ls, bucket);
    }
    const std::vector<Step> prog = program(s, rank, d->variant, n);
    std::vector<allred_seg> snd, rcv;
    for (const Step& step : prog) {
        snd.clear();
        rcv.clear();
        for (const Seg& g : step.send) snd.push_back(allred_seg{bucket + g.off, g.len * 2});
        for (const Seg& g : step.recv)
            rcv.push_back(allred_seg{(step.recv_to_bucket ? bucket : scratch) + g.off, g.len * 2});
        if (exchange(ctx, step.peer, (int)snd.size(), snd.data(), (int)rcv.size(), rcv.data()) != 0)
            return ALLRED_ERR_TRANSPORT;
        if (step.add)
            for (const Seg& g : step.recv) host_add(bucket + g.off, scratch + g.off, g.len);
    }
    if (d->local_ranks > 1)
        for (int r = 0; r < d->local_ranks; ++r) std::memcpy(buf + (size_t)r * n, bucket, n * 2);
    return ALLRED_OK;
}

}  // extern "C"
