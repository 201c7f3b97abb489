// peer.cpp — the shared-memory variant (allred_mem_2D) across GPUs: a
// peer-mapped one-shot reduce-scatter / all-gather over xGMI.
//
// The reference's SM variant (allred_mem_2D.cpp:4-165, kernels/*) has every
// core dump its vector into one shared DRAM buffer, reduce its own block from
// all copies, write it to the destination buffer and read everything back,
// with node-to-node semaphore barriers between the phases (sync_nodes,
// kernels/dataflow_kernel.cpp:201-230).  Across MI355X GPUs the "shared
// buffer" is each GPU's window, IPC-mapped into every peer; the phases are
//   copy bucket -> own window | barrier | reduce own block from all windows |
//   barrier | gather every other block from its owner's window,
// so every transfer reads from all N-1 peers at once (all xGMI links busy).
// Barrier flags live in uncached device memory and are written / polled with
// system-scope atomics (bounded spins set a status bit instead of hanging).
// Buckets up to allred_peer_set_oneshot_max() bytes (default 4 MiB) run the
// same three phases as ONE kernel (k_peer_oneshot): workgroup g syncs only
// with workgroup g of the peers, through per-workgroup flag slots.  With 64
// local ranks per GPU the local tree and the broadcast join that kernel too
// (k_hier_oneshot, per-tile flags behind the window parities; k_hier_ll, the
// same step with LL push hand-offs, LL boxes behind the flags).
// Windows are double-buffered by call parity: call k+2 can only overwrite a
// window after every peer passed call k+1's first barrier, i.e. finished
// reading call k's windows.
#include <hip/hip_runtime.h>

#include <cstring>

#include "internal.hpp"

using namespace tsa;

struct allred_peer {
    int nranks = 0, rank = 0, device = 0;
    uint64_t max_elems = 0;
    uint16_t* win = nullptr;        // own window: 2 parities x max_elems
    uint32_t* flags = nullptr;      // own flag area (uncached), layout in internal.hpp
    uint32_t* status = nullptr;     // device status word
    bool flags_uncached = false, win_uncached = false;
    size_t hfl_off = 0;             // byte offset of the per-tile flags behind the two window parities
    size_t hfl_bytes = 0;
    uint32_t* peer_hfl[ALLRED_MAX_NODES] = {};
    uint16_t* peer_win[ALLRED_MAX_NODES] = {};
    uint32_t* peer_flags[ALLRED_MAX_NODES] = {};
    bool opened[ALLRED_MAX_NODES] = {};
    uint32_t calls = 0;
    uint32_t seq = 0;               // progress-flag base of the scheduled form
    bool last_all_peer = false;     // previous call read every rank's window
    uint64_t oneshot_max = 4ull << 20;  // buckets up to this many bytes use the one-kernel form
    bool connected = false;
    // LL (push) hierarchical form: behind the per-tile flags, 2 parities x
    // [inbox ll_box_words][result box ll_box_words] 8-byte words, zeroed at create
    size_t ll_off = 0;
    uint64_t ll_box_words = 0;
    uint64_t* peer_ll[ALLRED_MAX_NODES] = {};
    bool hier_ll = false;
};

extern "C" {

int allred_peer_create(int nranks, int rank, int device, uint64_t max_elems, allred_peer** out) {
    if (!out || nranks < 1 || nranks > ALLRED_MAX_NODES || rank < 0 || rank >= nranks || max_elems == 0)
        return ALLRED_ERR_ARG;
    *out = nullptr;
    if (device >= 0 && hipSetDevice(device) != hipSuccess) return ALLRED_ERR_HIP;
    auto* p = new allred_peer();
    p->nranks = nranks;
    p->rank = rank;
    (void)hipGetDevice(&p->device);
    p->max_elems = (max_elems + 127) / 128 * 128;  // LO halves stay 64-element aligned
    // windows are uncached too: peers read them over xGMI straight from HBM, so
    // no write may linger in one of this GPU's eight per-XCD L2s.  Behind the
    // two parities: the hierarchical form's per-tile flags, [tiles][nranks + 1]
    // for up to max_elems / 2 elements per call (256-element tiles).
    p->hfl_off = 2 * p->max_elems * 2;
    p->hfl_bytes = 4 * (size_t)(nranks + 1) * (p->max_elems / 2 / 256 + 1);
    // LL boxes for buckets of up to min(max_elems, 4 Mi) elements: 128 words per 256-element tile
    const uint64_t ll_elems = p->max_elems < (4ull << 20) ? p->max_elems : (4ull << 20);
    p->ll_off = (p->hfl_off + p->hfl_bytes + 255) / 256 * 256;
    p->ll_box_words = (ll_elems / 256) * 128;
    const size_t ll_bytes = 2 * 2 * p->ll_box_words * 8;
    const size_t win_bytes = p->ll_off + ll_bytes;
    if (hipExtMallocWithFlags((void**)&p->win, win_bytes, hipDeviceMallocUncached) == hipSuccess) {
        p->win_uncached = true;
    } else if (hipMalloc((void**)&p->win, win_bytes) != hipSuccess) {
        delete p;
        return ALLRED_ERR_NOMEM;
    }
    if (hipExtMallocWithFlags((void**)&p->flags, kPeerFlagBytes, hipDeviceMallocUncached) == hipSuccess) {
        p->flags_uncached = true;
    } else if (hipMalloc((void**)&p->flags, kPeerFlagBytes) != hipSuccess) {
        (void)hipFree(p->win);
        delete p;
        return ALLRED_ERR_NOMEM;
    }
    if (hipMalloc((void**)&p->status, 4) != hipSuccess || hipMemset(p->flags, 0, kPeerFlagBytes) != hipSuccess ||
        hipMemset(reinterpret_cast<uint8_t*>(p->win) + p->hfl_off, 0, win_bytes - p->hfl_off) != hipSuccess ||
        hipMemset(p->status, 0, 4) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        (void)hipFree(p->win);
        (void)hipFree(p->flags);
        delete p;
        return ALLRED_ERR_HIP;
    }
    *out = p;
    return ALLRED_OK;
}

int allred_peer_handle(allred_peer* p, uint8_t* out) {
    if (!p || !out) return ALLRED_ERR_ARG;
    hipIpcMemHandle_t hw, hf;
    if (hipIpcGetMemHandle(&hw, p->win) != hipSuccess) return ALLRED_ERR_HIP;
    if (hipIpcGetMemHandle(&hf, p->flags) != hipSuccess) return ALLRED_ERR_HIP;
    static_assert(sizeof(hipIpcMemHandle_t) * 2 <= ALLRED_PEER_HANDLE_BYTES, "handle size");
    std::memset(out, 0, ALLRED_PEER_HANDLE_BYTES);
    std::memcpy(out, &hw, sizeof(hw));
    std::memcpy(out + ALLRED_PEER_HANDLE_BYTES / 2, &hf, sizeof(hf));
    return ALLRED_OK;
}

int allred_peer_connect(allred_peer* p, const uint8_t* all) {
    if (!p || !all) return ALLRED_ERR_ARG;
    for (int q = 0; q < p->nranks; ++q) {
        if (q == p->rank) {
            p->peer_win[q] = p->win;
            p->peer_flags[q] = p->flags;
            p->peer_hfl[q] = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(p->win) + p->hfl_off);
            p->peer_ll[q] = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(p->win) + p->ll_off);
            continue;
        }
        hipIpcMemHandle_t hw, hf;
        std::memcpy(&hw, all + (size_t)q * ALLRED_PEER_HANDLE_BYTES, sizeof(hw));
        std::memcpy(&hf, all + (size_t)q * ALLRED_PEER_HANDLE_BYTES + ALLRED_PEER_HANDLE_BYTES / 2, sizeof(hf));
        void* w = nullptr;
        void* f = nullptr;
        if (hipIpcOpenMemHandle(&w, hw, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return ALLRED_ERR_HIP;
        if (hipIpcOpenMemHandle(&f, hf, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return ALLRED_ERR_HIP;
        p->peer_win[q] = static_cast<uint16_t*>(w);
        p->peer_flags[q] = static_cast<uint32_t*>(f);
        p->peer_hfl[q] = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(w) + p->hfl_off);
        p->peer_ll[q] = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(w) + p->ll_off);
        p->opened[q] = true;
    }
    p->connected = true;
    return ALLRED_OK;
}

namespace {

// windows of this call's parity, as mapped in this process
void parity_windows(allred_peer* p, uint16_t** wins) {
    const size_t parity = p->calls & 1u;
    for (int q = 0; q < p->nranks; ++q) wins[q] = p->peer_win[q] + parity * p->max_elems;
}

}  // namespace

int allred_peer_allreduce(allred_peer* p, uint16_t* buf, uint64_t elems, int local_ranks, int local_side,
                          int local_algo, void* workspace, void* stream) {
    if (!p || !buf || !p->connected) return ALLRED_ERR_ARG;
    const size_t n = (size_t)elems;
    if (n == 0 || n > p->max_elems || n % (8 * (size_t)p->nranks)) return ALLRED_ERR_ARG;
    uint16_t* bucket = buf;
    int st = ALLRED_OK;
    if (p->hier_ll && local_ranks == 64 && p->nranks <= 8 && p->win_uncached && n % (256 * (size_t)p->nranks) == 0 &&
        (n / 256) * 128 <= p->ll_box_words) {
        // the hierarchical step in one launch with LL (push) hand-offs (k_hier_ll): same bits
        const uint8_t* order = nullptr;
        st = local_tree_order(local_algo, local_side, local_ranks, &order);
        if (st != ALLRED_OK) return st;
        uint64_t* ll[ALLRED_MAX_NODES];
        for (int q = 0; q < p->nranks; ++q) ll[q] = p->peer_ll[q] + (p->calls & 1u) * 2 * p->ll_box_words;
        st = launch_hier_ll(buf, n, order, ll, p->nranks, p->rank, n, p->ll_box_words, p->calls + 1u, p->status,
                            stream);
        if (st != ALLRED_OK) return st;
        ++p->calls;
        p->last_all_peer = true;
        return ALLRED_OK;
    }
    const bool one_kernel = n * 2 <= p->oneshot_max && p->win_uncached && p->flags_uncached;
    if (one_kernel && local_ranks == 64 && n % (256 * (size_t)p->nranks) == 0 && 2 * n <= p->max_elems) {
        // the whole hierarchical step in one launch (k_hier_oneshot): same bits as
        // tree_reduce + the mem_2D exchange + broadcast below
        const uint8_t* order = nullptr;
        st = local_tree_order(local_algo, local_side, local_ranks, &order);
        if (st != ALLRED_OK) return st;
        uint16_t* wins[ALLRED_MAX_NODES];
        parity_windows(p, wins);
        st = launch_hier_oneshot(buf, n, order, wins, p->peer_hfl, p->nranks, p->rank, n, p->calls + 1u, p->status,
                                 stream);
        if (st != ALLRED_OK) return st;
        ++p->calls;
        p->last_all_peer = true;
        return ALLRED_OK;
    }
    if (local_ranks > 1) {
        if (!workspace) return ALLRED_ERR_ARG;
        bucket = static_cast<uint16_t*>(workspace);
        st = allred_tree_reduce(buf, n, n, local_algo, local_side, local_ranks, bucket, stream);
        if (st != ALLRED_OK) return st;
    }
    uint16_t* wins[ALLRED_MAX_NODES];
    parity_windows(p, wins);
    if (one_kernel)
        st = launch_peer_oneshot(wins, p->peer_flags, p->nranks, p->rank, bucket, n, p->calls + 1u, p->status, stream);
    else
        st = launch_peer_allreduce(wins, p->peer_flags, p->nranks, p->rank, bucket, n, 2u * p->calls + 1u, p->status,
                                   stream);
    if (st != ALLRED_OK) return st;
    ++p->calls;
    p->last_all_peer = true;
    if (local_ranks > 1) st = allred_broadcast(buf, n, n, local_ranks, bucket, stream);
    return st;
}

int allred_peer_dist_allreduce(allred_peer* p, const allred_dist_desc* d, uint16_t* buf, void* workspace,
                               void* stream) {
    if (!p || !d || !buf || !p->connected) return ALLRED_ERR_ARG;
    if (d->total_nodes != p->nranks) return ALLRED_ERR_ARG;
    const size_t n = (size_t)d->elems;
    if (d->variant == ALLRED_MEM) {
        uint16_t* ws = workspace ? static_cast<uint16_t*>(workspace) + n : nullptr;  // dist workspace layout
        return allred_peer_allreduce(p, buf, n, d->local_ranks, d->local_side, d->local_algo, ws, stream);
    }
    PeerProg prog;
    int st = peer_prog(d, p->rank, &prog);
    if (st != ALLRED_OK) return st;
    if (n > (prog.lo ? p->max_elems / 2 : p->max_elems)) return ALLRED_ERR_ARG;
    uint16_t* bucket = buf;
    if (d->local_ranks > 1) {
        if (!workspace) return ALLRED_ERR_ARG;
        bucket = static_cast<uint16_t*>(workspace) + n;
        st = allred_tree_reduce(buf, n, n, d->local_algo, d->local_side, d->local_ranks, bucket, stream);
        if (st != ALLRED_OK) return st;
    }
    if (prog.S > 0) {
        uint16_t* wins[ALLRED_MAX_NODES];
        parity_windows(p, wins);
        if (p->last_all_peer) {
            // the previous call read every rank's window, this one only waits for
            // partners: one full barrier keeps call k+2 off windows still being read
            st = launch_peer_barrier(p->peer_flags, p->nranks, p->rank, 2u * p->calls + 1u, p->status, stream);
            if (st != ALLRED_OK) return st;
        }
        st = launch_peer_sched(wins, p->peer_flags, p->rank, bucket, prog, p->max_elems / 2 / 8, p->seq, p->status,
                               stream);
        if (st != ALLRED_OK) return st;
        p->seq += 2u * (uint32_t)prog.S + 2u;
        ++p->calls;
        p->last_all_peer = false;
    }
    if (d->local_ranks > 1) st = allred_broadcast(buf, n, n, d->local_ranks, bucket, stream);
    return st;
}

int allred_peer_set_oneshot_max(allred_peer* p, uint64_t bytes) {
    if (!p) return ALLRED_ERR_ARG;
    p->oneshot_max = bytes;
    return ALLRED_OK;
}

int allred_peer_set_hier_ll(allred_peer* p, int enable) {
    if (!p) return ALLRED_ERR_ARG;
    p->hier_ll = enable != 0;
    return ALLRED_OK;
}

int allred_peer_status(allred_peer* p, uint32_t* out) {
    if (!p || !out) return ALLRED_ERR_ARG;
    if (hipMemcpy(out, p->status, 4, hipMemcpyDeviceToHost) != hipSuccess) return ALLRED_ERR_HIP;
    if (!p->win_uncached) *out |= ALLRED_PEER_WIN_CACHED;
    if (!p->flags_uncached) *out |= ALLRED_PEER_FLAGS_CACHED;
    return ALLRED_OK;
}

int allred_peer_destroy(allred_peer* p) {
    if (!p) return ALLRED_OK;
    (void)hipDeviceSynchronize();
    for (int q = 0; q < p->nranks; ++q) {
        if (!p->opened[q]) continue;
        (void)hipIpcCloseMemHandle(p->peer_win[q]);
        (void)hipIpcCloseMemHandle(p->peer_flags[q]);
    }
    (void)hipFree(p->win);
    (void)hipFree(p->flags);
    (void)hipFree(p->status);
    delete p;
    return ALLRED_OK;
}

}  // extern "C"
