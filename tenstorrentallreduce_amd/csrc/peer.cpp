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
// local ranks per GPU the local tree and the broadcast join one kernel with LL
// push hand-offs (k_hier_ws, or k_hier_x2 two buckets deep; their hand-off area
// lives in the flag allocation behind the flags).
// Windows are double-buffered by call parity: call k+2 can only overwrite a
// window after every peer passed call k+1's first barrier, i.e. finished
// reading call k's windows.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "device_guard.hpp"
#include "internal.hpp"

using namespace tsa;

struct allred_peer {
    int nranks = 0, rank = 0, device = 0;
    uint64_t max_elems = 0;
    // own windows, one allocation per parity (max_elems each): every IPC-exported
    // allocation stays <= 1 GiB + 256 B, since opening a ~2 GiB one in a peer
    // process hung on the MI355X boxes (tools/peer_open_probe.py)
    uint16_t* win[2] = {};
    uint16_t* stage = nullptr;      // staging window of the push form (k_peer_sched_push), max_elems
    uint32_t* flags = nullptr;      // own flag area (uncached), layout in internal.hpp, then the LL boxes
    uint32_t* status = nullptr;     // device status word
    bool flags_uncached = false, win_uncached = false;
    uint16_t* peer_win[ALLRED_MAX_NODES][2] = {};
    uint16_t* peer_stage[ALLRED_MAX_NODES] = {};
    uint64_t sched_push_min = 0;    // BO buckets of at least this many bytes take the push form (0: never)
    uint32_t* peer_flags[ALLRED_MAX_NODES] = {};
    bool opened[ALLRED_MAX_NODES] = {};
    uint32_t calls = 0;
    uint32_t seq = 0;               // progress-flag base of the scheduled form
    uint64_t dist_calls = 0;        // allred_peer_dist_allreduce calls (hierarchical partial halves)
    bool last_all_peer = false;     // previous call read every rank's window
    uint64_t oneshot_max = 4ull << 20;  // buckets up to this many bytes use the one-kernel form
    bool connected = false;
    // LL (push) hierarchical form: behind the per-tile flags, 2 parities x
    // [inbox ll_box_words][result box ll_box_words] 8-byte words, zeroed at create
    size_t ll_off = 0;
    uint64_t ll_box_words = 0;
    uint64_t* peer_ll[ALLRED_MAX_NODES] = {};
    // the hierarchical forms' hand-off area (6 + 2-byte words, peer_kernels.hip h_pack), behind
    // the LL boxes: 2 parities x [inbox: tiles x kHSlot words][result box: same]
    size_t hl_off = 0;
    uint64_t hl_box_words = 0;
    uint64_t* peer_hl[ALLRED_MAX_NODES] = {};
    // per parity: (tiles, call) of the calls whose words may still sit in the area, largest
    // range oldest (every call rewrites tiles [0, its tiles)); hier_area_prepare reads it
    std::vector<std::pair<uint64_t, uint32_t>> hl_stairs[2];
    uint64_t hl_clears = 0;         // barrier-protected clears of a parity's area so far
    int hier_ll = 1;                // 0 off (launch form), 1 k_hier_ws (the step in one launch, LL push hand-offs)
    uint32_t max_groups = 0;        // grid cap of the hierarchical one-kernel forms (0 = one grid per GPU)
    uint64_t lo_ll_max = 256u << 10;  // one-channel LO buckets up to this many bytes use k_peer_lo_ll
    uint64_t mem_ll_max = 256u << 10;  // mem_2D buckets up to this many bytes use k_peer_mem_ll
    // allred_peer_allreduce_pipelined2: up to two started, unfinished buckets, older
    // first; with two, the older one's owned tiles are summed already
    int x2_n = 0;
    uint16_t* x2_buf[2] = {};
    uint32_t x2_k[2] = {};          // their call numbers
    uint64_t x2_elems = 0;          // the sequence's bucket size
};

extern "C" {

int allred_peer_create(int nranks, int rank, int device, uint64_t max_elems, allred_peer** out) {
    if (!out || nranks < 1 || nranks > ALLRED_MAX_NODES || rank < 0 || rank >= nranks || max_elems == 0)
        return ALLRED_ERR_ARG;
    // every IPC-exported window <= 1 GiB: a peer's hipIpcOpenMemHandle of a ~2 GiB
    // allocation never returned (profiles/r01_peer_open_probe_2gib_hang.txt); checked
    // before any HIP call, so the limit holds (and is testable) without a GPU
    if (max_elems > ALLRED_PEER_MAX_WINDOW_BYTES / 2) return ALLRED_ERR_ARG;
    *out = nullptr;
    if (device >= 0 && hipSetDevice(device) != hipSuccess) return ALLRED_ERR_HIP;
    auto* p = new allred_peer();
    p->nranks = nranks;
    p->rank = rank;
    (void)hipGetDevice(&p->device);
    p->max_elems = (max_elems + 127) / 128 * 128;  // LO halves stay 64-element aligned (still <= 2^29)
    // windows are uncached too: peers read them over xGMI straight from HBM, so
    // no write may linger in one of this GPU's eight per-XCD L2s.  The flag
    // allocation holds, behind the flags of internal.hpp, the LL boxes for
    // buckets of up to min(max_elems, 4 Mi) elements (128 words per
    // 256-element tile), two parities of [inbox][result box].
    const uint64_t ll_elems = p->max_elems < (4ull << 20) ? p->max_elems : (4ull << 20);
    p->ll_off = ((size_t)kPeerFlagBytes + 255) / 256 * 256;
    p->ll_box_words = (ll_elems / 256) * 128;
    p->hl_off = (p->ll_off + 2 * 2 * p->ll_box_words * 8 + 255) / 256 * 256;
    p->hl_box_words = (ll_elems / 256) * kHSlot;
    const size_t flag_bytes = p->hl_off + 2 * 2 * p->hl_box_words * 8;
    const size_t win_bytes = p->max_elems * 2;
    auto release = [p]() {
        for (uint16_t* w : p->win) (void)hipFree(w);
        (void)hipFree(p->stage);
        (void)hipFree(p->flags);
        (void)hipFree(p->status);
        delete p;
    };
    p->win_uncached = true;
    for (uint16_t*& w : p->win) {
        if (hipExtMallocWithFlags((void**)&w, win_bytes, hipDeviceMallocUncached) != hipSuccess) {
            w = nullptr;
            p->win_uncached = false;
        }
    }
    if (p->win_uncached && hipExtMallocWithFlags((void**)&p->stage, win_bytes, hipDeviceMallocUncached) != hipSuccess) {
        p->stage = nullptr;
        p->win_uncached = false;
    }
    if (!p->win_uncached) {   // all cached or all uncached
        for (uint16_t*& w : p->win) {
            (void)hipFree(w);
            if (hipMalloc((void**)&w, win_bytes) != hipSuccess) {
                w = nullptr;
                release();
                return ALLRED_ERR_NOMEM;
            }
        }
        (void)hipFree(p->stage);
        if (hipMalloc((void**)&p->stage, win_bytes) != hipSuccess) {
            p->stage = nullptr;
            release();
            return ALLRED_ERR_NOMEM;
        }
    }
    if (hipExtMallocWithFlags((void**)&p->flags, flag_bytes, hipDeviceMallocUncached) == hipSuccess) {
        p->flags_uncached = true;
    } else if (hipMalloc((void**)&p->flags, flag_bytes) != hipSuccess) {
        p->flags = nullptr;
        release();
        return ALLRED_ERR_NOMEM;
    }
    if (hipMalloc((void**)&p->status, 4) != hipSuccess || hipMemset(p->flags, 0, flag_bytes) != hipSuccess ||
        hipMemset(p->status, 0, 4) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        release();
        return ALLRED_ERR_HIP;
    }
    *out = p;
    return ALLRED_OK;
}

int allred_peer_handle(allred_peer* p, uint8_t* out) {
    if (!p || !out) return ALLRED_ERR_ARG;
    // [window parity 0][window parity 1][flags][staging window], 64 bytes each
    static_assert(sizeof(hipIpcMemHandle_t) * 4 <= ALLRED_PEER_HANDLE_BYTES, "handle size");
    hipIpcMemHandle_t h[4];
    if (hipIpcGetMemHandle(&h[0], p->win[0]) != hipSuccess) return ALLRED_ERR_HIP;
    if (hipIpcGetMemHandle(&h[1], p->win[1]) != hipSuccess) return ALLRED_ERR_HIP;
    if (hipIpcGetMemHandle(&h[2], p->flags) != hipSuccess) return ALLRED_ERR_HIP;
    if (hipIpcGetMemHandle(&h[3], p->stage) != hipSuccess) return ALLRED_ERR_HIP;
    std::memset(out, 0, ALLRED_PEER_HANDLE_BYTES);
    for (int i = 0; i < 4; ++i) std::memcpy(out + i * sizeof(hipIpcMemHandle_t), &h[i], sizeof(h[i]));
    return ALLRED_OK;
}

int allred_peer_connect(allred_peer* p, const uint8_t* all) {
    if (!p || !all || p->connected) return ALLRED_ERR_ARG;
    DeviceGuard guard(p->device);   // the peers' windows are mapped for this peer's device
    if (!guard.ok) return ALLRED_ERR_HIP;
    for (int q = 0; q < p->nranks; ++q) {
        if (q == p->rank) {
            p->peer_win[q][0] = p->win[0];
            p->peer_win[q][1] = p->win[1];
            p->peer_flags[q] = p->flags;
            p->peer_stage[q] = p->stage;
        } else {
            void* m[4] = {};
            for (int i = 0; i < 4; ++i) {
                hipIpcMemHandle_t h;
                std::memcpy(&h, all + (size_t)q * ALLRED_PEER_HANDLE_BYTES + i * sizeof(h), sizeof(h));
                if (hipIpcOpenMemHandle(&m[i], h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                    for (int k = 0; k < i; ++k) (void)hipIpcCloseMemHandle(m[k]);
                    return ALLRED_ERR_HIP;   // peers opened so far stay in opened[] for destroy
                }
            }
            p->peer_win[q][0] = static_cast<uint16_t*>(m[0]);
            p->peer_win[q][1] = static_cast<uint16_t*>(m[1]);
            p->peer_flags[q] = static_cast<uint32_t*>(m[2]);
            p->peer_stage[q] = static_cast<uint16_t*>(m[3]);
            p->opened[q] = true;
        }
        uint8_t* f = reinterpret_cast<uint8_t*>(p->peer_flags[q]);
        p->peer_ll[q] = reinterpret_cast<uint64_t*>(f + p->ll_off);
        p->peer_hl[q] = reinterpret_cast<uint64_t*>(f + p->hl_off);
    }
    p->connected = true;
    return ALLRED_OK;
}

int allred_peer_connect_all(int nranks, allred_peer* const* peers) {
    if (!peers || nranks < 1 || nranks > ALLRED_MAX_NODES) return ALLRED_ERR_ARG;
    for (int q = 0; q < nranks; ++q)
        if (!peers[q] || peers[q]->connected || peers[q]->nranks != nranks || peers[q]->rank != q) return ALLRED_ERR_ARG;
    for (int me = 0; me < nranks; ++me) {
        allred_peer* p = peers[me];
        DeviceGuard guard(p->device);
        if (!guard.ok) return ALLRED_ERR_HIP;
        for (int q = 0; q < nranks; ++q) {
            const allred_peer* o = peers[q];
            if (o->device != p->device) {   // another GPU of this process: map it (xGMI)
                const hipError_t e = hipDeviceEnablePeerAccess(o->device, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return ALLRED_ERR_HIP;
                (void)hipGetLastError();
            }
            p->peer_win[q][0] = o->win[0];
            p->peer_win[q][1] = o->win[1];
            p->peer_flags[q] = o->flags;
            p->peer_stage[q] = o->stage;
            uint8_t* f = reinterpret_cast<uint8_t*>(o->flags);
            p->peer_ll[q] = reinterpret_cast<uint64_t*>(f + o->ll_off);
            p->peer_hl[q] = reinterpret_cast<uint64_t*>(f + o->hl_off);
        }
    }
    for (int q = 0; q < nranks; ++q) peers[q]->connected = true;   // opened[] stays false: nothing to close
    return ALLRED_OK;
}

namespace {

// windows of this call's parity, as mapped in this process
void parity_windows(allred_peer* p, uint16_t** wins) {
    const size_t parity = p->calls & 1u;
    for (int q = 0; q < p->nranks; ++q) wins[q] = p->peer_win[q][parity];
}

// every GPU's hand-off area of call k's parity (the hierarchical forms)
void hier_areas(const allred_peer* p, uint32_t k, uint64_t** hl) {
    for (int q = 0; q < p->nranks; ++q) hl[q] = p->peer_hl[q] + (k & 1u) * 2 * p->hl_box_words;
}

// A bucket of `tiles` tiles starts at call k on parity k & 1 of the hand-off area.  Its
// readers accept a word whose 16-bit epoch is h_epoch(k + 1) = (k + 1) % 65535 + 1; a slot
// of its range still holding a word of an older same-parity call k' with k' = k (mod 65535)
// — k - k' a multiple of 131070 — would be taken as this call's.  Every call rewrites all
// slots of its own range, so the oldest word in [0, tiles) is the one the newest call
// covering slot tiles - 1 wrote (never written: zero, epoch 0, never awaited).  If that
// call is 131070 or more calls back, the parity's area is cleared first, between two
// barriers of the whole peer set (every GPU runs the same calls, so all take this path
// together): after the first no GPU is still writing into any area (each finished its
// previous launches, whose words every consumer had taken), before the second every GPU
// has cleared its own.  Call with no pipelined bucket pending on that parity.
constexpr uint32_t kHierWrapCalls = 131070;   // 2 x 65535: same-parity calls between equal epochs

void hier_area_note(allred_peer* p, uint64_t tiles, uint32_t k) {
    auto& st = p->hl_stairs[k & 1u];
    while (!st.empty() && st.back().first <= tiles) st.pop_back();
    st.emplace_back(tiles, k);
}

// The call whose words are the oldest ones in slots [0, tiles) of a parity's area: the
// newest call covering the highest written slot of the range, min(tiles, front's range) - 1
// (the stairs' front covers the most slots; beyond them nothing was written since the last
// clear).  A bucket larger than every entry therefore checks the front — the oldest call
// still in the area — not nothing.  None: the area holds no word (nothing to clear).
bool hier_area_oldest(const std::vector<std::pair<uint64_t, uint32_t>>& st, uint64_t tiles, uint32_t* call) {
    if (st.empty() || tiles == 0) return false;
    const uint64_t reach = tiles < st.front().first ? tiles : st.front().first;
    for (auto it = st.rbegin(); it != st.rend(); ++it)
        if (it->first >= reach) {
            *call = it->second;
            return true;
        }
    return false;   // unreachable: the front covers `reach`
}

int hier_area_prepare(allred_peer* p, uint64_t tiles, uint32_t k, void* stream) {
    auto& st = p->hl_stairs[k & 1u];
    uint32_t oldest = 0;
    if (hier_area_oldest(st, tiles, &oldest) && k - oldest >= kHierWrapCalls) {
        const uint32_t e = 2u * p->calls + 1u;   // barrier epochs: monotonic with every other barrier user
        int rc = launch_peer_barrier(p->peer_flags, p->nranks, p->rank, e, p->status, stream);
        if (rc != ALLRED_OK) return rc;
        if (hipMemsetAsync(p->peer_hl[p->rank] + (k & 1u) * 2 * p->hl_box_words, 0, 2 * p->hl_box_words * 8,
                           (hipStream_t)stream) != hipSuccess)
            return ALLRED_ERR_HIP;
        rc = launch_peer_barrier(p->peer_flags, p->nranks, p->rank, e + 1u, p->status, stream);
        if (rc != ALLRED_OK) return rc;
        st.clear();
        ++p->hl_clears;
    }
    hier_area_note(p, tiles, k);
    return ALLRED_OK;
}

}  // namespace

int allred_peer_allreduce_pipelined2(allred_peer* p, uint16_t* cur, uint64_t elems, int local_ranks, int local_side,
                                     int local_algo, void* stream) {
    if (!p || !p->connected) return ALLRED_ERR_ARG;
    const size_t n = (size_t)elems;
    if (n == 0 || n > p->max_elems || n % (256 * (size_t)p->nranks)) return ALLRED_ERR_ARG;
    if (local_ranks != 64 || p->nranks > 8 || !p->flags_uncached || (n / 256) * kHSlot > p->hl_box_words)
        return ALLRED_ERR_UNSUPPORTED;
    if ((p->x2_n > 0 && n != p->x2_elems) || (!cur && p->x2_n == 0)) return ALLRED_ERR_ARG;
    const uint8_t* order = nullptr;
    int st = local_tree_order(local_algo, local_side, local_ranks, &order);
    if (st != ALLRED_OK) return st;
    auto area = [&](uint32_t k, uint64_t** ll) { hier_areas(p, k, ll); };   // every GPU's area of call k's parity
    // mid: the newest pending bucket (its owned tiles are summed by this launch);
    // old: the older one when two are pending (its rows are written by this launch)
    const bool has_old = p->x2_n == 2;
    const uint32_t kc = p->calls, km = p->x2_k[p->x2_n - 1 < 0 ? 0 : p->x2_n - 1], ko = p->x2_k[0];
    uint64_t* llc[ALLRED_MAX_NODES];
    uint64_t* llm[ALLRED_MAX_NODES];
    uint64_t* llo[ALLRED_MAX_NODES];
    area(kc, llc);
    area(km, llm);
    area(ko, llo);
    uint16_t* old = has_old ? p->x2_buf[0] : nullptr;
    uint16_t* fin = !cur ? p->x2_buf[p->x2_n - 1] : nullptr;
    // cur's parity is old's: a sequence's buckets share one size, so only its first two starts
    // (nothing pending on cur's parity yet) can meet slots an earlier, smaller bucket left
    if (cur && p->x2_n < 2 && (st = hier_area_prepare(p, n / 256, kc, stream)) != ALLRED_OK) return st;
    if (cur && p->x2_n == 2) hier_area_note(p, n / 256, kc);
    st = launch_hier_x2(cur, old, fin, n, order, cur ? llc : nullptr, p->x2_n > 0 ? llm : nullptr,
                        has_old ? llo : nullptr, p->nranks, p->rank, n, p->hl_box_words, kc + 1u, km + 1u, ko + 1u,
                        p->status, p->max_groups, stream);
    if (st != ALLRED_OK) return st;
    if (!cur) {   // flushed: nothing pending
        p->x2_n = 0;
    } else {
        if (has_old) {   // old done: mid becomes the older pending bucket
            p->x2_buf[0] = p->x2_buf[1];
            p->x2_k[0] = p->x2_k[1];
            p->x2_n = 1;
        }
        p->x2_buf[p->x2_n] = cur;
        p->x2_k[p->x2_n] = kc;
        ++p->x2_n;
        p->x2_elems = n;
        ++p->calls;
    }
    p->last_all_peer = true;
    return ALLRED_OK;
}

int allred_peer_allreduce(allred_peer* p, uint16_t* buf, uint64_t elems, int local_ranks, int local_side,
                          int local_algo, void* workspace, void* stream) {
    if (!p || !buf || !p->connected) return ALLRED_ERR_ARG;
    if (p->x2_n) return ALLRED_ERR_ARG;   // finish the pipelined sequence first
    const size_t n = (size_t)elems;
    if (n == 0 || n > p->max_elems || n % (8 * (size_t)p->nranks)) return ALLRED_ERR_ARG;
    uint16_t* bucket = buf;
    int st = ALLRED_OK;
    if (p->hier_ll && local_ranks == 64 && p->nranks <= 8 && p->flags_uncached && n % (256 * (size_t)p->nranks) == 0 &&
        (n / 256) * kHSlot <= p->hl_box_words) {
        // the hierarchical step in one launch with LL (push) hand-offs (k_hier_ws): same bits
        const uint8_t* order = nullptr;
        st = local_tree_order(local_algo, local_side, local_ranks, &order);
        if (st != ALLRED_OK) return st;
        uint64_t* ll[ALLRED_MAX_NODES];
        hier_areas(p, p->calls, ll);
        if ((st = hier_area_prepare(p, n / 256, p->calls, stream)) != ALLRED_OK) return st;
        st = launch_hier_ws(buf, n, order, ll, p->nranks, p->rank, n, p->hl_box_words, p->calls + 1u, p->status,
                            p->max_groups, stream);
        if (st != ALLRED_OK) return st;
        ++p->calls;
        p->last_all_peer = true;
        return ALLRED_OK;
    }
    const bool one_kernel = n * 2 <= p->oneshot_max && p->win_uncached && p->flags_uncached;
    if (local_ranks > 1) {
        if (!workspace) return ALLRED_ERR_ARG;
        bucket = static_cast<uint16_t*>(workspace);
        st = allred_tree_reduce(buf, n, n, local_algo, local_side, local_ranks, bucket, stream);
        if (st != ALLRED_OK) return st;
    }
    const uint64_t ll_area = 2 * p->ll_box_words;   // LL words of one parity
    if (p->mem_ll_max && n * 2 <= p->mem_ll_max && p->nranks <= 8 && p->flags_uncached && (n / 8 + 31) / 32 * 32 * 8 <= ll_area) {
        // small buckets: LL pushes, two one-way trips (k_peer_mem_ll); same bits
        uint64_t* ll[ALLRED_MAX_NODES];
        for (int q = 0; q < p->nranks; ++q) ll[q] = p->peer_ll[q] + (p->calls & 1u) * ll_area;
        st = launch_peer_mem_ll(ll, p->nranks, p->rank, bucket, n, ll_area, p->calls + 1u, p->status, p->max_groups,
                                stream);
        if (st != ALLRED_OK) return st;
        ++p->calls;
        p->last_all_peer = false;   // no window was read; every rank finished the call before
        if (local_ranks > 1) st = allred_broadcast(buf, n, n, local_ranks, bucket, stream);
        return st;
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
    if (d->total_nodes != p->nranks || p->x2_n) return ALLRED_ERR_ARG;
    const size_t n = (size_t)d->elems;
    if (d->variant == ALLRED_MEM) {
        // the peer mem_2D kernels sum in fp32 with one rounding; the reference's bf16
        // dest-register accumulation runs over RCCL (launch_rows_sum) only
        if (d->mem_accum == ALLRED_ACC_BF16) return ALLRED_ERR_UNSUPPORTED;
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
        // the partial alternates between the workspace's halves (as allred_dist_allreduce)
        bucket = static_cast<uint16_t*>(workspace) + ((p->dist_calls++ & 1) ? 0 : n);
        st = allred_tree_reduce(buf, n, n, d->local_algo, d->local_side, d->local_ranks, bucket, stream);
        if (st != ALLRED_OK) return st;
    }
    const uint64_t ll_area = 2 * p->ll_box_words;   // LL words of one parity
    if (prog.S > 0 && prog.lo && prog.C == 1 && p->lo_ll_max && n * 2 <= p->lo_ll_max && p->nranks <= 8 &&
        p->flags_uncached && (n / 8 + 31) / 32 * 32 * 4 * (uint64_t)prog.S <= ll_area) {
        // small LO buckets: LL pushes, one one-way trip per step (k_peer_lo_ll); same bits
        uint64_t* ll[ALLRED_MAX_NODES];
        for (int q = 0; q < p->nranks; ++q) ll[q] = p->peer_ll[q] + (p->calls & 1u) * ll_area;
        st = launch_peer_lo_ll(ll, p->nranks, p->rank, bucket, prog, n, ll_area, p->calls + 1u, p->status, stream);
        if (st != ALLRED_OK) return st;
        ++p->calls;
        p->last_all_peer = false;   // no window was touched; every rank finished the call before
    } else if (prog.S > 0) {
        uint16_t* wins[ALLRED_MAX_NODES];
        parity_windows(p, wins);
        if (p->last_all_peer) {
            // the previous call read every rank's window, this one only waits for
            // partners: one full barrier keeps call k+2 off windows still being read
            st = launch_peer_barrier(p->peer_flags, p->nranks, p->rank, 2u * p->calls + 1u, p->status, stream);
            if (st != ALLRED_OK) return st;
        }
        if (!prog.lo && p->sched_push_min && n * 2 >= p->sched_push_min)   // the push form: same program, same bits
            st = launch_peer_sched_push(wins, p->peer_stage, p->peer_flags, p->rank, bucket, prog, p->seq, p->status,
                                        p->max_groups, stream);
        else
            st = launch_peer_sched(wins, p->peer_flags, p->rank, bucket, prog, p->max_elems / 2 / 8, p->seq, p->status,
                                   p->max_groups, stream);
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
    if (enable < 0 || enable > 1) return ALLRED_ERR_ARG;
    p->hier_ll = enable;
    return ALLRED_OK;
}

int allred_peer_set_sched_push(allred_peer* p, uint64_t min_bytes) {
    if (!p) return ALLRED_ERR_ARG;
    p->sched_push_min = min_bytes;
    return ALLRED_OK;
}

int allred_peer_set_lo_ll_max(allred_peer* p, uint64_t bytes) {
    if (!p) return ALLRED_ERR_ARG;
    p->lo_ll_max = bytes;
    return ALLRED_OK;
}

int allred_peer_set_mem_ll_max(allred_peer* p, uint64_t bytes) {
    if (!p) return ALLRED_ERR_ARG;
    p->mem_ll_max = bytes;
    return ALLRED_OK;
}

int allred_peer_set_max_groups(allred_peer* p, uint32_t groups) {
    if (!p) return ALLRED_ERR_ARG;
    p->max_groups = groups;
    return ALLRED_OK;
}

int allred_peer_status(allred_peer* p, uint32_t* out) {
    if (!p || !out) return ALLRED_ERR_ARG;
    if (hipMemcpy(out, p->status, 4, hipMemcpyDeviceToHost) != hipSuccess) return ALLRED_ERR_HIP;
    if (!p->win_uncached) *out |= ALLRED_PEER_WIN_CACHED;
    if (!p->flags_uncached) *out |= ALLRED_PEER_FLAGS_CACHED;
    return ALLRED_OK;
}

int allred_peer_clear_status(allred_peer* p) {
    if (!p) return ALLRED_ERR_ARG;
    if (p->x2_n) return ALLRED_ERR_ARG;   // a pipelined sequence is open: flush it first
    DeviceGuard guard(p->device);
    // the null stream only (no device-wide sync: other groups of this process may be mid-exchange)
    if (hipMemsetAsync(p->status, 0, 4, nullptr) != hipSuccess || hipStreamSynchronize(nullptr) != hipSuccess)
        return ALLRED_ERR_HIP;
    return ALLRED_OK;
}

int allred_peer_check(allred_peer* p, void* stream) {
    if (!p) return ALLRED_ERR_ARG;
    // the status word read on the caller's stream: nothing on the null stream, which every
    // thread of the process shares (in-process peers on one GPU must not queue behind each other)
    uint32_t st = 0;
    if (hipMemcpyAsync(&st, p->status, 4, hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
        hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
        return ALLRED_ERR_HIP;
    return (st & ALLRED_PEER_TIMEOUT) ? ALLRED_ERR_TRANSPORT : ALLRED_OK;
}

int allred_peer_destroy(allred_peer* p) {
    if (!p) return ALLRED_OK;
    (void)hipDeviceSynchronize();
    for (int q = 0; q < p->nranks; ++q) {
        if (!p->opened[q]) continue;
        (void)hipIpcCloseMemHandle(p->peer_win[q][0]);
        (void)hipIpcCloseMemHandle(p->peer_win[q][1]);
        (void)hipIpcCloseMemHandle(p->peer_flags[q]);
        (void)hipIpcCloseMemHandle(p->peer_stage[q]);
    }
    for (uint16_t* w : p->win) (void)hipFree(w);
    (void)hipFree(p->stage);
    (void)hipFree(p->flags);
    (void)hipFree(p->status);
    delete p;
    return ALLRED_OK;
}

}  // extern "C"
