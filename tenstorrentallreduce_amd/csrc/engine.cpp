// engine.cpp — virtual-rank allreduce plans (N ranks in one GPU's HBM) and
// the reference program surface (AllredConfig + RunProgram).
//
// A plan replaces the 64-core Tensix program of the reference:
//   BO  = reduce-scatter + all-gather over the schedule's block masks
//         (allred_BO_2D/kernels/dataflow_kernel.cpp:152-267, compute_kernel.cpp:35-67)
//   LO  = full-vector exchange + add per step (same kernels, bandwidth_optimal = 0;
//         allred_LOO_2D/kernels/dataflow_kernel.cpp for NUM_TILES < 64)
//   MEM = reduce own block from the shared buffer, then read everything back
//         (allred_mem_2D/kernels/*)
// ALLRED_EXEC_STEPS keeps the reference's step structure (every step's result
// stored to the ranks' buckets; BO / LO as one persistent launch of
// independent (block, column slice) units, k_bo_steps / k_lo_steps; MEM as
// reduce + broadcast); ALLRED_EXEC_FUSED does the identical arithmetic in one
// HBM pass (BO: k_tree*, LO: the butterfly k_butterfly*, or the BO tree pass
// when every rank's tree is the same (lo_rank_uniform), MEM: k_mem*).
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "device_guard.hpp"
#include "internal.hpp"

using namespace tsa;

struct allred_plan {
    allred_plan_desc desc{};
    allred_schedule sched{};
    int total = 1;
    int device = 0;
    size_t n = 0;           // elements per rank
    size_t block_elems = 0; // BO/MEM block
    // device tables
    int16_t* d_partner = nullptr;           // [steps][total]
    int16_t* d_rs_blocks = nullptr;         // per step: total * m_k entries (recv mask blocks)
    int16_t* d_ag_blocks = nullptr;         // per step: total * m_k entries (send mask blocks)
    std::vector<size_t> blk_off;            // offset of step k in the block tables
    std::vector<int> blk_per_rank;          // m_k
    uint8_t* d_order = nullptr;
    uint8_t* d_dag = nullptr;               // LO: interned DAG (lo_dag_lanes form), 64 ranks only
    uint8_t* d_steps_tab = nullptr;         // schedule form, one launch: BO per-block phase ranks / LO step pairs
    uint8_t* d_steps_pipe_tab = nullptr;    // the same programs in the pipelined form's layout (k_steps_pipe)
    bool steps_reg_tab = false;             // BO: k_steps_reg's program appended to d_steps_pipe_tab
    bool steps_persistent = false;          // schedule form as one launch (k_bo_steps / k_lo_steps)
    size_t ws_bytes = 0;
    int launches = 0;
    // memory type of recent bucket pointers (pinned host buckets take the
    // zero-copy form): a rotation of up to kPtrCache bucket sets costs one
    // hipPointerGetAttributes each, once
    static constexpr int kPtrCache = 64;
    const void* ptr_seen[kPtrCache] = {};
    bool ptr_host[kPtrCache] = {};
    int ptr_next = 0;
    bool lo_tree = false;  // fused LO runs as the BO tree pass (lo_rank_uniform)
};

namespace {

int popcount64(uint64_t x) { return __builtin_popcountll(x); }

void free_plan(allred_plan* p) {
    if (!p) return;
    if (p->d_partner) (void)hipFree(p->d_partner);
    if (p->d_rs_blocks) (void)hipFree(p->d_rs_blocks);
    if (p->d_ag_blocks) (void)hipFree(p->d_ag_blocks);
    if (p->d_order) (void)hipFree(p->d_order);
    if (p->d_dag) (void)hipFree(p->d_dag);
    if (p->d_steps_tab) (void)hipFree(p->d_steps_tab);
    if (p->d_steps_pipe_tab) (void)hipFree(p->d_steps_pipe_tab);
    delete p;
}

template <typename T>
int upload(T** dst, const std::vector<T>& host) {
    if (host.empty()) return ALLRED_OK;
    if (hipMalloc((void**)dst, host.size() * sizeof(T)) != hipSuccess) return ALLRED_ERR_NOMEM;
    if (hipMemcpy(*dst, host.data(), host.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
        return ALLRED_ERR_HIP;
    return ALLRED_OK;
}

// True when every rank's LO tree is the same tree up to swapping children:
// then the butterfly leaves the same bits on every rank (the fp32 add of two
// bf16 is commutative), and rank r's LO result — its own tree T(r), leaves
// tree_order[r] — is BO block r's result, which is T(r) too (the BO partial of
// block r at step k is exactly the LO value of its holder).  So the fused LO
// is the fused BO pass, one tree per column instead of one per rank: every
// RecDub schedule, Swing up to 16 ranks (tests/test_gpu_parity.py holds both
// against the oracle's butterfly).
bool lo_rank_uniform(const allred_schedule& s, int total) {
    std::map<std::pair<int, int>, int> ids;  // interned unordered pairs of subtrees
    std::vector<int> cur(total), nxt(total);
    for (int r = 0; r < total; ++r) cur[r] = r;
    for (int k = 0; k < s.steps; ++k) {
        for (int r = 0; r < total; ++r) {
            const int a = cur[r], b = cur[s.partner[r][k]];
            const auto key = a < b ? std::make_pair(a, b) : std::make_pair(b, a);
            const auto it = ids.emplace(key, total + (int)ids.size()).first;
            nxt[r] = it->second;
        }
        cur.swap(nxt);
    }
    for (int r = 1; r < total; ++r)
        if (cur[r] != cur[0]) return false;
    return true;
}

bool env_is(const char* name, const char* value) {
    const char* v = std::getenv(name);
    return v && std::string(v) == value;
}

// BO schedule form (k_bo_steps, kernels.hip): per block b, in phase order,
//   RS step 0          (r, p) for the N/2 holders r of b (recv_0(r) has b), row i = i-th holder
//   RS 1..S-1, AG S-1..1  (row of r, row of p) for the step's N >> (k+1) writers r (RS:
//                      holders of b, AG: receivers, b in send_k(r)), p = partner_k(r)
//   AG step 0          (r, row of p) for the N/2 receivers r (the step-0 non-holders)
//   then the N/2 holders' ranks in row order.
// Every operand of steps >= 1 is a step-0 holder's row (a partner that sends b
// at RS step k held b at step k-1; AG steps >= 1 stay among the holders), which
// the builder checks: 4(N-1) + N/2 bytes per block, empty if the check fails.
std::vector<uint8_t> bo_steps_table(const allred_schedule& s, int N) {
    const int S = s.steps, H = N / 2;
    std::vector<uint8_t> tab;
    for (int b = 0; b < N; ++b) {
        std::vector<int> row(N, -1), holders;
        for (int r = 0; r < N; ++r)
            if ((s.recv[r][0] >> b) & 1ull) row[r] = (int)holders.size(), holders.push_back(r);
        if ((int)holders.size() != H) return {};
        for (int r : holders) {
            tab.push_back((uint8_t)r);
            tab.push_back((uint8_t)s.partner[r][0]);
        }
        for (int q = 1; q < 2 * S; ++q) {
            const bool rs = q < S;
            const int k = rs ? q : 2 * S - 1 - q;
            int cnt = 0;
            for (int r = 0; r < N; ++r) {
                const uint64_t m = rs ? s.recv[r][k] : s.send[r][k];
                if (!((m >> b) & 1ull)) continue;
                const int p = s.partner[r][k];
                if (row[p] < 0) return {};
                if (q < 2 * S - 1) {
                    if (row[r] < 0) return {};
                    tab.push_back((uint8_t)row[r]);
                } else {
                    tab.push_back((uint8_t)r);
                }
                tab.push_back((uint8_t)row[p]);
                ++cnt;
            }
            if (cnt != (N >> (k + 1))) return {};
        }
        if (S == 0) return {};
        for (int r : holders) tab.push_back((uint8_t)r);
    }
    return tab;
}

// The BO program in k_steps_pipe's layout, 256 bytes per block: phase 0 and
// phases 1 .. 2S-2 as in bo_steps_table, then N bytes: the row holding rank
// r's result after AG step 0 (holders: their own row; receivers: the row of
// their step-0 partner, whose copy AG step 0 sends them).
std::vector<uint8_t> bo_steps_pipe_table(const std::vector<uint8_t>& tab, int N, int S) {
    if (S < 1 || N < 2 || tab.empty()) return {};
    const int H = N / 2, L = 4 * (N - 1) + H, body = 2 * H + 2 * (H - 1) * 2;
    if (tab.size() != (size_t)L * N || body + N > kBoPipeTabBytes) return {};
    std::vector<uint8_t> out((size_t)kBoPipeTabBytes * N, 0);
    for (int b = 0; b < N; ++b) {
        const uint8_t* t = &tab[(size_t)b * L];
        uint8_t* o = &out[(size_t)b * kBoPipeTabBytes];
        std::memcpy(o, t, (size_t)body);
        const uint8_t* ag0 = t + body;          // (receiver r, row of its partner) x H
        const uint8_t* holders = ag0 + 2 * H;   // holder ranks, row order
        for (int x = 0; x < H; ++x) {
            o[body + ag0[2 * x]] = ag0[2 * x + 1];
            o[body + holders[x]] = (uint8_t)x;
        }
    }
    return out;
}

// The BO program for the register-staged schedule form (k_steps_reg), appended
// to the pipe table: N blocks x 256 bytes, the pipe layout with step 0 recast
// for loads that cannot depend on the block — the step-0 pairs are the same
// for every block, only which of the two ranks holds (keeps the sum, adds
// first) and the holder's row differ.  Pair u = the u-th (r, partner_0(r)) with
// r < partner in rank order; byte u of a block = its row x | 0x80 when the
// higher rank holds; bytes H .. 2H-1 zero; phases and result rows as the pipe
// table.  Then the H pairs' ranks (2 bytes each), shared by every block.
// Empty if the step-0 pairs are not the pipe table's (never for a valid schedule).
std::vector<uint8_t> bo_steps_reg_table(const std::vector<uint8_t>& pipe, const allred_schedule& s, int N) {
    const int H = N / 2;
    if (pipe.size() != (size_t)kBoPipeTabBytes * N || s.steps < 1) return {};
    std::vector<uint8_t> pr;
    for (int r = 0; r < N; ++r)
        if (r < s.partner[r][0]) pr.push_back((uint8_t)r), pr.push_back((uint8_t)s.partner[r][0]);
    if ((int)pr.size() != 2 * H) return {};
    std::vector<uint8_t> out(pipe);
    for (int b = 0; b < N; ++b) {
        const uint8_t* t = &pipe[(size_t)b * kBoPipeTabBytes];
        uint8_t* o = &out[(size_t)b * kBoPipeTabBytes];
        std::memset(o, 0, 2 * (size_t)H);
        std::vector<int> seen(H, 0);
        for (int x = 0; x < H; ++x) {
            const int r = t[2 * x], q = t[2 * x + 1], lo = r < q ? r : q, hi = r < q ? q : r;
            int u = 0;
            while (u < H && !(pr[2 * u] == lo && pr[2 * u + 1] == hi)) ++u;
            if (u == H || seen[u]++) return {};
            o[u] = (uint8_t)(x | (r == hi ? 0x80 : 0));
        }
    }
    out.insert(out.end(), pr.begin(), pr.end());
    return out;
}

// LO schedule form (k_lo_steps, kernels.hip): per step, the N/2 exchanging
// pairs (r, p), r < p, numbered in order (after step k, pair i's two ranks
// hold the same value: LDS row i); then per step k >= 1, for each of its pairs
// the rows of its two ranks after step k-1.
std::vector<uint8_t> lo_steps_pairs(const allred_schedule& s, int N) {
    const int S = s.steps;
    std::vector<uint8_t> pairs, rows;
    std::vector<int> prev(N, -1), cur(N, -1);
    for (int k = 0; k < S; ++k) {
        int cnt = 0;
        for (int r = 0; r < N; ++r) {
            const int p = s.partner[r][k];
            if (r >= p) continue;
            pairs.push_back((uint8_t)r);
            pairs.push_back((uint8_t)p);
            if (k > 0) {
                rows.push_back((uint8_t)prev[r]);
                rows.push_back((uint8_t)prev[p]);
            }
            cur[r] = cur[p] = cnt++;
        }
        if (cnt != N / 2) return {};
        prev = cur;
    }
    pairs.insert(pairs.end(), rows.begin(), rows.end());
    return pairs;
}

// The LO program in k_steps_pipe's layout: step 0's N/2 (r, p) rank pairs ->
// row i; steps 1 .. S-1's (row of r, row of p) per pair; then N bytes: rank
// r's pair (row) at the last step.  A pair (r, p) of step k holds one value
// for both its ranks, so each row of step k-1 is an operand of exactly two
// pairs of step k: the operand graph is 2-regular (a union of cycles), and
// walking each cycle assigns every pair of step k one of its operand rows as
// its own row, a different one for every pair.  The table lists that operand
// first (a == x for pair x), so the lane that computed row x at step k-1 keeps
// it in a register and reads only the other operand from LDS.
std::vector<uint8_t> lo_steps_pipe_table(const allred_schedule& s, int N) {
    const int S = s.steps, H = N / 2;
    if (S == 0 || N < 2) return {};
    std::vector<uint8_t> out;
    std::vector<int> row(N, -1), nrow(N, -1);
    int cnt = 0;
    for (int r = 0; r < N; ++r) {   // step 0: pairs in rank order
        const int p = s.partner[r][0];
        if (r >= p) continue;
        out.push_back((uint8_t)r);
        out.push_back((uint8_t)p);
        row[r] = row[p] = cnt++;
    }
    if (cnt != H) return {};
    for (int k = 1; k < S; ++k) {
        // this step's pairs as edges between the previous step's rows
        std::vector<std::pair<int, int>> edge;   // (rank r, rank p), r < p
        std::vector<std::vector<int>> at(H);     // row -> incident edges
        for (int r = 0; r < N; ++r) {
            const int p = s.partner[r][k];
            if (r >= p) continue;
            at[row[r]].push_back((int)edge.size());
            at[row[p]].push_back((int)edge.size());
            edge.emplace_back(r, p);
        }
        if ((int)edge.size() != H) return {};
        for (const auto& a : at)
            if (a.size() != 2) return {};
        // walk every cycle: edge e leaves row u and is assigned to u
        std::vector<int> own(H, -1);   // edge -> its row
        std::vector<bool> used(H, false);
        for (int start = 0; start < H; ++start) {
            if (used[start]) continue;
            int u = start, e = at[u][0];
            while (own[e] < 0) {
                own[e] = u;
                used[u] = true;
                const int a = row[edge[e].first], b = row[edge[e].second];
                const int v = a == u ? b : a;   // the edge's other end
                e = at[v][0] == e ? at[v][1] : at[v][0];
                u = v;
            }
        }
        std::vector<uint8_t> step(2 * H, 0);
        for (int e = 0; e < H; ++e) {
            const int x = own[e];
            if (x < 0) return {};
            const int a = row[edge[e].first], b = row[edge[e].second];
            step[2 * x] = (uint8_t)x;               // kept in a register
            step[2 * x + 1] = (uint8_t)(a == x ? b : a);
            nrow[edge[e].first] = nrow[edge[e].second] = x;
        }
        out.insert(out.end(), step.begin(), step.end());
        row = nrow;
    }
    for (int r = 0; r < N; ++r) out.push_back((uint8_t)row[r]);
    return out;
}

// The LO butterfly as a DAG of its distinct sums, for the LDS pass of 64 ranks
// (k_butterfly_lds64_pipe<4>): step k's nodes are the distinct unordered pairs
// (value of r, value of partner_k(r)) of step-(k-1) values, numbered in order
// of first appearance.  Each node gets a kernel slot s (lane group s % 8, item
// s / 8) and an LDS tile row; both are free choices (writes of a step never
// conflict, its reads are all issued before them), so lo_dag_place() picks
// them such that every ds_read_b128 of the pass is bank-conflict free.
// Layout: [k*64 + 2s], [k*64 + 2s + 1] = input rows of the node in slot s
// (0xFF: empty slot), [384 + r] = final row of rank r, [448 + k] = d_k,
// [456 + 32k + s] = row the node in slot s is written to.  Empty when a step
// would have more than 32 nodes (a kernel lane group serves at most 4 x 8).
constexpr size_t kDagBytes = 456 + 32 * ALLRED_MAX_STEPS;

// Extra LDS cycles of the reads of one step: ds_read_b128 serves a wave in
// four 16-lane groups (MI355X_MICROARCH.md §LDS); lane 8g + col of item i
// reads operand row R at 16-byte slot R*32 + ((8w + col) ^ (R & 31)) (the
// tile swizzle), banks (address mod 16 slots); w only flips one address bit
// for every lane alike, so w = 0 stands for all waves.
int lo_dag_step_conflicts(const std::vector<std::pair<int, int>>& ops, const std::vector<int>& slot_of,
                          const std::vector<int>& in_row) {
    static const int groups[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                      {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                      {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                      {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
    int node_at[32];
    for (int& v : node_at) v = -1;
    for (size_t q = 0; q < slot_of.size(); ++q) node_at[slot_of[q]] = (int)q;
    int extra = 0;
    for (int i = 0; i < 4; ++i)
        for (int which = 0; which < 2; ++which)
            for (const auto& grp : groups) {
                int addr[16], n = 0, worst = 0;
                for (int lane : grp) {
                    const int q = node_at[8 * i + (lane >> 3)];
                    if (q < 0) continue;
                    const int r = in_row[which ? ops[q].second : ops[q].first];
                    const int a = r * 32 + ((lane & 7) ^ (r & 31));
                    bool seen = false;
                    int same_bank = 1;
                    for (int m = 0; m < n; ++m) {
                        if (addr[m] == a) seen = true;
                        else if (addr[m] % 16 == a % 16) ++same_bank;
                    }
                    if (seen) continue;   // identical addresses broadcast
                    addr[n++] = a;
                    if (same_bank > worst) worst = same_bank;
                }
                if (worst > 1) extra += worst - 1;
            }
    return extra;
}

// Local search (fixed seed: deterministic plans) over slot permutations and
// rows; the last step keeps rows 0..d_last-1.  Swing 8x8 from 92 extra read
// cycles per column group and tile (rows = slots = first appearance) to 0.
void lo_dag_place(const std::vector<std::vector<std::pair<int, int>>>& ops, std::vector<std::vector<int>>& slot,
                  std::vector<std::vector<int>>& row, int total) {
    const int K = (int)ops.size();
    std::vector<int> leaves(total);
    for (int r = 0; r < total; ++r) leaves[r] = r;
    auto cost = [&](int k) { return lo_dag_step_conflicts(ops[k], slot[k], k ? row[k - 1] : leaves); };
    std::vector<int> c(K);
    int sum = 0;
    for (int k = 0; k < K; ++k) sum += c[k] = cost(k);
    std::mt19937 rng(20261016u);
    for (int it = 0; it < 200000 && sum > 0; ++it) {
        const int k = (int)(rng() % K), n = (int)ops[k].size();
        if ((rng() & 1) || k == K - 1) {   // swap the slots of two nodes of step k
            if (n < 2) continue;
            const int a = (int)(rng() % n), b = (int)(rng() % n);
            if (a == b) continue;
            std::swap(slot[k][a], slot[k][b]);
            const int v = cost(k);
            if (v <= c[k]) sum += v - c[k], c[k] = v;
            else std::swap(slot[k][a], slot[k][b]);
        } else {   // move a node of step k to another row (swap with its holder)
            const int a = (int)(rng() % n), v = (int)(rng() % total), old = row[k][a];
            int other = -1;
            for (int q = 0; q < n; ++q)
                if (row[k][q] == v) other = q;
            row[k][a] = v;
            if (other >= 0) row[k][other] = old;
            const int nv = cost(k + 1);
            if (nv <= c[k + 1]) {
                sum += nv - c[k + 1], c[k + 1] = nv;
            } else {
                row[k][a] = old;
                if (other >= 0) row[k][other] = v;
            }
        }
    }
}

// Extra read cycles of a finished layout, recomputed from its bytes as the
// kernel reads them (the check behind allred_lo_dag's read_conflicts).
int lo_dag_conflicts(const std::vector<uint8_t>& dag, int steps, int total) {
    int extra = 0;
    std::vector<int> ident(total);
    for (int r = 0; r < total; ++r) ident[r] = r;
    for (int k = 0; k < steps; ++k) {
        std::vector<std::pair<int, int>> ops;
        std::vector<int> slot_of;
        for (int sl = 0; sl < 32; ++sl)
            if (dag[(size_t)k * 64 + 2 * sl] != 0xFF) {
                ops.emplace_back(dag[(size_t)k * 64 + 2 * sl], dag[(size_t)k * 64 + 2 * sl + 1]);
                slot_of.push_back(sl);
            }
        extra += lo_dag_step_conflicts(ops, slot_of, ident);
    }
    return extra;
}

// The device form of a DAG table: per lane group g, the 24 words
// a | b << 8 | out << 16 (-1: empty slot) of its slots g + 8i at steps k,
// word 4k + i, 96 contiguous bytes (six 16-byte loads per lane instead of 80
// byte loads: the byte-wise prologue cost 2.3 us per launch); then the final
// row of every rank at byte 768 + r.
constexpr size_t kDagLaneBytes = 768 + 64;
std::vector<uint8_t> lo_dag_lanes(const std::vector<uint8_t>& dag, int steps) {
    if (dag.empty()) return {};
    std::vector<uint8_t> out(kDagLaneBytes, 0);
    for (int g = 0; g < 8; ++g)
        for (int k = 0; k < ALLRED_MAX_STEPS; ++k)
            for (int i = 0; i < 4; ++i) {
                const int sl = 8 * i + g;
                int32_t w = -1;
                if (k < steps && dag[(size_t)k * 64 + 2 * sl] != 0xFF)
                    w = dag[(size_t)k * 64 + 2 * sl] | dag[(size_t)k * 64 + 2 * sl + 1] << 8 |
                        dag[456 + 32 * (size_t)k + sl] << 16;
                std::memcpy(&out[(size_t)g * 96 + (size_t)(4 * k + i) * 4], &w, 4);
            }
    std::memcpy(&out[768], &dag[384], 64);
    return out;
}

std::vector<uint8_t> lo_dag_build(const allred_schedule& s, int total) {
    if (total != 64) return {};
    std::vector<std::vector<std::pair<int, int>>> ops(s.steps);
    std::vector<int> cur(total), nxt(total);
    for (int r = 0; r < total; ++r) cur[r] = r;  // leaves: tile rows
    for (int k = 0; k < s.steps; ++k) {
        std::map<std::pair<int, int>, int> nodes;
        for (int r = 0; r < total; ++r) {
            const int a = cur[r], b = cur[s.partner[r][k]];
            const auto key = a < b ? std::make_pair(a, b) : std::make_pair(b, a);
            auto it = nodes.find(key);
            if (it == nodes.end()) {
                if (nodes.size() >= 32) return {};
                it = nodes.emplace(key, (int)nodes.size()).first;
                ops[k].push_back(key);
            }
            nxt[r] = it->second;
        }
        cur.swap(nxt);
    }
    std::vector<std::vector<int>> slot(s.steps), row(s.steps);
    for (int k = 0; k < s.steps; ++k)
        for (int q = 0; q < (int)ops[k].size(); ++q) slot[k].push_back(q), row[k].push_back(q);
    if (tune(Tune::lo_dag_place)) lo_dag_place(ops, slot, row, total);
    std::vector<uint8_t> dag(kDagBytes, 0);
    for (int k = 0; k < s.steps; ++k) {
        for (int sl = 0; sl < 32; ++sl) dag[(size_t)k * 64 + 2 * sl] = dag[(size_t)k * 64 + 2 * sl + 1] = 0xFF;
        for (int q = 0; q < (int)ops[k].size(); ++q) {
            const int sl = slot[k][q];
            dag[(size_t)k * 64 + 2 * sl] = (uint8_t)(k ? row[k - 1][ops[k][q].first] : ops[k][q].first);
            dag[(size_t)k * 64 + 2 * sl + 1] = (uint8_t)(k ? row[k - 1][ops[k][q].second] : ops[k][q].second);
            dag[456 + 32 * (size_t)k + sl] = (uint8_t)row[k][q];
        }
        dag[448 + k] = (uint8_t)ops[k].size();
    }
    for (int r = 0; r < total; ++r) dag[384 + r] = (uint8_t)(s.steps ? row[s.steps - 1][cur[r]] : r);
    return dag;
}

// The placed DAG of a schedule, cached per (algo, side, total, placement): the
// local search runs up to 200,000 iterations, so plans of the same schedule
// reuse its result.
std::vector<uint8_t> lo_dag(const allred_schedule& s, int total) {
    static std::mutex mu;
    static std::map<std::tuple<int, int, int, int64_t>, std::vector<uint8_t>> cache;
    const auto key = std::make_tuple(s.algo, s.side, total, tune(Tune::lo_dag_place));
    {
        std::lock_guard<std::mutex> g(mu);
        const auto it = cache.find(key);
        if (it != cache.end()) return it->second;
    }
    std::vector<uint8_t> dag = lo_dag_build(s, total);
    std::lock_guard<std::mutex> g(mu);
    return cache.emplace(key, std::move(dag)).first->second;
}

}  // namespace

extern "C" {

int allred_plan_create(const allred_plan_desc* desc, allred_plan** out) {
    if (!desc || !out) return ALLRED_ERR_ARG;
    *out = nullptr;
    const int side = desc->side_length;
    const int total = desc->total_nodes > 0 ? desc->total_nodes : side * side;
    if (desc->variant < ALLRED_BO || desc->variant > ALLRED_MEM) return ALLRED_ERR_ARG;
    if (desc->exec != ALLRED_EXEC_STEPS && desc->exec != ALLRED_EXEC_FUSED) return ALLRED_ERR_ARG;
    const size_t n = (size_t)desc->elems_per_rank;
    if (n == 0 || n % 8) return ALLRED_ERR_ARG;
    if (desc->variant != ALLRED_LO && n % (8 * (size_t)total)) return ALLRED_ERR_ARG;

    auto* p = new allred_plan();
    p->desc = *desc;
    p->total = total;
    p->n = n;
    p->block_elems = n / (size_t)total;
    int st = build_schedule(desc->algo, side, total, &p->sched, nullptr);
    if (st != ALLRED_OK) { free_plan(p); return st; }
    if (desc->device >= 0) {
        if (hipSetDevice(desc->device) != hipSuccess) { free_plan(p); return ALLRED_ERR_HIP; }
        p->device = desc->device;
    } else {
        (void)hipGetDevice(&p->device);
    }
    const int steps = p->sched.steps;
    std::vector<int16_t> partner((size_t)steps * total);
    std::vector<int16_t> rs, ag;
    for (int k = 0; k < steps; ++k) {
        p->blk_off.push_back(rs.size());
        p->blk_per_rank.push_back(popcount64(p->sched.recv[0][k]));
        for (int r = 0; r < total; ++r) {
            partner[(size_t)k * total + r] = (int16_t)p->sched.partner[r][k];
            for (int b = 0; b < total; ++b) {
                if ((p->sched.recv[r][k] >> b) & 1ull) rs.push_back((int16_t)b);
                if ((p->sched.send[r][k] >> b) & 1ull) ag.push_back((int16_t)b);
            }
        }
    }
    // rank-uniform LO = the BO tree pass; at 64 ranks below lo_tree_min_tiles tiles per rank
    // (32 kB) the register butterfly is faster (2 kB: 2.9 vs 3.5 us, profiles/r02_sweep.jsonl)
    p->lo_tree = desc->variant == ALLRED_LO && n % (8 * (size_t)total) == 0 && tune(Tune::lo_tree) &&
                 (total != 64 || n >= (uint64_t)tune(Tune::lo_tree_min_tiles) * 256) &&
                 lo_rank_uniform(p->sched, total);
    std::vector<uint8_t> order(&p->sched.tree_order[0][0],
                               &p->sched.tree_order[0][0] + ALLRED_MAX_NODES * ALLRED_MAX_NODES);
    // the DAG of distinct sums only where the fused LO runs the butterfly (not the tree route)
    if (desc->variant == ALLRED_LO && desc->exec == ALLRED_EXEC_FUSED && !p->lo_tree && tune(Tune::lo_dag)) {
        const std::vector<uint8_t> dag = lo_dag(p->sched, total);
        if ((st = upload(&p->d_dag, lo_dag_lanes(dag, p->sched.steps)))) {
            free_plan(p);
            return st;
        }
    }
    if ((st = upload(&p->d_partner, partner)) || (st = upload(&p->d_rs_blocks, rs)) ||
        (st = upload(&p->d_ag_blocks, ag)) || (st = upload(&p->d_order, order))) {
        free_plan(p);
        return st;
    }
    // schedule form: one persistent launch (default) or one launch per step (steps_form 1, A/B)
    p->steps_persistent = desc->exec == ALLRED_EXEC_STEPS && desc->variant != ALLRED_MEM && tune(Tune::steps_form) != 1;
    if (p->steps_persistent) {
        std::vector<uint8_t> tab;
        if (desc->variant == ALLRED_BO) {
            tab = bo_steps_table(p->sched, total);
            if (steps && tab.empty()) {
                free_plan(p);
                return ALLRED_ERR_SCHEDULE;
            }
        } else {
            tab = lo_steps_pairs(p->sched, total);
            if (steps && tab.empty()) {
                free_plan(p);
                return ALLRED_ERR_SCHEDULE;
            }
        }
        std::vector<uint8_t> pipe = desc->variant == ALLRED_BO ? bo_steps_pipe_table(tab, total, steps)
                                                               : lo_steps_pipe_table(p->sched, total);
        if (desc->variant == ALLRED_BO && !pipe.empty()) {   // + k_steps_reg's program (bo_steps_reg_table)
            const std::vector<uint8_t> reg = bo_steps_reg_table(pipe, p->sched, total);
            pipe.insert(pipe.end(), reg.begin(), reg.end());
            p->steps_reg_tab = !reg.empty();
        }
        if ((st = upload(&p->d_steps_tab, tab)) || (st = upload(&p->d_steps_pipe_tab, pipe))) {
            free_plan(p);
            return st;
        }
    }
    // workspace and launch count per execute
    if (desc->exec == ALLRED_EXEC_FUSED) {
        // 64 ranks from 1024 whole tiles: the persistent passes, in launches of
        // about fused_chunk_tiles tiles (allred_plan_launches recounts at call time)
        p->launches = (int)fused_launches(desc->variant, p->lo_tree, desc->algo, desc->side_length, n, total);
    } else if (p->steps_persistent) {
        p->launches = steps ? 1 : 0;
    } else if (desc->variant == ALLRED_BO) {
        p->launches = 2 * steps;
    } else if (desc->variant == ALLRED_LO) {
        p->ws_bytes = (size_t)total * n * 2;
        p->launches = steps + (steps % 2);
    } else {
        p->ws_bytes = n * 2;
        p->launches = 2;
    }
    *out = p;
    return ALLRED_OK;
}

uint64_t allred_preferred_rank_stride(uint64_t elems) { return (elems + 63) / 64 * 64 + 64; }

int allred_plan_destroy(allred_plan* plan) {
    free_plan(plan);
    return ALLRED_OK;
}

size_t allred_plan_workspace_bytes(const allred_plan* plan) { return plan ? plan->ws_bytes : 0; }

int allred_plan_launches(const allred_plan* plan) {
    if (!plan) return 0;
    // fused plans: what execute would enqueue now on device memory (the tune keys
    // it reads at launch time included); pinned host buckets take one launch
    if (plan->desc.exec == ALLRED_EXEC_FUSED)
        return (int)fused_launches(plan->desc.variant, plan->lo_tree, plan->desc.algo, plan->desc.side_length, plan->n,
                                   plan->total);
    return plan->launches;
}

int allred_lo_dag(int algo, int side_length, int total_nodes, uint8_t* out, size_t cap, int* read_conflicts) {
    if (!out && cap) return ALLRED_ERR_ARG;
    const int total = total_nodes > 0 ? total_nodes : side_length * side_length;
    allred_schedule s{};
    int st = build_schedule(algo, side_length, total, &s, nullptr);
    if (st) return st;
    const std::vector<uint8_t> dag = lo_dag(s, total);
    if (read_conflicts) *read_conflicts = dag.empty() ? 0 : lo_dag_conflicts(dag, s.steps, total);
    if (dag.empty()) return 0;
    if (cap < dag.size()) return ALLRED_ERR_ARG;
    std::memcpy(out, dag.data(), dag.size());
    return (int)dag.size();
}

int allred_steps_program(int algo, int variant, int side_length, int total_nodes, uint8_t* out, size_t cap) {
    if (!out && cap) return ALLRED_ERR_ARG;
    const bool reg = variant == (ALLRED_BO | ALLRED_STEPS_REG);
    if (variant != ALLRED_BO && variant != ALLRED_LO && !reg) return ALLRED_ERR_ARG;
    const int total = total_nodes > 0 ? total_nodes : side_length * side_length;
    allred_schedule s{};
    int st = build_schedule(algo, side_length, total, &s, nullptr);
    if (st) return st;
    std::vector<uint8_t> prog = variant == ALLRED_LO ? lo_steps_pipe_table(s, total)
                                                     : bo_steps_pipe_table(bo_steps_table(s, total), total, s.steps);
    if (reg) prog = bo_steps_reg_table(prog, s, total);
    if (prog.empty()) return 0;
    if (cap < prog.size()) return ALLRED_ERR_ARG;
    std::memcpy(out, prog.data(), prog.size());
    return (int)prog.size();
}

uint64_t allred_plan_stamp_words(const allred_plan* p) {
    if (!p || !p->steps_persistent || p->sched.steps == 0) return 0;
    const int S = p->sched.steps;
    if (p->desc.variant == ALLRED_BO) return bo_steps_units(p->block_elems, p->total) * (uint64_t)(2 * S + 1);
    return lo_steps_units(p->n) * (uint64_t)(S + 1);
}

int allred_plan_rank_zones(const allred_plan* p, const uint64_t* stamps, uint64_t* zone_start, uint64_t* zone_end) {
    if (!p || !stamps || !zone_start || !zone_end || allred_plan_stamp_words(p) == 0) return ALLRED_ERR_ARG;
    const int N = p->total, S = p->sched.steps;
    for (int r = 0; r < N; ++r) zone_start[r] = ~0ull, zone_end[r] = 0;
    if (p->desc.variant == ALLRED_BO) {
        // every rank's copy of every block is read at RS step 0 (holders add their
        // partners' copies) and written in the last phase (AG step 0 for the
        // receivers, the holders' results beside it): the zone opens at the
        // earliest unit start and closes at the latest unit end
        const uint64_t units = bo_steps_units(p->block_elems, N);
        for (uint64_t u = 0; u < units; ++u) {
            const uint64_t* st = stamps + u * (uint64_t)(2 * S + 1);
            for (int r = 0; r < N; ++r) {
                if (st[0] < zone_start[r]) zone_start[r] = st[0];
                if (st[2 * S] > zone_end[r]) zone_end[r] = st[2 * S];
            }
        }
    } else {
        const uint64_t units = lo_steps_units(p->n);
        for (uint64_t u = 0; u < units; ++u) {
            const uint64_t* st = stamps + u * (uint64_t)(S + 1);
            for (int r = 0; r < N; ++r) {
                if (st[0] < zone_start[r]) zone_start[r] = st[0];
                if (st[S] > zone_end[r]) zone_end[r] = st[S];
            }
        }
    }
    return ALLRED_OK;
}

int allred_plan_execute_profiled(allred_plan* p, uint16_t* ranks, uint64_t stride, void* workspace,
                                 uint64_t* stamps, void* stream) {
    if (!p || !ranks || stride < p->n) return ALLRED_ERR_ARG;
    if (p->ws_bytes && !workspace) return ALLRED_ERR_ARG;
    if (stamps && allred_plan_stamp_words(p) == 0) return ALLRED_ERR_UNSUPPORTED;
    DeviceGuard guard(p->desc.device);   // a plan made for device d launches on d, then restores the caller's
    if (!guard.ok) return ALLRED_ERR_HIP;
    const int N = p->total, steps = p->sched.steps;
    const bool acc16 = p->desc.mem_accum == ALLRED_ACC_BF16;
    int st = ALLRED_OK;
    if (p->desc.exec == ALLRED_EXEC_FUSED) {
        if (p->desc.variant == ALLRED_MEM) return launch_mem_fused(ranks, stride, p->n, N, acc16, stream);
        if (p->desc.variant == ALLRED_LO && !p->lo_tree) {
            // the build-time DAG in registers where one was generated for this schedule
            if (tune(Tune::lo_dag_reg) && p->n / 256 >= (uint64_t)tune(Tune::lo_dag_reg_min_tiles)) {
                st = launch_lo_dag_reg(ranks, stride, p->n, p->desc.algo, p->desc.side_length, N, stream);
                if (st != ALLRED_ERR_UNSUPPORTED) return st;
            }
            return launch_butterfly(ranks, stride, p->n, N, p->d_partner, steps, p->d_dag, stream);
        }
        int slot = -1;
        for (int i = 0; i < allred_plan::kPtrCache && slot < 0; ++i)
            if (p->ptr_seen[i] == ranks) slot = i;
        if (slot < 0) {   // pinned host buckets (zero-copy) take the pipelined form
            hipPointerAttribute_t at{};
            slot = p->ptr_next;
            p->ptr_next = (p->ptr_next + 1) % allred_plan::kPtrCache;
            p->ptr_host[slot] = hipPointerGetAttributes(&at, ranks) == hipSuccess && at.type == hipMemoryTypeHost;
            (void)hipGetLastError();
            p->ptr_seen[slot] = ranks;
        }
        return launch_tree_fused(ranks, stride, p->n, N, p->d_order, stream, p->ptr_host[slot]);
    }
    if (p->steps_persistent) {
        if (p->desc.variant == ALLRED_BO)
            return launch_bo_steps(ranks, stride, N, steps, p->d_steps_tab, p->d_steps_pipe_tab,
                                   p->steps_reg_tab ? p->d_steps_pipe_tab + (size_t)kBoPipeTabBytes * N : nullptr,
                                   p->block_elems,
                                   stamps, stream);
        return launch_lo_steps(ranks, stride, N, steps, p->d_steps_tab, p->d_steps_pipe_tab, p->n, stamps, stream);
    }
    if (p->desc.variant == ALLRED_BO) {
        for (int k = 0; k < steps && st == ALLRED_OK; ++k)
            st = launch_rs_step(ranks, stride, N, p->d_partner + (size_t)k * N, p->d_rs_blocks + p->blk_off[k],
                                p->blk_per_rank[k], p->block_elems, stream);
        for (int k = steps - 1; k >= 0 && st == ALLRED_OK; --k)
            st = launch_ag_step(ranks, stride, N, p->d_partner + (size_t)k * N, p->d_ag_blocks + p->blk_off[k],
                                p->blk_per_rank[k], p->block_elems, stream);
        return st;
    }
    if (p->desc.variant == ALLRED_LO) {
        uint16_t* ws = static_cast<uint16_t*>(workspace);
        for (int k = 0; k < steps && st == ALLRED_OK; ++k) {
            const bool to_ws = (k % 2) == 0;
            st = launch_lo_step(to_ws ? ranks : ws, to_ws ? stride : p->n, to_ws ? ws : ranks, to_ws ? p->n : stride,
                                N, p->d_partner + (size_t)k * N, p->n, stream);
        }
        if (st == ALLRED_OK && steps % 2) st = launch_copy_ranks(ws, p->n, ranks, stride, N, p->n, stream);
        return st;
    }
    uint16_t* dst = static_cast<uint16_t*>(workspace);
    st = launch_mem_reduce(ranks, stride, p->n, N, dst, acc16, stream);
    if (st == ALLRED_OK) st = launch_broadcast(ranks, stride, p->n, N, dst, stream);
    return st;
}

int allred_plan_execute(allred_plan* p, uint16_t* ranks, uint64_t stride, void* workspace, void* stream) {
    return allred_plan_execute_profiled(p, ranks, stride, workspace, nullptr, stream);
}

int allred_bf16_add(uint16_t* dst, const uint16_t* src, size_t n, void* stream) {
    return launch_bf16_add(dst, src, n, stream);
}

int allred_bf16_add_masked(uint16_t* dst, const uint16_t* src, uint64_t mask, size_t block_elems, void* stream) {
    uint64_t off[ALLRED_MAX_NODES], len[ALLRED_MAX_NODES];
    int ns = 0;
    for (int b = 0; b < 64;) {   // one segment per run of set bits
        if (!((mask >> b) & 1ull)) { ++b; continue; }
        int e = b;
        while (e < 64 && ((mask >> e) & 1ull)) ++e;
        off[ns] = (uint64_t)b * block_elems;
        len[ns++] = (uint64_t)(e - b) * block_elems;
        b = e;
    }
    return launch_bf16_add_segs(dst, src, off, len, ns, stream);
}

// ---------------------------------------------------------------------------
// argv parsing: AllredConfig::AllredConfig (allred_helper.cpp:205-220) and the
// mains (allred_BO_2D.cpp:22-24, allred_LO_2D.cpp:15, allred_mem_2D.cpp:11)
// ---------------------------------------------------------------------------
static int stoi_like(const char* s, int* out) {  // std::stoi: leading integer, else throw
    if (!s) return ALLRED_ERR_ARG;
    char* end = nullptr;
    errno = 0;
    const long v = std::strtol(s, &end, 10);
    if (end == s || errno == ERANGE || v > 2147483647L || v < -2147483647L - 1) return ALLRED_ERR_ARG;
    *out = (int)v;
    return ALLRED_OK;
}

int allred_args_parse(int argc, const char* const* argv, int variant, allred_args* a) {
    if (!a || argc < 0 || (argc > 0 && !argv)) return ALLRED_ERR_ARG;
    std::memset(a, 0, sizeof(*a));
    int v = 0;
    a->variant = variant;
    if (argc >= 2) { if (stoi_like(argv[1], &v)) return ALLRED_ERR_ARG; a->swing = v == 1; }
    if (argc >= 3) { if (stoi_like(argv[2], &v)) return ALLRED_ERR_ARG; a->run_kernel = v == 1; }
    a->side_length = 1;
    if (argc >= 4) { if (stoi_like(argv[3], &v)) return ALLRED_ERR_ARG; a->side_length = allred_highest_power_of_two(v); }
    if (argc >= 5) { if (stoi_like(argv[4], &v)) return ALLRED_ERR_ARG; a->seed = v; }
    a->tiles = 1;
    if (argc >= 6) { if (stoi_like(argv[5], &v)) return ALLRED_ERR_ARG; a->tiles = v < 1 ? 1 : v; }
    a->error = 1;
    if (argc >= 7) { if (stoi_like(argv[6], &v)) return ALLRED_ERR_ARG; a->error = v; }
    if (variant == ALLRED_BO) {
        if (argc >= 8) { if (stoi_like(argv[7], &v)) return ALLRED_ERR_ARG; a->print_core = v; }
        if (argc >= 9) { if (stoi_like(argv[8], &v)) return ALLRED_ERR_ARG; a->bandwidth_optimal = v != 0; }
    }
    // extension: rank count (argv[9] or ALLRED_NODES), 0 = side^2
    int total = 0;
    const char* env_nodes = std::getenv("ALLRED_NODES");
    if (argc >= 10) { if (stoi_like(argv[9], &total)) return ALLRED_ERR_ARG; }
    else if (env_nodes && stoi_like(env_nodes, &total)) return ALLRED_ERR_ARG;
    a->total_nodes = total > 0 ? total : a->side_length * a->side_length;
    // the one-pass form is the default (bit-identical); ALLRED_EXEC=steps keeps
    // the reference's step structure (every step's result in the buckets)
    a->exec = env_is("ALLRED_EXEC", "steps") ? ALLRED_EXEC_STEPS : ALLRED_EXEC_FUSED;
    a->round_mode = env_is("ALLRED_BF16_ROUND", "rne") ? 1 : 0;
    // the reference's AllredConfig is bound to the IDevice its main created
    // (allred_BO_2D.cpp:8); here ALLRED_DEVICE (or AllredConfig's device
    // argument) names the HIP device ordinal, -1 = the current device
    a->device = -1;
    const char* env_dev = std::getenv("ALLRED_DEVICE");
    if (env_dev && stoi_like(env_dev, &a->device)) return ALLRED_ERR_ARG;
    a->mem_accum = env_is("ALLRED_MEM_ACC", "bf16") ? ALLRED_ACC_BF16 : ALLRED_ACC_FP32;
    // extension: the ranks over G GPUs of this node (argv[10] or ALLRED_GPUS), 0 = one device
    const char* env_gpus = std::getenv("ALLRED_GPUS");
    if (argc >= 11) { if (stoi_like(argv[10], &a->gpus)) return ALLRED_ERR_ARG; }
    else if (env_gpus && stoi_like(env_gpus, &a->gpus)) return ALLRED_ERR_ARG;
    if (a->gpus < 0) a->gpus = 0;
    const bool large = variant == ALLRED_MEM || (variant == ALLRED_BO && a->bandwidth_optimal);
    a->num_tiles = allred_normalize_tiles(a->tiles, a->total_nodes, large ? 1 : 0);
    return ALLRED_OK;
}

// ---------------------------------------------------------------------------
// allred_run: AllredConfig ctor data setup (allred_helper.cpp:264-288) +
// RunProgram (allred_helper.hpp:84-96) on the HIP engine.
// ---------------------------------------------------------------------------
#define HIPCK(x)                                   \
    do {                                           \
        if ((x) != hipSuccess) { st = ALLRED_ERR_HIP; goto done; } \
    } while (0)
#define ST(x)                                      \
    do {                                           \
        st = (x);                                  \
        if (st != ALLRED_OK) goto done;            \
    } while (0)

}  // extern "C"

// tt-metal's profile_log_device.csv layout, as python/profiler_results_analyzer*.py
// read it (metadata line, column header, one row per zone event): every rank's
// ALL_RED_LOOP ZONE_START / ZONE_END (DeviceZoneScopedN, allred_BO_2D/kernels/
// dataflow_kernel.cpp:147).  Ranks sit on the Wormhole worker cores the
// reference's grid ran on (physical x / y of python/timing_taker.py:17-18);
// times in s_memrealtime ticks (100 MHz "cycles").
int tsa::write_profile_log(const char* path, int N, int side, const uint64_t* start, const uint64_t* end) {
    static const int phys_x[8] = {1, 2, 3, 4, 6, 7, 8, 9}, phys_y[8] = {1, 2, 3, 4, 5, 7, 8, 9};
    FILE* f = std::fopen(path, "w");
    if (!f) return ALLRED_ERR_ARG;
    std::fprintf(f, "ARCH: gfx950, CHIP_FREQ[MHz]: 100\n");
    std::fprintf(f, "PCIe slot, core_x, core_y, RISC processor type, timer_id, time[cycles since reset], stat value, "
                    "run ID, run host ID,  zone name, type, source line, source file\n");
    for (int r = 0; r < N; ++r) {
        const int x = r % side, y = r / side;
        const int cx = x < 8 ? phys_x[x] : x + 2, cy = y < 8 ? phys_y[y] : y + 2;
        for (int e = 0; e < 2; ++e)
            std::fprintf(f, "0,%d,%d,BRISC,%d,%llu,0,0,0,ALL_RED_LOOP,%s,0,kernels.hip\n", cx, cy, e,
                         (unsigned long long)(e ? end[r] : start[r]), e ? "ZONE_END" : "ZONE_START");
    }
    std::fclose(f);
    return ALLRED_OK;
}

extern "C" {

int allred_run(const allred_args* a, int verbose, allred_report* rep) {
    if (!a) return ALLRED_ERR_ARG;
    allred_report local_rep{};
    allred_report* R = rep ? rep : &local_rep;
    std::memset(R, 0, sizeof(*R));
    R->mismatches = -1;
    const int N = a->total_nodes;
    const size_t n = (size_t)a->num_tiles * 1024;  // bf16 per rank (2048-byte tiles)
    const size_t bytes = n * 2;
    const int variant = a->variant == ALLRED_MEM ? ALLRED_MEM
                        : (a->variant == ALLRED_BO && a->bandwidth_optimal) ? ALLRED_BO : ALLRED_LO;
    const int print_core = a->print_core;
    if (print_core < 0 || print_core >= N) return ALLRED_ERR_ARG;
    R->bytes_per_rank = bytes;
    R->total_nodes = N;
    if (a->gpus > 0) return run_multi_gpu(a, verbose, R);   // dist.cpp: one host thread per GPU
    DeviceGuard guard(a->device);
    if (!guard.ok) return ALLRED_ERR_HIP;

    allred_plan_desc d{};
    d.algo = a->swing ? ALLRED_SWING : ALLRED_RECDUB;
    d.variant = variant;
    d.exec = a->exec;
    d.side_length = a->side_length;
    d.total_nodes = N;
    d.device = a->device;
    d.elems_per_rank = n;
    d.mem_accum = a->mem_accum;
    allred_plan* plan = nullptr;
    int st = allred_plan_create(&d, &plan);
    if (st != ALLRED_OK) return st;
    R->launches = plan->launches;

    std::vector<uint32_t> src0(bytes / 4), src1(bytes / 4);
    uint16_t *h_in = nullptr, *h_out = nullptr, *d_ranks = nullptr, *d_scratch = nullptr, *d_stage = nullptr;
    uint64_t* d_stamps = nullptr;
    void* d_ws = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr, e3 = nullptr;
    hipStream_t s = nullptr;
    const size_t all_bytes = (size_t)N * bytes;
    const size_t stride = (size_t)allred_preferred_rank_stride(n);
    const size_t dev_bytes = (size_t)N * stride * 2;
    float ms = 0;
    // ALLRED_PROFILE_LOG=<path> (the reference's TT_METAL_DEVICE_PROFILER=1 +
    // profile_log_device.csv): per-rank ALL_RED_LOOP zones of the timed run
    const char* profile_log = std::getenv("ALLRED_PROFILE_LOG");
    const uint64_t stamp_words = profile_log ? allred_plan_stamp_words(plan) : 0;
    // end-to-end mode: "zerocopy" = the kernel reads / writes the pinned host
    // buckets in place (both PCIe directions at once; the default for the
    // fused BO pass, whose pipelined form is built for it), "dma" = one H2D
    // and one D2H around the device-resident allreduce.  ALLRED_E2E overrides.
    const char* e2e_mode = std::getenv("ALLRED_E2E");
    const bool zero_copy = e2e_mode ? std::strcmp(e2e_mode, "zerocopy") == 0
                                    : (variant == ALLRED_BO && a->exec == ALLRED_EXEC_FUSED && N >= 8);
    // "dma" over column chunks: the fused BO pass reduces every column with the same tree
    // (tree_order[0]), so a column chunk of every rank is an allreduce of its own —
    // H2D(c + 1) | pass(c) | D2H(c - 1) on three streams, each copy a 2D DMA straight into /
    // out of the skewed device layout (no staging pass); same bits as the whole-bucket pass.
    // ALLRED_E2E_CHUNKS=c equal chunks (1 = one copy each way around one pass); unset: 8, where the
    // box's strided copies keep the rate of plain ones (probed below: ALLRED_E2E_STRIDED_RATIO), else 1.
    // Each 2D copy costs ~10 us over its bytes (measured: 8 chunks 1.09 ms, 16 1.19, 32 1.5,
    // a 1-2-4-9-9-4-2-1 32nds ramp 1.18; profiles/r05_e2e_probe.json)
    std::vector<size_t> csz;
    const size_t col_unit = 8 * (size_t)N;
    {
        const char* c = std::getenv("ALLRED_E2E_CHUNKS");
        const size_t k = c ? (size_t)std::max(1, std::atoi(c)) : 8;
        if (n % k == 0 && (n / k) % col_unit == 0) csz.assign(k, n / k);
    }
    const int chunks = (int)csz.size();
    bool chunked = !zero_copy && chunks > 1 && variant == ALLRED_BO && a->exec == ALLRED_EXEC_FUSED &&
                         !profile_log;
    std::vector<std::pair<size_t, allred_plan*>> cplans;   // one plan per distinct chunk size
    auto chunk_plan = [&](size_t len) -> allred_plan* {
        for (auto& cp : cplans)
            if (cp.first == len) return cp.second;
        return nullptr;
    };
    hipStream_t sh = nullptr, sd = nullptr;
    hipEvent_t p[4] = {};   // the 2D / 1D copy-rate probe
    std::vector<hipEvent_t> cev;   // per chunk: H2D done, pass start, pass done
    if (a->seed < 0) {
        allred_constant_bf16_vector(bytes, 1.0f, src0.data());
        src1 = src0;
    } else {
        allred_random_bf16_vector(bytes, 100, a->seed, a->round_mode, src0.data());
        allred_random_bf16_vector(bytes, 100, a->seed + 1, a->round_mode, src1.data());
    }
    HIPCK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    HIPCK(hipHostMalloc((void**)&h_in, all_bytes, hipHostMallocDefault));
    HIPCK(hipHostMalloc((void**)&h_out, all_bytes, hipHostMallocDefault));
    // even x loads src_1, odd x loads src_0 (allred_BO_2D.cpp:79-85)
    for (int r = 0; r < N; ++r)
        std::memcpy(h_in + (size_t)r * n, ((r % a->side_length) % 2 == 0) ? src1.data() : src0.data(), bytes);
    HIPCK(hipMalloc((void**)&d_ranks, dev_bytes));
    HIPCK(hipMalloc((void**)&d_scratch, dev_bytes));
    HIPCK(hipMalloc((void**)&d_stage, all_bytes));
    if (plan->ws_bytes) HIPCK(hipMalloc(&d_ws, plan->ws_bytes));
    if (stamp_words) HIPCK(hipMalloc((void**)&d_stamps, stamp_words * 8));
    HIPCK(hipEventCreate(&e0));
    HIPCK(hipEventCreate(&e1));
    HIPCK(hipEventCreate(&e2));
    HIPCK(hipEventCreate(&e3));
    if (chunked) {
        for (size_t len : csz) {
            if (chunk_plan(len)) continue;
            allred_plan_desc cd = d;
            cd.elems_per_rank = len;
            allred_plan* cp = nullptr;
            ST(allred_plan_create(&cd, &cp));
            cplans.emplace_back(len, cp);
        }
        HIPCK(hipStreamCreateWithFlags(&sh, hipStreamNonBlocking));
        HIPCK(hipStreamCreateWithFlags(&sd, hipStreamNonBlocking));
        cev.assign(3 * (size_t)chunks, nullptr);
        for (auto& e : cev) HIPCK(hipEventCreate(&e));
    }
    // warm-up on a scratch copy (first-launch code-object load stays out of the timing)
    HIPCK(hipMemcpyAsync(d_stage, h_in, all_bytes, hipMemcpyHostToDevice, s));
    ST(launch_copy_ranks(d_stage, n, d_scratch, stride, N, n, s));
    if (a->run_kernel) ST(allred_plan_execute(plan, d_scratch, stride, d_ws, s));
    if (a->run_kernel)
        for (auto& cp : cplans) ST(allred_plan_execute(cp.second, d_scratch, stride, d_ws, s));
    HIPCK(hipStreamSynchronize(s));
    if (chunked && !std::getenv("ALLRED_E2E_CHUNKS")) {
        // (untimed) the chunks pay only where a strided (2D) copy keeps the rate of a plain one: on
        // some boxes a 2D device-to-host copy into the rank-major host buckets runs at ~23 GB/s
        // against ~52 for a 1D copy (8 chunks 2.1-2.2 ms there, one copy each way 1.55;
        // profiles/r05_e2e_probe.json) — then the buckets go as one copy each way.  Each copy
        // twice, the second timed (a first copy pays one-time costs)
        float t2d = 0, t1d = 0;
        for (auto& e : p) HIPCK(hipEventCreate(&e));
        const size_t cb = csz[0] * 2 * (size_t)N;
        HIPCK(hipMemcpy2DAsync(h_out, n * 2, d_scratch, stride * 2, csz[0] * 2, (size_t)N, hipMemcpyDeviceToHost, sd));
        HIPCK(hipEventRecord(p[0], sd));
        HIPCK(hipMemcpy2DAsync(h_out, n * 2, d_scratch, stride * 2, csz[0] * 2, (size_t)N, hipMemcpyDeviceToHost, sd));
        HIPCK(hipEventRecord(p[1], sd));
        HIPCK(hipMemcpyAsync(h_out, d_stage, cb, hipMemcpyDeviceToHost, sd));
        HIPCK(hipEventRecord(p[2], sd));
        HIPCK(hipMemcpyAsync(h_out, d_stage, cb, hipMemcpyDeviceToHost, sd));
        HIPCK(hipEventRecord(p[3], sd));
        HIPCK(hipStreamSynchronize(sd));
        HIPCK(hipEventElapsedTime(&t2d, p[0], p[1]));
        HIPCK(hipEventElapsedTime(&t1d, p[2], p[3]));
        // keep the chunks while the strided copy takes at most `ratio` x the plain one's time
        // (ALLRED_E2E_STRIDED_RATIO, default 1.5; 0 forces the one-copy form, a huge ratio the
        // chunks: tests/test_gpu_cli.py drives both outcomes of this decision)
        const char* rs = std::getenv("ALLRED_E2E_STRIDED_RATIO");
        const float ratio = rs ? std::strtof(rs, nullptr) : 1.5f;
        if (t2d > ratio * t1d) chunked = false;
    }
    if (chunked) {
        // timed: chunk c's H2D on sh, its pass on s behind it, its D2H on sd behind the
        // pass; the two PCIe directions and the passes overlap across chunks
        HIPCK(hipEventRecord(e0, sh));
        size_t off = 0;
        int launches = 0;
        for (int c = 0; c < chunks; off += csz[(size_t)c], ++c) {
            hipEvent_t h = cev[3 * (size_t)c], k0 = cev[3 * (size_t)c + 1], k1 = cev[3 * (size_t)c + 2];
            const size_t cs = csz[(size_t)c];
            allred_plan* cplan = chunk_plan(cs);
            launches += cplan->launches;
            HIPCK(hipMemcpy2DAsync(d_ranks + off, stride * 2, h_in + off, n * 2, cs * 2, (size_t)N,
                                   hipMemcpyHostToDevice, sh));
            HIPCK(hipEventRecord(h, sh));
            HIPCK(hipStreamWaitEvent(s, h, 0));
            HIPCK(hipEventRecord(k0, s));
            if (a->run_kernel) ST(allred_plan_execute(cplan, d_ranks + off, stride, d_ws, s));
            HIPCK(hipEventRecord(k1, s));
            HIPCK(hipStreamWaitEvent(sd, k1, 0));
            HIPCK(hipMemcpy2DAsync(h_out + off, n * 2, d_ranks + off, stride * 2, cs * 2, (size_t)N,
                                   hipMemcpyDeviceToHost, sd));
        }
        HIPCK(hipEventRecord(e3, sd));
        HIPCK(hipStreamSynchronize(sd));
        // device time: the passes themselves (each from its stream reaching it to its end)
        float dev_ms = 0;
        for (int c = 0; c < chunks; ++c) {
            float m = 0;
            HIPCK(hipEventElapsedTime(&m, cev[3 * (size_t)c + 1], cev[3 * (size_t)c + 2]));
            dev_ms += m;
        }
        R->device_seconds = dev_ms * 1e-3;
        HIPCK(hipEventElapsedTime(&ms, e0, e3));
        R->e2e_seconds = ms * 1e-3;
        R->launches = launches;
    } else if (zero_copy) {
        // the kernels read and write the pinned host buckets in place over PCIe
        // (both directions at once); no staging copies, no HBM round trip
        uint16_t* h_dev = nullptr;
        HIPCK(hipHostGetDevicePointer((void**)&h_dev, h_in, 0));
        HIPCK(hipEventRecord(e0, s));
        HIPCK(hipEventRecord(e1, s));
        if (a->run_kernel) ST(allred_plan_execute_profiled(plan, h_dev, n, d_ws, d_stamps, s));
        HIPCK(hipEventRecord(e2, s));
        HIPCK(hipEventRecord(e3, s));
        HIPCK(hipStreamSynchronize(s));
        std::memcpy(h_out, h_in, all_bytes);  // (untimed) the result, for validation below
    } else {
        // timed: H2D | allreduce | D2H.  The 64 host buckets are contiguous: one
        // DMA each way (per-bucket copies pay ~70 us each), then one HBM pass
        // into / out of the skewed device layout
        HIPCK(hipEventRecord(e0, s));
        HIPCK(hipMemcpyAsync(d_stage, h_in, all_bytes, hipMemcpyHostToDevice, s));
        ST(launch_copy_ranks(d_stage, n, d_ranks, stride, N, n, s));
        HIPCK(hipEventRecord(e1, s));
        if (a->run_kernel) ST(allred_plan_execute_profiled(plan, d_ranks, stride, d_ws, d_stamps, s));
        HIPCK(hipEventRecord(e2, s));
        ST(launch_copy_ranks(d_ranks, stride, d_stage, n, N, n, s));
        HIPCK(hipMemcpyAsync(h_out, d_stage, all_bytes, hipMemcpyDeviceToHost, s));
        HIPCK(hipEventRecord(e3, s));
        HIPCK(hipStreamSynchronize(s));
    }
    if (!chunked) {
        HIPCK(hipEventElapsedTime(&ms, e1, e2));
        R->device_seconds = ms * 1e-3;
        HIPCK(hipEventElapsedTime(&ms, e0, e3));
        R->e2e_seconds = ms * 1e-3;
    }
    if (profile_log) {
        std::vector<uint64_t> zs(N, 0), ze(N, (uint64_t)(R->device_seconds * 1e8));
        if (stamp_words && a->run_kernel) {   // the schedule form's per-unit stamps -> per-rank zones
            std::vector<uint64_t> host(stamp_words);
            HIPCK(hipMemcpy(host.data(), d_stamps, stamp_words * 8, hipMemcpyDeviceToHost));
            ST(allred_plan_rank_zones(plan, host.data(), zs.data(), ze.data()));
        }   // else: one device interval (hipEvents) for every rank, ticks from 0
        ST(write_profile_log(profile_log, N, a->side_length, zs.data(), ze.data()));
    }
    {
        float maxe = 0;
        const uint32_t* res = reinterpret_cast<const uint32_t*>(h_out + (size_t)print_core * n);
        R->mismatches = allred_validate_result_vector(res, src0.data(), src1.data(), bytes / 4, (float)a->error,
                                                      (uint32_t)N, verbose, &maxe);
        R->max_error = maxe;
        if (std::getenv("ALLRED_CHECK_ALL")) {  // extension: the reference checks one core only
            for (int r = 0; r < N; ++r) {
                if (r == print_core) continue;
                R->mismatches += allred_validate_result_vector(
                    reinterpret_cast<const uint32_t*>(h_out + (size_t)r * n), src0.data(), src1.data(), bytes / 4,
                    (float)a->error, (uint32_t)N, 0, nullptr);
            }
        }
    }
done:
    if (sh) (void)hipStreamSynchronize(sh);
    if (sd) (void)hipStreamSynchronize(sd);
    for (hipEvent_t e : cev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : p)
        if (e) (void)hipEventDestroy(e);
    if (sh) (void)hipStreamDestroy(sh);
    if (sd) (void)hipStreamDestroy(sd);
    for (auto& cp : cplans) allred_plan_destroy(cp.second);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (e2) (void)hipEventDestroy(e2);
    if (e3) (void)hipEventDestroy(e3);
    if (d_ws) (void)hipFree(d_ws);
    if (d_stamps) (void)hipFree(d_stamps);
    if (d_ranks) (void)hipFree(d_ranks);
    if (d_scratch) (void)hipFree(d_scratch);
    if (d_stage) (void)hipFree(d_stage);
    if (h_in) (void)hipHostFree(h_in);
    if (h_out) (void)hipHostFree(h_out);
    if (s) (void)hipStreamDestroy(s);
    allred_plan_destroy(plan);
    return st;
}

}  // extern "C"

namespace tsa {
namespace {
struct LaunchNote {
    const void* func = nullptr;
    const char* name = "";
    unsigned grid = 0, block = 0;
    int device = -1;
};
thread_local LaunchNote g_last_launch;
}  // namespace

void note_launch(const void* func, const char* name, unsigned grid, unsigned block) {
    LaunchNote& l = g_last_launch;
    l.func = func;
    l.name = name;
    l.grid = grid;
    l.block = block;
    (void)hipGetDevice(&l.device);
}
}  // namespace tsa

extern "C" int allred_last_launch(allred_launch_info* out) {
    if (!out) return ALLRED_ERR_ARG;
    std::memset(out, 0, sizeof(*out));
    const tsa::LaunchNote& l = tsa::g_last_launch;
    if (!l.func) return ALLRED_ERR_ARG;   // no recorded launch on this thread
    std::snprintf(out->kernel, sizeof(out->kernel), "%s", l.name);
    out->grid = l.grid;
    out->block = l.block;
    out->device = l.device;
    // the attributes below are queried now, not at launch (the launch path stays cheap)
    DeviceGuard guard(l.device);
    if (!guard.ok) return ALLRED_ERR_HIP;
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, l.func) != hipSuccess) return ALLRED_ERR_HIP;
    out->lds_bytes = (uint32_t)fa.sharedSizeBytes;
    out->regs = fa.numRegs;
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, l.func, (int)l.block, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, l.device) != hipSuccess)
        return ALLRED_ERR_HIP;
    out->resident_per_cu = per_cu;
    out->cus = cus;
    return ALLRED_OK;
}
