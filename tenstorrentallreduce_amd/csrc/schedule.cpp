// schedule.cpp — the 2D Swing / Recursive-Doubling schedules (host C++).
//
// Replaces, with the same arguments and results:
//   highest_power_of_two         allred_helper.cpp:122-133
//   get_step_directions          allred_helper.cpp:136-142
//   get_comm_partner_recdub_2D   allred_helper.cpp:145-163
//   get_comm_partner_swing_2D    allred_helper.cpp:166-191
//   get_swing_block_comm_indexes allred_BO_2D.cpp:220-237
//   get_recdub_block_comm_indexes allred_BO_2D.cpp:242-270
//   the per-core schedule loop   allred_BO_2D.cpp:75-212
//   NUM_TILES normalisation      allred_helper.cpp:224-234
// Checked against the reference's own functions by tests/golden/schedule_ref.json.
#include <string>

#include "internal.hpp"

namespace tsa {

int steps_for(int total) {
    int s = 0;
    while ((1 << s) < total) ++s;
    return s;
}

namespace {

// Swing hop length for pair-step k: the Jacobsthal-like sequence
// 1, -1, 3, -5, 11, -21 = (1 - (-2)^(k+1)) / 3 (allred_helper.cpp:172).
int swing_distance(int k) {
    int pw = 1;  // (-2)^(k+1)
    for (int i = 0; i <= k; ++i) pw *= -2;
    return (1 - pw) / 3;
}

inline void set_bit(uint32_t* blocks, int idx) {
    if (idx < 0 || idx >= 64) return;  // out-of-grid peer: the schedule check rejects it
    if (idx < 32)
        blocks[0] |= 1u << idx;
    else
        blocks[1] |= 1u << (idx - 32);
}

}  // namespace
}  // namespace tsa

using namespace tsa;

extern "C" {

int allred_abi_version(void) { return ALLRED_ABI_VERSION; }

const char* allred_status_string(int st) {
    switch (st) {
        case ALLRED_OK: return "ok";
        case ALLRED_ERR_ARG: return "invalid argument";
        case ALLRED_ERR_SCHEDULE: return "grid is not a valid allreduce schedule";
        case ALLRED_ERR_HIP: return "HIP runtime error";
        case ALLRED_ERR_RCCL: return "RCCL error";
        case ALLRED_ERR_NOMEM: return "out of memory";
        case ALLRED_ERR_UNSUPPORTED: return "unsupported configuration";
        case ALLRED_ERR_TRANSPORT: return "exchange callback failed";
        default: return "unknown status";
    }
}

int allred_highest_power_of_two(int value) {
    int p = 8;
    while (p > 1 && value < p) p >>= 1;
    return p;
}

uint32_t allred_get_step_directions(int node_x, int node_y) {
    // one 6-step pattern per (x, y) parity class; bit i = "the SE RISC sends at step i"
    const bool xo = (node_x % 2) != 0, yo = (node_y % 2) != 0;
    if (!xo) return yo ? 0x19u : 0x33u;
    return yo ? 0x0cu : 0x26u;
}

int allred_get_comm_partner_recdub_2d(int node, int recdub_step, int horizontal_step,
                                      int message_pass_depth, uint32_t* step_directions,
                                      int side_length) {
    const int along = horizontal_step ? node % side_length : node / side_length;
    const int across = horizontal_step ? node / side_length : node % side_length;
    const bool lower_half = (along % (2 * message_pass_depth)) < message_pass_depth;
    if (step_directions) {
        const uint32_t bit = 1u << recdub_step;
        *step_directions = lower_half ? (*step_directions | bit) : (*step_directions & ~bit);
    }
    const int other = lower_half ? along + message_pass_depth : along - message_pass_depth;
    return horizontal_step ? across * side_length + other : other * side_length + across;
}

int allred_get_comm_partner_swing_2d(int node, int step, int horizontal_step, int side_length,
                                     int total_nodes) {
    const int row = node / side_length;
    const int d = swing_distance(step / 2);
    if (horizontal_step) {
        int p = (node % 2 == 0) ? node + d : node - d;
        // stay inside this row: wrap by one row length (also catches p < 0)
        if (p < 0 || p / side_length < row)
            p += side_length;
        else if (p / side_length > row)
            p -= side_length;
        return p;
    }
    int p = (row % 2 == 0) ? node + side_length * d : node - side_length * d;
    if (p < 0)
        p += total_nodes;
    else if (p >= total_nodes)
        p -= total_nodes;
    return p;
}

void allred_get_swing_block_comm_indexes(int node, int step, uint32_t* blocks, int horizontal_step,
                                         int side_length, int total_nodes) {
    const int steps = steps_for(total_nodes);
    bool h = horizontal_step != 0;
    for (int s = step; s < steps; ++s) {
        const int peer = allred_get_comm_partner_swing_2d(node, s, h, side_length, total_nodes);
        set_bit(blocks, peer);
        h = !h;
        allred_get_swing_block_comm_indexes(peer, s + 1, blocks, h, side_length, total_nodes);
    }
}

void allred_get_recdub_block_comm_indexes(int node, int step, uint32_t* blocks, int horizontal_step,
                                          int side_length, int total_nodes, int message_pass_depth,
                                          uint32_t* step_directions) {
    const int steps = steps_for(total_nodes);
    bool h = horizontal_step != 0;
    int depth = message_pass_depth;
    for (int s = step; s < steps; ++s) {
        const int peer =
            allred_get_comm_partner_recdub_2d(node, s, h, depth, step_directions, side_length);
        set_bit(blocks, peer);
        if (!h) depth *= 2;
        h = !h;
        allred_get_recdub_block_comm_indexes(peer, s + 1, blocks, h, side_length, total_nodes, depth,
                                             step_directions);
    }
}

int allred_normalize_tiles(int tiles, int total_nodes, int large_buffer) {
    const int t = tiles < 1 ? 1 : tiles;
    if (large_buffer) return t * total_nodes;        // BO / mem: tiles per block * nodes
    if (t >= 64) return (t + 63) / 64 * 64;          // LO: multiple of 64 tiles
    int p = 1;                                       // LO small: next power of two
    while (p < t) p *= 2;
    return p;
}

int allred_get_comm_partner_swing_1d(int node, int step, int num_nodes) {
    const int d = swing_distance(step);
    const int p = (node % 2 == 0) ? node + d : node - d;
    return ((p % num_nodes) + num_nodes) % num_nodes;
}

int allred_get_comm_partner_recdub_1d(int node, int step, uint32_t* step_directions) {
    const int depth = 1 << step;
    const bool lower_half = (node % (2 * depth)) < depth;
    if (step_directions)
        *step_directions = lower_half ? (*step_directions | (1u << step)) : (*step_directions & ~(1u << step));
    return lower_half ? node + depth : node - depth;
}

int allred_schedule_build(int algo, int side_length, int total_nodes, allred_schedule* out) {
    return build_schedule(algo, side_length, total_nodes, out, nullptr);
}

}  // extern "C"

namespace tsa {

int build_schedule(int algo, int side, int total, allred_schedule* out, std::string* why) {
    // (side is adjusted for the 1D algorithms)
    auto fail = [&](const std::string& m) {
        if (why) *why = m;
        return ALLRED_ERR_SCHEDULE;
    };
    if (!out) return ALLRED_ERR_ARG;
    std::memset(out, 0, sizeof(*out));
    const bool one_d = algo == ALLRED_RECDUB_1D || algo == ALLRED_SWING_1D;
    if (algo < ALLRED_RECDUB || algo > ALLRED_SWING_1D) return fail("unknown algorithm");
    if (one_d) side = total;
    if (side < 1 || (!one_d && (side > 8 || (side & (side - 1)))) || total < 1 || total > ALLRED_MAX_NODES ||
        (total & (total - 1)) || total % side)
        return fail("grid must be side in {1,2,4,8}, total a power of two <= 64 and a multiple of side");
    const int steps = steps_for(total);
    out->algo = algo;
    out->side = side;
    out->total = total;
    out->steps = steps;

    // per-core loop of allred_BO_2D.cpp:95-198 (2D) / the 1D prototypes' partner loops
    uint32_t step_directions = 0, dummy = 0;
    for (int r = 0; r < total; ++r) {
        bool h = true;
        int depth = 1;
        for (int k = 0; k < steps; ++k) {
            uint32_t snd[2] = {0, 0}, rcv[2] = {0, 0};
            int p;
            if (algo == ALLRED_SWING) {
                p = allred_get_comm_partner_swing_2d(r, k, h, side, total);
            } else if (algo == ALLRED_RECDUB) {
                p = allred_get_comm_partner_recdub_2d(r, k, h, depth, &step_directions, side);
            } else if (algo == ALLRED_SWING_1D) {
                p = allred_get_comm_partner_swing_1d(r, k, total);
            } else {
                p = allred_get_comm_partner_recdub_1d(r, k, &step_directions);
            }
            if (p < 0 || p >= total)
                return fail("rank " + std::to_string(r) + " step " + std::to_string(k) +
                            ": partner " + std::to_string(p) + " outside the grid");
            out->partner[r][k] = p;
            if (one_d) continue;  // masks below, from the full partner table
            set_bit(snd, p);
            set_bit(rcv, r);
            if (algo == ALLRED_SWING) {
                h = !h;
                allred_get_swing_block_comm_indexes(p, k + 1, snd, h, side, total);
                allred_get_swing_block_comm_indexes(r, k + 1, rcv, h, side, total);
            } else {
                if (!h) depth *= 2;
                h = !h;
                allred_get_recdub_block_comm_indexes(p, k + 1, snd, h, side, total, depth, &dummy);
                allred_get_recdub_block_comm_indexes(r, k + 1, rcv, h, side, total, depth, &dummy);
            }
            out->send[r][k] = (uint64_t)snd[0] | ((uint64_t)snd[1] << 32);
            out->recv[r][k] = (uint64_t)rcv[0] | ((uint64_t)rcv[1] << 32);
        }
        const uint32_t keep = steps >= 32 ? ~0u : ((1u << steps) - 1u);
        out->dirs[r] = (algo == ALLRED_SWING ? allred_get_step_directions(r % side, r / side)
                        : algo == ALLRED_SWING_1D ? 0u : step_directions) & keep;
    }
    if (one_d) {
        // the 2D recursion's rule on the 1D partner table: a rank's step-k
        // blocks are every rank reachable from it at steps > k
        auto reach = [&](int node, int from) {
            uint64_t set = 1ull << node;
            for (int k2 = from; k2 < steps; ++k2) {
                uint64_t add = 0;
                for (int v = 0; v < total; ++v)
                    if ((set >> v) & 1ull) add |= 1ull << out->partner[v][k2];
                set |= add;
            }
            return set;
        };
        for (int r = 0; r < total; ++r)
            for (int k = 0; k < steps; ++k) {
                out->send[r][k] = reach(out->partner[r][k], k + 1);
                out->recv[r][k] = reach(r, k + 1);
            }
    }

    // ---- validation: the schedule must be an allreduce ----
    const uint64_t all = total == 64 ? ~0ull : ((1ull << total) - 1ull);
    for (int r = 0; r < total; ++r) {
        uint64_t have = all;  // blocks r is still responsible for
        for (int k = 0; k < steps; ++k) {
            const int p = out->partner[r][k];
            if (out->partner[p][k] != r) return fail("partners are not symmetric");
            if (out->send[r][k] != out->recv[p][k]) return fail("send mask != partner's recv mask");
            if (out->recv[r][k] & out->recv[p][k]) return fail("recv masks of a pair overlap");
            if ((out->recv[r][k] | out->recv[p][k]) != have)
                return fail("a pair's recv masks do not split their common blocks");
            have = out->recv[r][k];
        }
        if (steps > 0 && out->recv[r][steps - 1] != (1ull << r))
            return fail("reduce-scatter does not leave block r at rank r");
    }
    // per-rank reduction trees: leaves(x, k) = leaves(x, k-1) ++ leaves(p_{k-1}(x), k-1);
    // a valid allreduce needs every tree to be a permutation of all ranks
    // (contributor sets of a merging pair are disjoint)
    struct Leaves {
        const allred_schedule* s;
        std::vector<int>* out;
        void operator()(int r, int k) const {
            if (k == 0) { out->push_back(r); return; }
            (*this)(r, k - 1);
            (*this)(s->partner[r][k - 1], k - 1);
        }
    };
    for (int x = 0; x < total; ++x) {
        std::vector<int> order;
        Leaves{out, &order}(x, steps);
        uint64_t seen = 0;
        for (int v : order) {
            if ((seen >> v) & 1ull) return fail("rank " + std::to_string(x) + " would add a contribution twice");
            seen |= 1ull << v;
        }
        if (seen != all) return fail("rank " + std::to_string(x) + " does not reach every rank");
        for (int i = 0; i < total; ++i) out->tree_order[x][i] = (uint8_t)order[i];
    }
    return ALLRED_OK;
}

}  // namespace tsa
