// TEST INFRASTRUCTURE ONLY — never linked into the product.
//
// Driver around the reference's own schedule functions, compiled from the
// reference sources where they lie (see oracle/Makefile target `ref`):
//   /root/reference/allred_helper/allred_helper.cpp:122-191
//       highest_power_of_two, get_step_directions,
//       get_comm_partner_recdub_2D, get_comm_partner_swing_2D
//   /root/reference/allred_BO_2D/allred_BO_2D.cpp:217-270
//       get_swing_block_comm_indexes, get_recdub_block_comm_indexes
//   /root/reference/scratch_work/all_red_swing_1D/all_red_swing_1D.cpp:32-36
//       get_comm_partner (the 1D Swing partner of the 8-core prototype)
// Those line ranges need only <cmath>/<cstdint>; nothing of tt-metal is
// stubbed.  This file restates the per-core schedule loop of
// allred_BO_2D.cpp:75-202 (which lives inside the tt-metal `main` and cannot
// be compiled here) around those functions and prints, per (algo, side,
// total_nodes) grid, every rank's partners, send/recv block masks and
// direction bits as JSON.  Output feeds tests/golden/schedule_ref.json.
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>

// prototypes exactly as allred_helper.hpp:24-30 and allred_BO_2D.cpp:4-5; the
// definitions are the reference's own, compiled by the Makefile into _ref/ref_sched.o
#include "ref_protos.h"

static void emit(bool swing, int side, int total, bool last) {
    int steps = (int)std::log2((double)total);
    std::printf("  {\"algo\": \"%s\", \"side\": %d, \"total\": %d, \"steps\": %d, \"ranks\": [\n",
                swing ? "swing" : "recdub", side, total, steps);
    uint32_t step_directions = 0, dummy = 0;
    for (int core_i = 0; core_i < total; ++core_i) {
        std::vector<int> partners(steps);
        std::vector<uint32_t> send(2 * steps, 0), recv(2 * steps, 0);
        bool horizontal = true;
        if (!swing) {
            int depth = 1;
            for (int s = 0; s < steps; ++s) {
                int p = get_comm_partner_recdub_2D(core_i, s, horizontal, depth, step_directions, side);
                partners[s] = p;
                uint32_t* bs = &send[2 * s];
                uint32_t* br = &recv[2 * s];
                if (p < 32) bs[0] |= (1u << p); else bs[1] |= (1u << (p - 32));
                if (core_i < 32) br[0] |= (1u << core_i); else br[1] |= (1u << (core_i - 32));
                depth = horizontal ? depth : 2 * depth;
                horizontal = !horizontal;
                get_recdub_block_comm_indexes(p, s + 1, bs, horizontal, side, total, depth, dummy);
                get_recdub_block_comm_indexes(core_i, s + 1, br, horizontal, side, total, depth, dummy);
            }
        } else {
            for (int s = 0; s < steps; ++s) {
                int p = get_comm_partner_swing_2D(core_i, s, horizontal, side, total);
                partners[s] = p;
                uint32_t* bs = &send[2 * s];
                uint32_t* br = &recv[2 * s];
                if (p < 32) bs[0] |= (1u << p); else bs[1] |= (1u << (p - 32));
                if (core_i < 32) br[0] |= (1u << core_i); else br[1] |= (1u << (core_i - 32));
                horizontal = !horizontal;
                get_swing_block_comm_indexes(p, s + 1, bs, horizontal, side, total);
                get_swing_block_comm_indexes(core_i, s + 1, br, horizontal, side, total);
            }
            step_directions = get_step_directions(core_i % side, core_i / side);
        }
        std::printf("    {\"rank\": %d, \"partners\": [", core_i);
        for (int s = 0; s < steps; ++s) std::printf("%s%d", s ? ", " : "", partners[s]);
        std::printf("], \"send\": [");
        for (int s = 0; s < steps; ++s)
            std::printf("%s%llu", s ? ", " : "",
                        (unsigned long long)send[2 * s] | ((unsigned long long)send[2 * s + 1] << 32));
        std::printf("], \"recv\": [");
        for (int s = 0; s < steps; ++s)
            std::printf("%s%llu", s ? ", " : "",
                        (unsigned long long)recv[2 * s] | ((unsigned long long)recv[2 * s + 1] << 32));
        std::printf("], \"dirs\": %u}%s\n", step_directions & ((1u << steps) - 1u),
                    core_i + 1 < total ? "," : "");
    }
    std::printf("  ]}%s\n", last ? "" : ",");
}

int main() {
    // grids: the reference's square S x S (S = 1,2,4,8) and the rectangular
    // (S, N) mappings used for 2/4/8 GPUs; (8,16) is the known
    // invalid rectangle (out-of-range RecDub partners) kept as a negative case.
    struct G { int side, total; };
    const G grids[] = {{1, 1}, {2, 2}, {2, 4}, {4, 8}, {4, 16}, {8, 64}, {8, 16}};
    const int ng = sizeof(grids) / sizeof(grids[0]);
    std::printf("{\"highest_power_of_two\": [");
    for (int v = -2; v <= 20; ++v) std::printf("%s[%d, %d]", v > -2 ? ", " : "", v, highest_power_of_two(v));
    std::printf("],\n \"step_directions\": [");
    for (int y = 0; y < 8; ++y)
        for (int x = 0; x < 8; ++x)
            std::printf("%s[%d, %d, %u]", (x || y) ? ", " : "", x, y, get_step_directions(x, y));
    std::printf("],\n \"swing_1d\": [");
    for (int nn = 2; nn <= 64; nn *= 2) {
        int st = (int)std::log2((double)nn);
        std::printf("%s{\"total\": %d, \"partners\": [", nn > 2 ? ", " : "", nn);
        for (int node = 0; node < nn; ++node) {
            std::printf("%s[", node ? ", " : "");
            for (int k = 0; k < st; ++k) std::printf("%s%d", k ? ", " : "", ref1d::get_comm_partner(node, k, nn));
            std::printf("]");
        }
        std::printf("]}");
    }
    std::printf("],\n \"grids\": [\n");
    for (int g = 0; g < ng; ++g) {
        emit(true, grids[g].side, grids[g].total, false);
        emit(false, grids[g].side, grids[g].total, g + 1 == ng);
    }
    std::printf("]}\n");
    return 0;
}
