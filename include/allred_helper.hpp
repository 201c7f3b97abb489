// allred_helper.hpp — source-compatible replacement for the reference's
// allred_helper/allred_helper.hpp (EngineerCharlie/TenstorrentAllreduce).
//
// The pure functions keep the reference signatures exactly
// (allred_helper.hpp:15-30, allred_BO_2D.cpp:4-5) so result checks and
// schedule code written against the reference compile unchanged.  The
// tt-metal-typed parts (CreateComputeKernel / CreateDataflowKernel, the
// IDevice / CommandQueue / Program ctor of AllredConfig) have no MI355X
// meaning: AllredConfig takes (argc, argv, variant, device ordinal) — the
// variant stands for the calling main (allred_BO_2D / _LO_2D / _mem_2D, whose
// large_buffer flag it implies), the ordinal for the IDevice* — and
// RunProgram() runs the HIP engine on that device (see include/allred.h).
// Everything is a thin inline layer over liballred.so's C-ABI.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

#include "allred.h"

// allred_helper.cpp:18-120
inline void validate_result_vector(const std::vector<uint32_t>& result_vec,
                                   const std::vector<uint32_t>& src_vec_0,
                                   const std::vector<uint32_t>& src_vec_1, std::size_t num_els,
                                   float ERROR, uint32_t total_nodes) {
    allred_validate_result_vector(result_vec.data(), src_vec_0.data(), src_vec_1.data(), num_els,
                                  ERROR, total_nodes, 1, nullptr);
}

// allred_helper.cpp:122-133
inline int highest_power_of_two(int value) { return allred_highest_power_of_two(value); }

// allred_helper.cpp:136-142
inline uint32_t get_step_directions(int node_x, int node_y) {
    return allred_get_step_directions(node_x, node_y);
}

// allred_helper.cpp:145-163
inline int get_comm_partner_recdub_2D(int node, int recdub_step, bool horizontal_step,
                                      int message_pass_depth, uint32_t& step_directions,
                                      int SIDE_LENGTH) {
    return allred_get_comm_partner_recdub_2d(node, recdub_step, horizontal_step ? 1 : 0,
                                             message_pass_depth, &step_directions, SIDE_LENGTH);
}

// allred_helper.cpp:166-191
inline int get_comm_partner_swing_2D(int node, int step, bool horizontal_step, int SIDE_LENGTH,
                                     int TOTAL_NODES) {
    return allred_get_comm_partner_swing_2d(node, step, horizontal_step ? 1 : 0, SIDE_LENGTH,
                                            TOTAL_NODES);
}

// allred_BO_2D.cpp:220-237
inline void get_swing_block_comm_indexes(int node, int step, uint32_t* blocks, bool horizontal_step,
                                         int SIDE_LENGTH, int TOTAL_NODES) {
    allred_get_swing_block_comm_indexes(node, step, blocks, horizontal_step ? 1 : 0, SIDE_LENGTH,
                                        TOTAL_NODES);
}

// allred_BO_2D.cpp:242-270
inline void get_recdub_block_comm_indexes(int node, int step, uint32_t* blocks, bool horizontal_step,
                                          int SIDE_LENGTH, int TOTAL_NODES, int message_pass_depth,
                                          uint32_t& step_directions) {
    allred_get_recdub_block_comm_indexes(node, step, blocks, horizontal_step ? 1 : 0, SIDE_LENGTH,
                                         TOTAL_NODES, message_pass_depth, &step_directions);
}

// allred_helper.hpp:47-97.  Public members keep the reference names.
class AllredConfig {
public:
    bool SWING_VERSION = false;
    bool RUN_KERNEL = false;
    int RND_SRC = 0;
    int NUM_TILES = 1;
    int TOTAL_NUM_TILES = 0;
    int ERROR = 1;
    int num_els = 0;
    uint32_t TOTAL_NODES = 1;
    uint32_t SWING_ALGO_STEPS = 0;
    uint32_t single_tile_size = 2048;
    std::vector<uint32_t> src_vec_0, src_vec_1, result_vec;
    allred_args args{};
    allred_report report{};
    int status = ALLRED_OK;

    // allred_helper.cpp:194-289 (argv parsing, NUM_TILES normalisation, inputs).
    // `variant`: ALLRED_BO for allred_BO_2D (arg 8 picks BO/LO), ALLRED_LO,
    // ALLRED_MEM (large_buffer = true in allred_mem_2D.cpp:15).  `device`: the
    // HIP device ordinal the program runs on (the reference's IDevice*,
    // allred_helper.hpp:75-82); -1 = ALLRED_DEVICE or the current device.
    AllredConfig(int argc, char** argv, int variant, int device = -1) {
        status = allred_args_parse(argc, const_cast<const char* const*>(argv), variant, &args);
        if (status != ALLRED_OK) return;
        if (device >= 0) args.device = device;
        SWING_VERSION = args.swing != 0;
        RUN_KERNEL = args.run_kernel != 0;
        RND_SRC = args.seed;
        NUM_TILES = args.num_tiles;
        ERROR = args.error;
        TOTAL_NODES = (uint32_t)(args.total_nodes);
        uint32_t s = 0;
        while ((1u << s) < TOTAL_NODES) ++s;
        SWING_ALGO_STEPS = s;
        num_els = (int)(single_tile_size * (uint32_t)NUM_TILES / sizeof(uint32_t));
    }

    // allred_helper.hpp:84-96: run, read back print_core's result, validate.
    int RunProgram(bool verbose = true) {
        if (status != ALLRED_OK) return status;
        status = allred_run(&args, verbose ? 1 : 0, &report);
        return status;
    }
};
