// ORACLE test infrastructure: the prototypes of the reference's schedule functions,
// exactly as allred_helper.hpp:24-30, allred_BO_2D.cpp:4-5 and
// scratch_work/all_red_swing_1D/all_red_swing_1D.cpp:32 declare them.  The
// Makefile compiles the reference's own definitions (by line range, piped from
// the reference tree into the compiler: no copy is written) against this header.
#pragma once
#include <cmath>
#include <cstdint>

int highest_power_of_two(int);
uint32_t get_step_directions(int, int);
int get_comm_partner_swing_2D(int, int, bool, int, int);
int get_comm_partner_recdub_2D(int, int, bool, int, uint32_t&, int);
void get_swing_block_comm_indexes(int, int, uint32_t*, bool, int, int);
void get_recdub_block_comm_indexes(int, int, uint32_t*, bool, int, int, int, uint32_t&);
namespace ref1d {
int get_comm_partner(int node, int step, int num_nodes);
}
