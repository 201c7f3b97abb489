// config_main.cpp — a reference-style host program written against the
// source-compatible include/allred_helper.hpp only (no HIP, no torch): the
// shape of allred_BO_2D.cpp:7-215 (CreateDevice -> AllredConfig -> RunProgram)
// with the HIP device ordinal in place of the tt-metal IDevice*.
//   allred_config_main <device> <8 reference args...>
// Prints the reference's "All values match!" / mismatch report.
#include <cstdio>
#include <cstdlib>

#include "allred_helper.hpp"

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <device> <swing> <run> <side> <seed> <tiles> <err> <printcore> <bo>\n", argv[0]);
        return 2;
    }
    const int device = std::atoi(argv[1]);
    argv[1] = argv[0];   // the reference's argv layout from here on
    AllredConfig cfg(argc - 1, argv + 1, ALLRED_BO, device);
    if (cfg.status != ALLRED_OK) return 1;
    if (cfg.RunProgram() != ALLRED_OK) return 1;
    std::printf("ranks %u tiles %d device %d launches %d\n", cfg.TOTAL_NODES, cfg.NUM_TILES, cfg.args.device,
                cfg.report.launches);
    return 0;
}
