// cli.cpp — the reference executables on MI355X:
//   allred_BO_2D  <swing> <run> <side> <seed> <tiles> <err> <printcore> <bo>   (allred_BO_2D.cpp:7-215)
//   allred_LO_2D  <swing> <run> <side> <seed> <tiles> <err>                   (allred_LO_2D.cpp:9-106)
//   allred_mem_2D <swing> <run> <side> <seed> <tiles> <err>                   (allred_mem_2D.cpp:4-165)
// Same positional arguments, defaults and clamping (allred_helper.cpp:205-220);
// prints "All values match!" or the reference's mismatch report.
// Extensions (never needed for reference invocations):
//   argv[9] or ALLRED_NODES   rank count (rectangular grids, e.g. 8 = 4x2)
//   ALLRED_EXEC=fused         one-launch execution of the same arithmetic
//   ALLRED_BF16_ROUND=rne     RNE bfloat16(float) for inputs/expected values
//   ALLRED_CHECK_ALL=1        validate every rank, not only <printcore>
//   ALLRED_REPORT=1           print a JSON timing line to stderr
//   ALLRED_STRICT=1           exit 1 on mismatch (the reference always exits 0)
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "allred.h"

#ifndef ALLRED_CLI_VARIANT
#define ALLRED_CLI_VARIANT ALLRED_BO
#endif

int main(int argc, char** argv) {
    allred_args args;
    int st = allred_args_parse(argc, const_cast<const char* const*>(argv), ALLRED_CLI_VARIANT, &args);
    if (st != ALLRED_OK) {
        std::fprintf(stderr, "terminate called after throwing an instance of 'std::invalid_argument'\n  what():  stoi\n");
        return 134;
    }
    allred_report rep;
    st = allred_run(&args, 1, &rep);
    if (st != ALLRED_OK) {
        std::fprintf(stderr, "%s: %s\n", argv[0], allred_status_string(st));
        return 1;
    }
    if (std::getenv("ALLRED_REPORT")) {
        std::fprintf(stderr,
                     "{\"ranks\": %d, \"bytes_per_rank\": %llu, \"launches\": %d, \"device_s\": %.9g, "
                     "\"e2e_s\": %.9g, \"mismatches\": %lld, \"max_error\": %g}\n",
                     rep.total_nodes, (unsigned long long)rep.bytes_per_rank, rep.launches, rep.device_seconds,
                     rep.e2e_seconds, (long long)rep.mismatches, rep.max_error);
    }
    if (std::getenv("ALLRED_STRICT") && rep.mismatches != 0) return 1;
    return 0;
}
