/*
 * allred_oracle_cli.c — CPU ORACLE front end (test infrastructure only).
 *
 * Loopback multi-process CPU restatement of the reference, driven with the
 * reference's positional argv (allred_helper.cpp:205-220,
 * allred_BO_2D.cpp:22-24) plus oracle-only options:
 *
 *   allred_oracle_cli <variant:bo|mem> <swing> <run> <side> <seed> <tiles>
 *                     <err> <printcore> <bo> [reps] [total_nodes] [round]
 *
 * Prints one JSON line: per-rep completion times (max end - min start, the
 * ALL_RED_LOOP normalisation of python/profiler_results_analyzer*.py), the
 * summary statistics of profiler_results_analyzer.py:39-56, mismatch count
 * and the number of online cores.  Used by bench.py's cpu_baseline leg.
 *
 * ORACLE_PROFILE_LOG=<path> also writes every rank's ALL_RED_LOOP
 * ZONE_START / ZONE_END of every rep in the layout of tt-metal's
 * profile_log_device.csv (metadata line, then the columns
 * python/profiler_results_analyzer.py:9-22 reads: core_x, core_y, RISC
 * processor type, time[cycles since reset], zone name, type), with a 1000 MHz
 * "chip" clock, i.e. one cycle = 1 ns of host time.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "allred_oracle.h"

static int cmp_d(const void* a, const void* b) {
    double x = *(const double*)a, y = *(const double*)b;
    return (x > y) - (x < y);
}

static double pct(const double* v, int n, double q) { /* numpy 'linear' percentile */
    double pos = q * (n - 1);
    int lo = (int)pos;
    int hi = lo + 1 < n ? lo + 1 : lo;
    return v[lo] + (v[hi] - v[lo]) * (pos - lo);
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s bo|mem swing run side seed tiles err printcore bo [reps] [total] [round]\n", argv[0]);
        return 2;
    }
    or_loopback_args a;
    memset(&a, 0, sizeof(a));
    a.variant = strcmp(argv[1], "mem") == 0 ? 2 : 0;
    a.swing = argc > 2 ? atoi(argv[2]) == 1 : 0;
    a.side = argc > 4 ? atoi(argv[4]) : 1;
    a.seed = argc > 5 ? atoi(argv[5]) : 0;
    a.tiles_arg = argc > 6 ? atoi(argv[6]) : 1;
    a.error = argc > 7 ? atoi(argv[7]) : 1;
    a.print_core = argc > 8 ? atoi(argv[8]) : 0;
    a.bo = argc > 9 ? atoi(argv[9]) != 0 : 0;
    a.reps = argc > 10 ? atoi(argv[10]) : 20;
    a.total = argc > 11 ? atoi(argv[11]) : 0;
    a.round_mode = argc > 12 ? atoi(argv[12]) : 0;
    if (a.reps < 1) a.reps = 1;
    double* t = (double*)calloc((size_t)a.reps, sizeof(double));
    int side = or_highest_power_of_two(a.side);
    int total = a.total > 0 ? a.total : side * side;
    const char* log_path = getenv("ORACLE_PROFILE_LOG");
    double* stamps = log_path ? (double*)calloc((size_t)a.reps * (size_t)total * 2, sizeof(double)) : NULL;
    long bad = or_loopback_run_stamps(&a, t, stamps);
    if (stamps && bad >= 0) {
        FILE* f = fopen(log_path, "w");
        if (f) {
            fprintf(f, "ARCH: cpu_loopback, CHIP_FREQ[MHz]: 1000\n");
            fprintf(f, "PCIe slot, core_x, core_y, RISC processor type, timer_id, time[cycles since reset], stat value, "
                       "run ID, run host ID,  zone name, type, source line, source file\n");
            /* ranks on the Wormhole worker cores of the reference's grid (physical
             * x / y of python/timing_taker.py:17-18), as the MI355X engine's log */
            static const int phys_x[8] = {1, 2, 3, 4, 6, 7, 8, 9}, phys_y[8] = {1, 2, 3, 4, 5, 7, 8, 9};
            for (int rep = 0; rep < a.reps; ++rep)
                for (int r = 0; r < total; ++r)
                    for (int e = 0; e < 2; ++e) {
                        const int x = r % side, y = r / side;
                        fprintf(f, "0,%d,%d,BRISC,%d,%llu,0,%d,%d,ALL_RED_LOOP,%s,0,allred_oracle.c\n",
                                x < 8 ? phys_x[x] : x + 2, y < 8 ? phys_y[y] : y + 2, e,
                                (unsigned long long)(stamps[((size_t)rep * total + r) * 2 + e] * 1e9), rep, rep,
                                e ? "ZONE_END" : "ZONE_START");
                    }
            fclose(f);
        }
    }
    free(stamps);
    int nt = or_normalize_tiles(a.tiles_arg, total, a.variant == 2 ? 1 : a.bo);
    double* s = (double*)calloc((size_t)a.reps, sizeof(double));
    memcpy(s, t, sizeof(double) * (size_t)a.reps);
    qsort(s, (size_t)a.reps, sizeof(double), cmp_d);
    double mean = 0;
    for (int i = 0; i < a.reps; ++i) mean += s[i];
    mean /= a.reps;
    printf("{\"ranks\": %d, \"bytes_per_rank\": %d, \"reps\": %d, \"mismatches\": %ld, \"online_cores\": %ld, "
           "\"min_s\": %.9g, \"q1_s\": %.9g, \"mean_s\": %.9g, \"median_s\": %.9g, \"q3_s\": %.9g, \"max_s\": %.9g, "
           "\"seconds\": [",
           total, nt * 2048, a.reps, bad, sysconf(_SC_NPROCESSORS_ONLN), s[0], pct(s, a.reps, 0.25), mean,
           pct(s, a.reps, 0.5), pct(s, a.reps, 0.75), s[a.reps - 1]);
    for (int i = 0; i < a.reps; ++i) printf("%s%.9g", i ? ", " : "", t[i]);
    printf("]}\n");
    if (bad == 0) printf("All values match!\n");
    free(t);
    free(s);
    return bad < 0 ? 1 : 0;
}
