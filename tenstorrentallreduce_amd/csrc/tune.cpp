// tune.cpp — the one tuning entry point of liballred.so (allred_tune_set /
// allred_tune_get, include/allred.h).  Every key selects between kernel forms
// that give bit-identical results; the defaults are the measured product
// forms, so nothing needs setting.  Initial values may come
// from ALLRED_TUNE="key=value,key=value", read once when the library loads.
// No reference counterpart: the reference compiles one kernel per variant
// (allred_BO_2D.cpp:203-211 picks the kernel directory by string).
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <string>

#include "internal.hpp"

namespace tsa {
namespace {

struct Key {
    const char* name;
    int64_t def, lo, hi;
};

// order = enum class Tune (internal.hpp)
const Key kKeys[] = {
    {"fused_form", 0, 0, 3},          // 0 auto | 1 k_tree | 2 k_tree_lds | 3 k_tree_lds_pipe
    {"lo_tree", 1, 0, 1},             // rank-uniform fused LO through the BO tree pass
    {"lo_dag", 1, 0, 1},              // 64-rank fused LO as the DAG of distinct sums
    {"lo_dag_place", 1, 0, 1},        // bank-conflict-free DAG placement
    {"lo_dag_min_tiles", 256, 1, 1ll << 40},
    {"mem_reduce_lds", 1, 0, 1},      // mem_2D schedule-form reduce through LDS
    {"steps_form", 0, 0, 2},          // 0 pipelined launch | 1 one launch per step | 2 all units resident
    {"pipe_grid", 0, 0, 1 << 20},     // 0 auto
    {"lo_dag_reg", 1, 0, 1},          // non-rank-uniform Swing fused LO: build-time DAG in registers
    {"lo_dag_reg_min_tiles", 64, 1, 1ll << 40},   // 256-element tiles per rank (64: 32 kB)
    {"check", 0, 0, 1},               // N > 1 programs: verify against the partners', poison receive regions
    {"fused_chunk_tiles", 1280, 0, 1ll << 40},   // persistent fused passes: tiles per launch (0: one launch)
    {"lo_tree_min_tiles", 64, 0, 1ll << 40},   // 64-rank rank-uniform LO: tree pass from this many 256-element tiles
    {"tree_bcast_lag", 1, 0, 1},      // k_tree_bcast_x: the row stores one iteration behind the tree (0: same iteration)
    {"tree_bcast_bal", 0, 0, 1},      // k_tree_bcast_x: every wave stages / stores 8 result columns (0: wave 0 all)
    {"steps_groups", 0, 0, 5},        // k_steps_reg: workgroups per CU, 0 auto (BO 3, LO 4 or 3) | 3 | 4 | 5
    {"rccl_fault", 0, 0, 7},          // fault injection (tests): 1 init, 2 group end, 4 stream drain never settle
    {"multi_fault", 0, 0, 64},        // fault injection (tests): 1..32 GPU value - 1 fails its timed allreduce, 33..64 its warm-up
    {"steps_tab", 1, 0, 1},           // k_steps_reg BO: 1 stages only its units' block programs (J < P), 0 every block's
    {"steps_early", 1, 0, 2},         // k_steps_reg: the first strip's loads before the program staging: 0 never | 1 auto (full grid) | 2 always
    {"peer_fence", 0, 0, 1},          // peer kernels: 1 system-scope release / acquire fences around every cross-GPU hand-off
    {"hier_ws_ahead", 1, 1, 2},       // k_hier_ws: the reducing waves' loads 1 | 2 tiles ahead
    {"hier_ws_cols", 16, 8, 32},      // k_hier_ws: 16-byte columns per reducing wave, 8 (quarters) | 16 (halves) | 32 (whole tiles)
};
constexpr int kCount = (int)(sizeof(kKeys) / sizeof(kKeys[0]));
static_assert(kCount == (int)Tune::count, "kKeys and enum Tune disagree");

std::atomic<int64_t> g_val[kCount];

int find(const char* key) {
    if (!key) return -1;
    for (int i = 0; i < kCount; ++i)
        if (std::strcmp(kKeys[i].name, key) == 0) return i;
    return -1;
}

bool set(int i, int64_t v) {
    if (v < kKeys[i].lo || v > kKeys[i].hi) return false;
    if (i == (int)Tune::steps_groups && (v == 1 || v == 2)) return false;   // 0 auto, 3, 4, 5 only
    if (i == (int)Tune::hier_ws_cols && v != 8 && v != 16 && v != 32) return false;   // quarters, halves, whole tiles
    g_val[i].store(v, std::memory_order_relaxed);
    return true;
}

struct Init {
    Init() {
        for (int i = 0; i < kCount; ++i) g_val[i].store(kKeys[i].def, std::memory_order_relaxed);
        const char* env = std::getenv("ALLRED_TUNE");
        if (!env) return;
        std::string s(env);
        size_t pos = 0;
        while (pos < s.size()) {
            size_t end = s.find(',', pos);
            if (end == std::string::npos) end = s.size();
            const std::string item = s.substr(pos, end - pos);
            const size_t eq = item.find('=');
            if (eq != std::string::npos) {
                const int i = find(item.substr(0, eq).c_str());
                if (i >= 0) set(i, std::strtoll(item.c_str() + eq + 1, nullptr, 10));
            }
            pos = end + 1;
        }
    }
} g_init;

}  // namespace

int64_t tune(Tune k) { return g_val[(int)k].load(std::memory_order_relaxed); }

}  // namespace tsa

extern "C" {

int allred_tune_set(const char* key, int64_t value) {
    const int i = tsa::find(key);
    if (i < 0 || !tsa::set(i, value)) return ALLRED_ERR_ARG;
    return ALLRED_OK;
}

int allred_tune_get(const char* key, int64_t* value) {
    const int i = tsa::find(key);
    if (i < 0 || !value) return ALLRED_ERR_ARG;
    *value = tsa::g_val[i].load(std::memory_order_relaxed);
    return ALLRED_OK;
}

}  // extern "C"
