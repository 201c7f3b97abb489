// host_data.cpp — the reference's host-side data helpers.
//
//   create_random_vector_of_bfloat16 / create_constant_vector_of_bfloat16
//       tt-metal tt-metalium/bfloat16.hpp (not vendored), called at
//       allred_helper.cpp:277-285: std::mt19937(seed) feeding
//       std::uniform_real_distribution<float>(0, rand_max), two draws per
//       uint32 (first in the low half), bfloat16(float) on each.
//   validate_result_vector  allred_helper.cpp:18-120 (same messages).
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <functional>
#include <random>
#include <string>

#include "internal.hpp"

using namespace tsa;

namespace {
inline uint16_t to_bf16(float f, int round_mode) {
    return round_mode ? bf16_from_float_rne(f) : bf16_from_float_trunc(f);
}
inline uint16_t half_of(const uint32_t* v, size_t i) {
    return (uint16_t)((i & 1) ? (v[i >> 1] >> 16) : (v[i >> 1] & 0xffffu));
}
inline uint32_t pack2(uint16_t lo, uint16_t hi) { return (uint32_t)lo | ((uint32_t)hi << 16); }
}  // namespace

extern "C" {

void allred_random_bf16_vector(size_t num_bytes, int rand_max, int seed, int round_mode, uint32_t* out) {
    std::mt19937 gen(seed);
    std::uniform_real_distribution<float> dist(0.0f, (float)rand_max);
    const size_t words = num_bytes / sizeof(uint32_t);
    for (size_t i = 0; i < words; ++i) {
        const float a = dist(gen) + 0.0f;
        const float b = dist(gen) + 0.0f;
        out[i] = pack2(to_bf16(a, round_mode), to_bf16(b, round_mode));
    }
}

void allred_constant_bf16_vector(size_t num_bytes, float value, uint32_t* out) {
    const uint16_t h = bf16_from_float_trunc(value);
    const size_t words = num_bytes / sizeof(uint32_t);
    for (size_t i = 0; i < words; ++i) out[i] = pack2(h, h);
}

long allred_validate_result_vector(const uint32_t* result, const uint32_t* src0, const uint32_t* src1,
                                   size_t num_els, float error, uint32_t total_nodes, int verbose,
                                   float* max_error_out) {
    const char* mode = std::getenv("ALLRED_BF16_ROUND");
    const int round_mode = (mode && std::string(mode) == "rne") ? 1 : 0;
    const size_t count = num_els * 2;
    std::vector<uint16_t> trgt(count);
    bool all_match = true;
    long bad = 0, num_matches = 0;
    size_t last_match = 0, last_wrong = 0, max_idx = 0;
    float max_error = 0.0f;
    std::string blocks = "Mismatch blocks: ";
    const float mult = (float)(total_nodes / 2);  // integer division, as the reference
    for (size_t i = 0; i < count; ++i) {
        const float a = bf16_to_float(half_of(src0, i)), b = bf16_to_float(half_of(src1, i));
        trgt[i] = to_bf16((a + b) * mult, round_mode);
        const float actual = bf16_to_float(half_of(result, i));
        const float expected = bf16_to_float(trgt[i]);
        const float diff = std::fabs(actual - expected);
        if (all_match && diff > error) {
            if (verbose) {
                std::printf("Mismatch at index %zu:\n", i);
                std::printf("  Expected: %d\n", (int)expected);
                std::printf("  Actual  : %d\n", (int)actual);
                std::printf("  Original values: %f %f\n\n", a, b);
            }
            all_match = false;
            ++bad;
            if (i % 1024 == 0) blocks += std::to_string(i / 1024) + " ";
        } else if (diff <= error) {
            last_match = i;
            ++num_matches;
        } else {
            ++bad;
            last_wrong = i;
            if (diff > max_error) {
                max_error = diff;
                max_idx = i;
            }
            if (i % 1024 == 0) blocks += std::to_string(i / 1024) + " ";
        }
    }
    if (max_error_out) *max_error_out = max_error;
    if (!verbose) return bad;
    if (all_match) {
        std::printf("All values match!\n");
        return bad;
    }
    auto val = [&](const uint32_t* v, size_t i) { return (int)bf16_to_float(half_of(v, i)); };
    std::printf("Total matches: %ld\n", num_matches);
    std::printf("Last match at index %d: %d\n\n", (int)last_match, val(result, last_match));
    std::printf("Last wrong at index %d: %d Shpuld be: %d\n\n", (int)last_wrong, val(result, last_wrong),
                (int)bf16_to_float(trgt[last_wrong]));
    std::printf("Result (nocast) = %d, casted = %d\n", (int)result[0], val(result, 0));
    std::printf("Expected (nocast) = %d, casted = %d\n", (int)pack2(trgt[0], trgt[1]),
                (int)bf16_to_float(trgt[0]));
    std::printf("Actual last result (nocast) = %d, casted = %d\n", (int)result[num_els - 1],
                val(result, 2 * num_els - 1));
    std::printf("Expected last result (nocast) = %d, casted = %d\n",
                (int)pack2(trgt[2 * num_els - 2], trgt[2 * num_els - 1]),
                (int)bf16_to_float(trgt[2 * num_els - 1]));
    std::printf("Max error: %f\n", max_error);
    std::printf("Max error index: %d, values %f vs %f\n", (int)max_idx,
                bf16_to_float(half_of(result, max_idx)), bf16_to_float(trgt[max_idx]));
    if (max_idx + 10 < count)
        std::printf("Max error index +10: %d, values %f vs %f", (int)(max_idx + 10),
                    bf16_to_float(half_of(result, max_idx + 10)), bf16_to_float(trgt[max_idx + 10]));
    std::printf("\n%s\n________________\n", blocks.c_str());
    return bad;
}

}  // extern "C"
