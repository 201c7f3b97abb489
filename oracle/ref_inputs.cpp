// TEST INFRASTRUCTURE ONLY — never linked into the product.
//
// Golden-input generator.  The reference draws its inputs with tt-metal's
// create_random_vector_of_bfloat16(bytes, 100, seed) (allred_helper.cpp:283-284),
// which lives in tt-metalium/bfloat16.hpp — NOT vendored in /root/reference
// and not pinned to a version.  Its published algorithm is restated here on
// top of the C++ standard library objects it uses, so the std::mt19937 and
// std::uniform_real_distribution<float> below are libstdc++'s own:
//   auto rand_float = std::bind(std::uniform_real_distribution<float>(0, rand_max),
//                               std::mt19937(seed));
//   two draws per uint32, first in the low half, bfloat16(float) each.
// Both bfloat16(float) conventions are emitted: truncation (the ctor of the
// v0.5x era the reference's API matches) and round-to-nearest-even (later
// tt-metal).  Output feeds tests/golden/inputs_ref.json.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <random>
#include <vector>

static uint16_t bf16_trunc(float f) { uint32_t u; std::memcpy(&u, &f, 4); return (uint16_t)(u >> 16); }
static uint16_t bf16_rne(float f) {
    uint32_t u; std::memcpy(&u, &f, 4);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

static std::vector<uint32_t> make(size_t num_bytes, int rand_max, int seed, bool rne) {
    auto rand_float = std::bind(std::uniform_real_distribution<float>(0, rand_max), std::mt19937(seed));
    std::vector<uint32_t> vec(num_bytes / sizeof(uint32_t), 0);
    for (size_t i = 0; i < vec.size(); ++i) {
        float a = rand_float() + 0.0f;
        float b = rand_float() + 0.0f;
        uint16_t ha = rne ? bf16_rne(a) : bf16_trunc(a);
        uint16_t hb = rne ? bf16_rne(b) : bf16_trunc(b);
        vec[i] = (uint32_t)ha | ((uint32_t)hb << 16);
    }
    return vec;
}

static uint64_t fnv1a(const std::vector<uint32_t>& v) {
    uint64_t h = 1469598103934665603ull;
    for (uint32_t w : v)
        for (int k = 0; k < 4; ++k) { h ^= (w >> (8 * k)) & 0xffu; h *= 1099511628211ull; }
    return h;
}

int main() {
    const int seeds[] = {0, 1, 13, 14, 42};
    const size_t sizes[] = {2048, 655360};
    std::printf("{\"generator\": \"libstdc++ mt19937 + uniform_real_distribution<float>(0,100)\", \"vectors\": [\n");
    bool first = true;
    for (int rne = 0; rne < 2; ++rne)
        for (int seed : seeds)
            for (size_t bytes : sizes) {
                auto v = make(bytes, 100, seed, rne != 0);
                std::printf("%s  {\"seed\": %d, \"bytes\": %zu, \"round\": \"%s\", \"fnv1a64\": \"%016llx\", \"head\": [",
                            first ? "" : ",\n", seed, bytes, rne ? "rne" : "trunc", (unsigned long long)fnv1a(v));
                for (int i = 0; i < 16; ++i) std::printf("%s%u", i ? ", " : "", v[i]);
                std::printf("]}");
                first = false;
            }
    std::printf("\n]}\n");
    return 0;
}
