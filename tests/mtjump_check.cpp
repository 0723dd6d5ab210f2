// Host check of the segmented sampler's jump-ahead (mt_jump.h): for a few segment lengths L and
// k = 1 .. 4, the 624 words x[n0 + kL + 1 + j] rebuilt as XOR_{c_i = 1} x[n0 + i + 1 + j] from
// c = x^(kL) mod phi equal the directly generated MT19937 stream.  Built and run by
// tests/test_abi.py::test_mt_jump_windows (g++, no GPU).
#include "mt_jump.h"

#include <chrono>
#include <cstdio>
#include <vector>

int main() {
    const int64_t Ls[] = {20561, 33696, 100003};
    const int nk = 4;
    const int64_t n0 = 624 * 3;   // a key block a few blocks into the stream
    const int64_t need = n0 + nk * 100003 + 1 + 624 + 8;
    std::vector<uint32_t> x((size_t)need);
    x[0] = 12345U;
    for (int i = 1; i < 624; ++i) x[i] = 1812433253U * (x[i - 1] ^ (x[i - 1] >> 30)) + (uint32_t)i;
    for (size_t n = 624; n < x.size(); ++n) {
        const uint32_t y = (x[n - 624] & 0x80000000U) | (x[n - 623] & 0x7fffffffU);
        x[n] = x[n - 227] ^ (y >> 1) ^ ((y & 1U) ? 0x9908b0dfU : 0U);
    }
    size_t bad = 0, checked = 0;
    for (int64_t L : Ls) {
        std::vector<uint32_t> c((size_t)nk * sacx::MT_JUMP_WORDS);
        const auto t0 = std::chrono::steady_clock::now();
        sacx::mt_jump_polys(L, nk, c.data());
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        int weight = 0;
        for (int k = 1; k <= nk; ++k) {
            const uint32_t* ck = c.data() + (size_t)(k - 1) * sacx::MT_JUMP_WORDS;
            for (int j = 0; j < 624; ++j) {
                uint32_t acc = 0;
                for (int i = 0; i < sacx::MT_DEG; ++i)
                    if ((ck[i >> 5] >> (i & 31)) & 1U) acc ^= x[(size_t)(n0 + i + 1 + j)];
                bad += acc != x[(size_t)(n0 + k * L + 1 + j)];
                ++checked;
            }
            if (k == 1)
                for (int w = 0; w < sacx::MT_JUMP_WORDS; ++w) weight += __builtin_popcount(ck[w]);
        }
        std::printf("L = %lld: %d jumps in %.1f ms, weight of x^L mod phi %d\n", (long long)L, nk, ms, weight);
    }
    std::printf("%zu of %zu jumped words checked: %zu mismatches\n", checked, checked, bad);
    return bad ? 1 : 0;
}
