// Host side of a4: the patch-index draws of dip/lrf.py:76,
// np.random.choice(n, patch_size, replace=False), for a whole query set in one
// call and on the caller's own numpy RandomState stream (MT19937), so that the
// draws -- and the state the caller's RNG is left in -- are those of the
// reference's per-query loop (demo.py:109-114 interleaves two clouds' calls).
//
// Legacy RandomState.choice without replacement and without p is
// permutation(n)[:k]; permutation is a Fisher-Yates shuffle of arange(n) that
// walks i = n-1 .. 1 and swaps x[i] with x[j], j uniform in [0, i] drawn by
// masked rejection on 32-bit MT19937 outputs (mask = smallest 2^b - 1 >= i;
// redraw while (u & mask) > i).  Every call consumes the draws of the full
// shuffle, whatever k is.
#include <stdint.h>
#include <vector>

#include "pcr_internal.h"

namespace {

constexpr int kMtN = 624, kMtM = 397;

struct Mt {
    uint32_t *key;
    int pos;

    void regenerate() {
        auto mix = [](uint32_t a, uint32_t b) {
            const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
            return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        };
        int i = 0;
        for (; i < kMtN - kMtM; ++i) key[i] = key[i + kMtM] ^ mix(key[i], key[i + 1]);
        for (; i < kMtN - 1; ++i) key[i] = key[i + kMtM - kMtN] ^ mix(key[i], key[i + 1]);
        key[kMtN - 1] = key[kMtM - 1] ^ mix(key[kMtN - 1], key[0]);
        pos = 0;
    }

    static uint32_t temper(uint32_t y) {
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }
};

}  // namespace

extern "C" int pcr_legacy_choice_batch(uint32_t *key, int32_t *pos, const int32_t *pop,
                                       int32_t calls, int32_t k, int32_t *out) {
    pcr::clear_error();
    PCR_REQUIRE(calls >= 0 && k >= 0, PCR_ERR_ARG, "legacy_choice: negative size");
    if (calls == 0) return PCR_OK;
    PCR_REQUIRE(key && pos && pop && out, PCR_ERR_ARG, "legacy_choice: null pointer");
    PCR_REQUIRE(*pos >= 0 && *pos <= kMtN, PCR_ERR_ARG, "legacy_choice: MT19937 pos out of range");
    int32_t nmax = 0;
    for (int32_t c = 0; c < calls; ++c) {
        PCR_REQUIRE(pop[c] >= k && pop[c] > 0, PCR_ERR_ARG,
                    "legacy_choice: cannot take a larger sample than population when replace=False");
        nmax = pop[c] > nmax ? pop[c] : nmax;
    }
    // tempered outputs of one 624-word block at a time (the tempering loop
    // vectorises); the shuffle consumes them branch-free: a rejected draw swaps
    // x[i] with itself and leaves i unchanged.  (A serial acceptance scan plus a
    // parallel replay of the shuffles measured slower: the scan is the same
    // dependency chain.)
    Mt mt{key, *pos};
    std::vector<int32_t> x((size_t)nmax);
    uint32_t tv[kMtN];
    int tpos = mt.pos;
    for (int t = tpos; t < kMtN; ++t) tv[t] = Mt::temper(mt.key[t]);
    for (int32_t c = 0; c < calls; ++c) {
        const int32_t n = pop[c];
        for (int32_t i = 0; i < n; ++i) x[i] = i;
        int32_t i = n - 1;
        while (i >= 1) {
            if (tpos >= kMtN) {
                mt.regenerate();
                for (int t = 0; t < kMtN; ++t) tv[t] = Mt::temper(mt.key[t]);
                tpos = 0;
            }
            const uint32_t mask = 0xffffffffu >> __builtin_clz((uint32_t)i);
            const uint32_t u = tv[tpos++] & mask;
            const bool acc = u <= (uint32_t)i;
            const int32_t j = acc ? (int32_t)u : i;
            const int32_t t = x[j];
            x[j] = x[i];
            x[i] = t;
            i -= acc;
        }
        for (int32_t q = 0; q < k; ++q) out[(size_t)c * k + q] = x[q];
    }
    mt.pos = tpos;
    *pos = mt.pos;
    return PCR_OK;
}
