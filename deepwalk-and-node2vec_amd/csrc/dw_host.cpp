// Host-side runtime pieces of the C ABI (no device code).
//
// dw_host_shuffle: CPython 3.10's random.shuffle over range(n), bit for bit, in native code.
// The reference shuffles its start-node list with the global `random` once in the
// RandomWalkDataset constructor and again at every epoch end (datasets.py:45,86-88); in Python
// that loop costs ~0.5 s per epoch for 1M nodes. The Mersenne Twister below is CPython's
// _randommodule.c genrand_uint32 (MT19937, N = 624, M = 397), `getrandbits(k) = genrand >> (32 -
// k)` for k <= 32, and Lib/random.py `_randbelow_with_getrandbits` / `shuffle`:
//     for i in reversed(range(1, n)): j = randbelow(i + 1); x[i], x[j] = x[j], x[i]
//     randbelow(m): k = m.bit_length(); r = getrandbits(k); while r >= m: r = getrandbits(k)
// The caller passes the generator state as random.getstate()[1] (624 words + index) and writes
// the advanced state back with random.setstate, so the global stream continues exactly where
// Python's own shuffle would have left it.
#include <stdint.h>

#include "dw_common.h"

namespace {

constexpr int MT_N = 624, MT_M = 397;
constexpr uint32_t MATRIX_A = 0x9908b0dfu, UPPER = 0x80000000u, LOWER = 0x7fffffffu;

struct MT {
    uint32_t *mt;   // 624 words
    uint32_t idx;

    uint32_t next() {
        if (idx >= MT_N) {
            int kk = 0;
            uint32_t y;
            for (; kk < MT_N - MT_M; ++kk) {
                y = (mt[kk] & UPPER) | (mt[kk + 1] & LOWER);
                mt[kk] = mt[kk + MT_M] ^ (y >> 1) ^ ((y & 1u) ? MATRIX_A : 0u);
            }
            for (; kk < MT_N - 1; ++kk) {
                y = (mt[kk] & UPPER) | (mt[kk + 1] & LOWER);
                mt[kk] = mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ ((y & 1u) ? MATRIX_A : 0u);
            }
            y = (mt[MT_N - 1] & UPPER) | (mt[0] & LOWER);
            mt[MT_N - 1] = mt[MT_M - 1] ^ (y >> 1) ^ ((y & 1u) ? MATRIX_A : 0u);
            idx = 0;
        }
        uint32_t y = mt[idx++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
};

inline int bit_length(uint64_t m) {
    int k = 0;
    while (m) {
        ++k;
        m >>= 1;
    }
    return k;
}

}  // namespace

extern "C" {

int dw_host_shuffle(uint32_t *mt_state, int64_t *perm, int64_t n) {
    DW_REQUIRE(mt_state && (perm || n == 0), "dw_host_shuffle: null pointer");
    DW_REQUIRE(n >= 0 && n <= (int64_t(1) << 32), "dw_host_shuffle: n must be in [0, 2^32]");
    DW_REQUIRE(mt_state[MT_N] <= static_cast<uint32_t>(MT_N), "dw_host_shuffle: bad MT index");
    MT g{mt_state, mt_state[MT_N]};
    for (int64_t i = 0; i < n; ++i) perm[i] = i;
    for (int64_t i = n - 1; i >= 1; --i) {
        const uint64_t m = static_cast<uint64_t>(i) + 1;   // randbelow(i + 1), i + 1 <= 2^32
        const int k = bit_length(m);
        uint64_t r;
        do {
            if (k <= 32) {
                r = g.next() >> (32 - k);
            } else {   // k = 33 (m = 2^32): getrandbits fills 32-bit words, least significant first
                const uint64_t lo = g.next();
                r = lo | (static_cast<uint64_t>(g.next() >> 31) << 32);
            }
        } while (r >= m);
        const int64_t j = static_cast<int64_t>(r);
        const int64_t t = perm[i];
        perm[i] = perm[j];
        perm[j] = t;
    }
    mt_state[MT_N] = g.idx;
    return DW_OK;
}

}  // extern "C"
