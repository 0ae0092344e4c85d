// Host side of the device MT19937 stream (dw_mt.hip): jump-ahead polynomials.
//
// The reference draws one `random.random()` per walk step (random_walk_generator.py:68,113 via
// random.choices) from CPython's global Mersenne Twister (Modules/_randommodule.c: MT19937,
// genrand_res53 = ((a >> 5) * 2^26 + (b >> 6)) / 2^53 from two consecutive 32-bit outputs).
// The device generator splits the stream into chains that start at absolute positions
// 624 * S * c of the raw (untempered) word sequence x[] and runs them in parallel; each chain's
// first words come from a jump: with t^J mod phi(t) = sum_l c_l t^l,
//     x[J + j] = XOR_{l : c_l = 1} x[l + j]      for every j >= 1
// (the 32 bit planes of x each satisfy the recurrence whose characteristic polynomial is phi;
// Haramoto et al., "Efficient jump ahead for F2-linear random number generators", 2008).
// phi is MT19937's characteristic polynomial: degree 19937, 135 terms (below; recovered by
// Berlekamp-Massey from the generator's bit sequence and checked against CPython's stream in
// tests/test_host.py). This file computes, for each chain c >= 1, the exponents l of
// t^(624 S c - 2) mod phi — chain c reads x[624 S c - 1 .. 624 S c + 623], the word before its
// first window too (a double of the stream can straddle two chains).
#include <string.h>
#include <wmmintrin.h>

#include <vector>

#include "../../include/dw_hip.h"

namespace dw {
void set_error(const char *fmt, ...);
}

#define DW_REQUIRE_H(cond, ...)          \
    do {                                 \
        if (!(cond)) {                   \
            ::dw::set_error(__VA_ARGS__); \
            return DW_E_INVALID_ARG;     \
        }                                \
    } while (0)

namespace {

constexpr int DEG = 19937;
constexpr int NW = (DEG + 63) / 64;   // 312 words per reduced polynomial
// exponents of phi(t) below t^19937 (phi = t^19937 + sum t^e)
constexpr int PHI_TERMS[] = {
    0,     1189,  1416,  1585,  1643,  1870,  2493,  2773,  3000,  3227,  3454,  3681,  3908,
    4135,  4362,  4753,  5661,  6337,  6569,  7129,  7477,  7525,  7583,  7752,  7979,  8206,
    9505,  9901,  9969,  10128, 10693, 10761, 10920, 11089, 11147, 11157, 11215, 11321, 11374,
    11384, 11485, 11611, 11712, 11717, 11838, 11881, 11944, 11997, 12277, 12335, 12393, 12504,
    12509, 12620, 12673, 12731, 12736, 12789, 12905, 12958, 12963, 13137, 13185, 13190, 13243,
    13301, 13412, 13528, 13533, 13639, 13697, 13760, 13813, 13866, 14093, 14151, 14209, 14320,
    14325, 14436, 14547, 14552, 14605, 14721, 14774, 14779, 14953, 15001, 15006, 15059, 15117,
    15228, 15344, 15349, 15455, 15513, 15576, 15629, 15682, 15909, 15967, 16025, 16136, 16141,
    16252, 16363, 16368, 16421, 16537, 16590, 16595, 16817, 16822, 16875, 16933, 17044, 17160,
    17271, 17329, 17445, 17498, 17725, 17783, 17841, 17952, 18068, 18179, 18237, 18406, 18633,
    18691, 18860, 19087, 19314};
constexpr int N_TERMS = sizeof(PHI_TERMS) / sizeof(PHI_TERMS[0]);   // 134 (+ t^19937)
static_assert(N_TERMS == 134, "phi has 135 terms");

using Poly = std::vector<uint64_t>;

inline void clmul_sw(uint64_t a, uint64_t b, uint64_t &lo, uint64_t &hi) {
    lo = hi = 0;
    for (int i = 0; i < 64; ++i)
        if ((b >> i) & 1u) {
            lo ^= a << i;
            if (i) hi ^= a >> (64 - i);
        }
}

__attribute__((target("pclmul"))) void mul_full_hw(const uint64_t *a, const uint64_t *b,
                                                    uint64_t *prod) {
    for (int i = 0; i < NW; ++i) {
        if (!a[i]) continue;
        const __m128i va = _mm_set_epi64x(0, static_cast<long long>(a[i]));
        for (int j = 0; j < NW; ++j) {
            const __m128i r =
                _mm_clmulepi64_si128(va, _mm_set_epi64x(0, static_cast<long long>(b[j])), 0);
            prod[i + j] ^= static_cast<uint64_t>(_mm_cvtsi128_si64(r));
            prod[i + j + 1] ^= static_cast<uint64_t>(_mm_cvtsi128_si64(_mm_unpackhi_epi64(r, r)));
        }
    }
}

void mul_full_sw(const uint64_t *a, const uint64_t *b, uint64_t *prod) {
    for (int i = 0; i < NW; ++i) {
        if (!a[i]) continue;
        for (int j = 0; j < NW; ++j) {
            uint64_t lo, hi;
            clmul_sw(a[i], b[j], lo, hi);
            prod[i + j] ^= lo;
            prod[i + j + 1] ^= hi;
        }
    }
}

inline void xor_at(uint64_t *p, int64_t q, uint64_t v) {   // p ^= v << q (bit offset q)
    const int64_t w = q >> 6;
    const int s = static_cast<int>(q & 63);
    p[w] ^= v << s;
    if (s) p[w + 1] ^= v >> (64 - s);
}

// prod (2 NW words) mod phi -> prod[0 .. NW) (bits >= DEG cleared)
void reduce(uint64_t *prod) {
    for (int w = 2 * NW - 1; w >= NW; --w) {
        const uint64_t v = prod[w];
        if (!v) continue;
        prod[w] = 0;
        const int64_t base = 64ll * w - DEG;   // bit b of word w is t^(base + DEG + b)
        for (int k = 0; k < N_TERMS; ++k) xor_at(prod, base + PHI_TERMS[k], v);
    }
    const int top = DEG - 64 * (NW - 1);     // 33 bits of word NW-1 are below DEG
    const uint64_t v = prod[NW - 1] >> top;
    if (v) {
        prod[NW - 1] &= (uint64_t(1) << top) - 1;
        for (int k = 0; k < N_TERMS; ++k) xor_at(prod, PHI_TERMS[k], v);
    }
}

bool have_pclmul() {
    static const bool h = __builtin_cpu_supports("pclmul");
    return h;
}

Poly mulmod(const Poly &a, const Poly &b) {
    std::vector<uint64_t> prod(2 * NW + 1, 0);
    if (have_pclmul())
        mul_full_hw(a.data(), b.data(), prod.data());
    else
        mul_full_sw(a.data(), b.data(), prod.data());
    reduce(prod.data());
    return Poly(prod.begin(), prod.begin() + NW);
}

Poly monomial(int64_t e) {   // t^e, e < DEG
    Poly p(NW, 0);
    p[e >> 6] = uint64_t(1) << (e & 63);
    return p;
}

Poly powmod_t(uint64_t e) {   // t^e mod phi
    if (e < static_cast<uint64_t>(DEG)) return monomial(static_cast<int64_t>(e));
    Poly r = monomial(0), b = monomial(1);
    while (e) {
        if (e & 1u) r = mulmod(r, b);
        e >>= 1;
        if (e) b = mulmod(b, b);
    }
    return r;
}

}  // namespace

extern "C" {

int dw_mt_jump_table(int64_t window_stride, int64_t n_chains, int64_t *offsets, uint16_t *positions,
                     int64_t capacity) {
    DW_REQUIRE_H(window_stride >= 1 && window_stride <= (int64_t(1) << 40),
                 "dw_mt_jump_table: window_stride must be in [1, 2^40]");
    DW_REQUIRE_H(n_chains >= 1 && n_chains <= (int64_t(1) << 20),
                 "dw_mt_jump_table: n_chains must be in [1, 2^20]");
    DW_REQUIRE_H(offsets, "dw_mt_jump_table: offsets is null");
    DW_REQUIRE_H(capacity >= 0 && (positions || capacity == 0),
                 "dw_mt_jump_table: positions is null");
    const uint64_t stride_words = 624ull * static_cast<uint64_t>(window_stride);
    offsets[0] = 0;
    offsets[1] = 0;   // chain 0 starts from the generator state itself
    if (n_chains == 1) return DW_OK;
    Poly g = powmod_t(stride_words);          // t^(624 S)
    Poly tc = powmod_t(stride_words - 2);     // chain 1: t^(624 S - 2)
    int64_t k = 0;
    bool full = false;
    for (int64_t c = 1; c < n_chains; ++c) {
        if (c > 1) tc = mulmod(tc, g);
        for (int w = 0; w < NW; ++w) {
            uint64_t v = tc[w];
            while (v) {
                const int b = __builtin_ctzll(v);
                v &= v - 1;
                if (k < capacity)
                    positions[k] = static_cast<uint16_t>(64 * w + b);
                else
                    full = true;
                ++k;
            }
        }
        offsets[c + 1] = k;
    }
    DW_REQUIRE_H(!full, "dw_mt_jump_table: capacity %lld < %lld positions needed",
                 static_cast<long long>(capacity), static_cast<long long>(k));
    return DW_OK;
}

}  // extern "C"
