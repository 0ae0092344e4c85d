// CPython's `random.random()` stream generated on gfx950 (hot path A's reference-exact uniforms).
//
// Reference: the walkers consume one random.random() per step (random_walk_generator.py:68,113,
// `random.choices(..., k=1)`), in walk-major order; CPython draws it from MT19937
// (Modules/_randommodule.c): genrand_uint32 twists the 624-word state in place when its index
// reaches 624 and tempers mt[index++]; random() = ((a >> 5) * 67108864 + (b >> 6)) / 2^53 for two
// consecutive outputs a, b. The host replay path drew these with numpy and copied 8 B per step
// over PCIe; here they are made in HBM.
//
// Layout of the work. Let x[] be the raw (untempered) word sequence with x[0..623] = the state's
// array; the stream's word k is x[index + k]. x is cut into windows of 624 words (window w =
// x[624w .. 624w+623], i.e. CPython's twist blocks) and the windows into chains of S windows.
// One workgroup runs one chain:
//   * chain 0 starts from the state array itself;
//   * chain c >= 1 first rebuilds x[0 .. 20562) from the state in LDS (32 twists), then reads its
//     first window — and the word before it — from the jump x[J + j] = XOR_l x[l + j]
//     (j = 1..625, J = 624 S c - 2; the exponents l of t^J mod phi come from dw_mt_jump_table);
//   * then it twists window after window (three dependent phases of <= 227 words each, the
//     recurrence's parallelism: x[k] = x[k-227] ^ f(x[k-624], x[k-623])) and writes the doubles
//     whose SECOND word falls in the window (the first may sit in the previous window or chain).
// The chain holding the stream's last word also writes the final state (that window + index), so
// `random` can continue exactly where n calls of random.random() would have left it.
#include "dw_common.h"

namespace {

constexpr int MT_N = 624;
constexpr int MT_M = 397;
constexpr int MT_D = MT_N - MT_M;   // 227: words per dependent phase
constexpr uint32_t MATRIX_A = 0x9908b0dfu, UPPER = 0x80000000u, LOWER = 0x7fffffffu;
constexpr int MT_THREADS = 320;   // the chain loop: 227-word phases, 312 doubles; the jump: 2 words
constexpr int BASE_WORDS = 19937 + 625;   // x[0 .. 20562): every x[l + j] a jump reads
constexpr int MAX_POS = 19937 + 7;        // a jump's exponents (< 19937), padded to 8

__device__ __forceinline__ uint32_t twist(uint32_t a, uint32_t b, uint32_t m) {
    const uint32_t y = (a & UPPER) | (b & LOWER);
    return m ^ (y >> 1) ^ ((y & 1u) ? MATRIX_A : 0u);
}

__device__ __forceinline__ uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ double res53(uint32_t a, uint32_t b) {   // genrand_res53
    return (static_cast<double>(temper(a) >> 5) * 67108864.0 +
            static_cast<double>(temper(b) >> 6)) *
           (1.0 / 9007199254740992.0);
}

__global__ void __launch_bounds__(MT_THREADS)
    k_mt_chains(const uint32_t *__restrict__ mt_in, int32_t index, int64_t n,
                double *__restrict__ out, uint32_t *__restrict__ state_out, int64_t S,
                int64_t n_windows, const uint16_t *__restrict__ jpos,
                const int64_t *__restrict__ joff) {
    __shared__ uint32_t base[BASE_WORDS];
    __shared__ uint32_t win[2][MT_N];
    __shared__ __attribute__((aligned(16))) uint16_t pos[MAX_POS + 1];   // this chain's exponents
    __shared__ uint32_t carry;   // x[624 w0 - 1]: the first word of a double straddling chains
    const int t = threadIdx.x;
    const int64_t c = blockIdx.x;
    const int64_t w0 = c * S;
    const int64_t w1 = (w0 + S < n_windows) ? w0 + S : n_windows;
    if (n == 0) {   // nothing drawn: the state is unchanged
        if (c == 0) {
            for (int k = t; k < MT_N; k += MT_THREADS) state_out[k] = mt_in[k];
            if (t == 0) state_out[MT_N] = static_cast<uint32_t>(index);
        }
        return;
    }
    if (c == 0) {
        for (int k = t; k < MT_N; k += MT_THREADS) win[0][k] = mt_in[k];
        if (t == 0) carry = 0;
    } else {
        // the jump's exponents into LDS (read back as broadcasts, 8 per 16-B read), then
        // x[0 .. BASE_WORDS) from the state, window by window in three dependent phases
        const int64_t e0 = joff[c];
        const int cnt = static_cast<int>(joff[c + 1] - e0);
        for (int k = t; k < cnt; k += MT_THREADS) pos[k] = jpos[e0 + k];
        for (int k = cnt + t; k < ((cnt + 7) & ~7); k += MT_THREADS) pos[k] = 0;
        for (int k = t; k < MT_N; k += MT_THREADS) base[k] = mt_in[k];
        __syncthreads();
        for (int w = 1; MT_N * w < BASE_WORDS; ++w) {
            for (int ph = 0; ph < 3; ++ph) {
                const int kk = ph * MT_D + t;                       // phases of 227 words
                const int k = MT_N * w + kk;
                if (t < MT_D && kk < MT_N && k < BASE_WORDS)
                    base[k] = twist(base[k - MT_N], base[k - MT_N + 1], base[k - MT_D]);
                __syncthreads();
            }
        }
        // the jump: thread t computes x[J + j] for j = t + 1 and t + 321 (<= 625),
        // J = 624 S c - 2. 32 exponents per trip (four 16-B broadcast reads, the next trip's
        // fetched before this trip's 64 word reads are consumed), so the LDS pipe stays busy at
        // 1.25 waves per SIMD
        const uint32_t *b0 = base + t + 1;
        const uint32_t *b1 = base + (t + MT_THREADS < MT_N + 1 ? t + MT_THREADS + 1 : t + 1);
        uint32_t acc0 = 0, acc1 = 0;
        int e = 0;
        constexpr int TRIP = 32;
        uint4 pk[TRIP / 8];
        if (cnt >= TRIP) {
#pragma unroll
            for (int q = 0; q < TRIP / 8; ++q) pk[q] = *reinterpret_cast<const uint4 *>(pos + 8 * q);
        }
        for (; e + TRIP <= cnt; e += TRIP) {
            uint32_t r0[TRIP], r1[TRIP];
#pragma unroll
            for (int q = 0; q < TRIP / 8; ++q) {
                const uint32_t l[8] = {pk[q].x & 0xFFFFu, pk[q].x >> 16, pk[q].y & 0xFFFFu,
                                       pk[q].y >> 16,     pk[q].z & 0xFFFFu, pk[q].z >> 16,
                                       pk[q].w & 0xFFFFu, pk[q].w >> 16};
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    r0[8 * q + u] = b0[l[u]];
                    r1[8 * q + u] = b1[l[u]];
                }
            }
            if (e + 2 * TRIP <= cnt) {
#pragma unroll
                for (int q = 0; q < TRIP / 8; ++q)
                    pk[q] = *reinterpret_cast<const uint4 *>(pos + e + TRIP + 8 * q);
            }
#pragma unroll
            for (int u = 0; u < TRIP; ++u) {
                acc0 ^= r0[u];
                acc1 ^= r1[u];
            }
        }
        for (; e < cnt; ++e) {
            acc0 ^= b0[pos[e]];
            acc1 ^= b1[pos[e]];
        }
        if (t == 0) carry = acc0;
        else win[0][t - 1] = acc0;
        if (t + MT_THREADS < MT_N + 1) win[0][t + MT_THREADS - 1] = acc1;
    }
    __syncthreads();
    const int64_t first = index, last = index + 2 * n - 1;   // the stream's absolute words
    for (int64_t w = w0; w < w1; ++w) {
        const int cur = static_cast<int>((w - w0) & 1);
        if (w > w0) {   // window w = twist(window w - 1), the in-place loop's three phases
            const uint32_t *o = win[cur ^ 1];
            uint32_t *nw = win[cur];
            if (t < MT_D) nw[t] = twist(o[t], o[t + 1], o[t + MT_M]);
            __syncthreads();
            if (t < MT_D) nw[MT_D + t] = twist(o[MT_D + t], o[MT_D + t + 1], nw[t]);
            __syncthreads();
            if (t < MT_N - 2 * MT_D) {
                const int kk = 2 * MT_D + t;
                nw[kk] = twist(o[kk], kk + 1 < MT_N ? o[kk + 1] : nw[0], nw[kk - MT_D]);
            }
            __syncthreads();
        }
        // doubles whose second word a2 lies in this window: (a2 - index) odd
        const int64_t p0 = static_cast<int64_t>(MT_N) * w;
        const int par = static_cast<int>((p0 - first + 1) & 1);
        if (t < MT_N / 2) {
            const int64_t a2 = p0 + 2 * t + par;
            if (a2 > first && a2 <= last) {
                const int o2 = static_cast<int>(a2 - p0);
                const uint32_t x2 = win[cur][o2];
                const uint32_t x1 = o2 > 0 ? win[cur][o2 - 1]
                                           : (w == w0 ? carry : win[cur ^ 1][MT_N - 1]);
                out[(a2 - first) >> 1] = res53(x1, x2);
            }
        }
        if (w == n_windows - 1) {   // the window holding the last word: the final state
            for (int k = t; k < MT_N; k += MT_THREADS) state_out[k] = win[cur][k];
            if (t == 0) state_out[MT_N] = static_cast<uint32_t>(last + 1 - p0);
        }
    }
}

}  // namespace

extern "C" {

int dw_mt_uniforms(const uint32_t *mt, int32_t index, int64_t n, double *out,
                   uint32_t *state_out, int64_t window_stride, const uint16_t *jump_pos,
                   const int64_t *jump_off, int64_t n_chains_table, void *stream) {
    DW_REQUIRE(index >= 0 && index <= MT_N, "dw_mt_uniforms: index must be in [0, 624]");
    DW_REQUIRE(n >= 0 && n <= (int64_t(1) << 40), "dw_mt_uniforms: n must be in [0, 2^40]");
    DW_REQUIRE(window_stride >= 1, "dw_mt_uniforms: window_stride must be >= 1");
    DW_REQUIRE(mt && state_out && (out || n == 0), "dw_mt_uniforms: null pointer");
    int64_t n_windows = 1, chains = 1;
    if (n > 0) {
        n_windows = (index + 2 * n - 1) / MT_N + 1;
        chains = (n_windows + window_stride - 1) / window_stride;
    }
    DW_REQUIRE(chains == 1 || (jump_pos && jump_off && chains <= n_chains_table),
               "dw_mt_uniforms: %lld chains of %lld windows need a jump table of that many "
               "chains (dw_mt_jump_table), have %lld",
               static_cast<long long>(chains), static_cast<long long>(window_stride),
               static_cast<long long>(n_chains_table));
    DW_REQUIRE(chains < (int64_t(1) << 31), "dw_mt_uniforms: too many chains");
    hipLaunchKernelGGL(k_mt_chains, dim3(static_cast<unsigned>(chains)), dim3(MT_THREADS), 0,
                       dw::as_stream(stream), mt, index, n, out, state_out, window_stride,
                       n_windows, jump_pos, jump_off);
    DW_LAUNCH_CHECK("dw_mt_uniforms");
    return DW_OK;
}

}  // extern "C"
