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
// Two launches:
//   * k_mt_jump, one 1,024-thread workgroup per chain c >= 1: it rebuilds x[0 .. 20562) from the
//     state in LDS (32 twists), then computes the chain's first window — and the word before it
//     — as the jump x[J + j] = XOR_l x[l + j] (j = 1..625, J = 624 S c - 2; the exponents l of
//     t^J mod phi come from dw_mt_jump_table) into a workspace. A jump is ~10^4 exponents x 625
//     LDS reads: bound by the LDS, which wants four waves per SIMD for 4-B reads;
//   * k_mt_chains, one 320-thread workgroup per chain (chain 0 from the state array itself, the
//     others from the workspace) with 5 KiB of LDS, so several chains share a CU: it twists
//     window after window (three dependent phases of <= 227 words each, the recurrence's
//     parallelism: x[k] = x[k-227] ^ f(x[k-624], x[k-623])) and writes the doubles whose SECOND
//     word falls in the window (the first may sit in the previous window or chain).
// The chain holding the stream's last word also writes the final state (that window + index), so
// `random` can continue exactly where n calls of random.random() would have left it.
#include "dw_common.h"

namespace {

constexpr int MT_N = 624;
constexpr int MT_M = 397;
constexpr int MT_D = MT_N - MT_M;   // 227: words per dependent phase
constexpr uint32_t MATRIX_A = 0x9908b0dfu, UPPER = 0x80000000u, LOWER = 0x7fffffffu;
constexpr int MT_THREADS = 320;    // the chain loop: 227-word phases, 312 doubles per window
constexpr int JUMP_THREADS = 1024; // the jumps: one output word per thread, 4 waves per SIMD
constexpr int BASE_WORDS = 19937 + 625;   // x[0 .. 20562): every x[l + j] a jump reads
constexpr int MAX_POS = 19937 + 7;        // a jump's exponents (< 19937), padded to 8
constexpr int JWIN = 640;                 // words per chain in the jump workspace (625 used)

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

__global__ void __launch_bounds__(JUMP_THREADS)
    k_mt_jump(const uint32_t *__restrict__ mt_in, const uint16_t *__restrict__ jpos,
              const int64_t *__restrict__ joff, uint32_t *__restrict__ jwin) {
    __shared__ uint32_t base[BASE_WORDS];
    __shared__ __attribute__((aligned(16))) uint16_t pos[MAX_POS + 1];   // this chain's exponents
    const int t = threadIdx.x;
    const int64_t c = blockIdx.x + 1;
    // the exponents into LDS (read back as broadcasts, 8 per 16-B read), then x[0 .. BASE_WORDS)
    // from the state, window by window in three dependent phases
    const int64_t e0 = joff[c];
    const int cnt = static_cast<int>(joff[c + 1] - e0);
    for (int k = t; k < cnt; k += JUMP_THREADS) pos[k] = jpos[e0 + k];
    for (int k = t; k < MT_N; k += JUMP_THREADS) base[k] = mt_in[k];
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
    // thread t <= 624 computes x[J + t + 1], J = 624 S c - 2; 32 exponents per trip (four 16-B
    // broadcast reads, the next trip's fetched before this trip's 32 word reads are consumed)
    if (t > MT_N) return;
    const uint32_t *b0 = base + t + 1;
    uint32_t acc = 0;
    int e = 0;
    constexpr int TRIP = 32;
    uint4 pk[TRIP / 8];
    if (cnt >= TRIP) {
#pragma unroll
        for (int q = 0; q < TRIP / 8; ++q) pk[q] = *reinterpret_cast<const uint4 *>(pos + 8 * q);
    }
    for (; e + TRIP <= cnt; e += TRIP) {
        uint32_t r[TRIP];
#pragma unroll
        for (int q = 0; q < TRIP / 8; ++q) {
            const uint32_t l[8] = {pk[q].x & 0xFFFFu, pk[q].x >> 16, pk[q].y & 0xFFFFu,
                                   pk[q].y >> 16,     pk[q].z & 0xFFFFu, pk[q].z >> 16,
                                   pk[q].w & 0xFFFFu, pk[q].w >> 16};
#pragma unroll
            for (int u = 0; u < 8; ++u) r[8 * q + u] = b0[l[u]];
        }
        if (e + 2 * TRIP <= cnt) {
#pragma unroll
            for (int q = 0; q < TRIP / 8; ++q)
                pk[q] = *reinterpret_cast<const uint4 *>(pos + e + TRIP + 8 * q);
        }
#pragma unroll
        for (int u = 0; u < TRIP; ++u) acc ^= r[u];
    }
    for (; e < cnt; ++e) acc ^= b0[pos[e]];
    jwin[c * JWIN + t] = acc;   // [0] = x[624 S c - 1], [1 + k] = x[624 S c + k]
}

// MODE 0: random.random() doubles, two words each (genrand_res53); MODE 1: torch's CPU
// randint over [0, range) for range < 2^28 (aten uniform_int_from_to_distribution takes ONE
// 32-bit output, `random() % range`), one word each, int64 out; MODE 2: the same for
// 2^28 <= range < 2^32, where it takes random64() = (first output << 32 | second) % range (the
// threshold measured against torch 2.10's CPU generator, tests/test_host.py). index_dev != 0:
// the index is
// mt_in[624] (a state held in HBM, e.g. inside a captured graph) and the grid covers the worst
// case; blocks past the last window return.
template <int MODE>
__global__ void __launch_bounds__(MT_THREADS)
    k_mt_chains(const uint32_t *__restrict__ mt_in, int32_t index_arg, int32_t index_dev,
                int64_t n, void *__restrict__ out_v, uint64_t range,
                uint32_t *__restrict__ state_out, int64_t S, const uint32_t *__restrict__ jwin) {
    __shared__ uint32_t win[2][MT_N];
    __shared__ uint32_t carry;   // x[624 w0 - 1]: the first word of a double straddling chains
    constexpr int WPD = MODE == 1 ? 1 : 2;   // words per draw
    const int32_t index = index_dev ? static_cast<int32_t>(mt_in[MT_N]) : index_arg;
    const int64_t n_windows = n > 0 ? (index + WPD * n - 1) / MT_N + 1 : 1;
    const int t = threadIdx.x;
    const int64_t c = blockIdx.x;
    const int64_t w0 = c * S;
    if (w0 >= n_windows) return;   // (block-uniform: a device index sized the grid for 624)
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
        const uint32_t *jw = jwin + c * JWIN;
        for (int k = t; k < MT_N; k += MT_THREADS) win[0][k] = jw[k + 1];
        if (t == 0) carry = jw[0];
    }
    __syncthreads();
    const int64_t first = index, last = index + WPD * n - 1;   // the stream's absolute words
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
        const int64_t p0 = static_cast<int64_t>(MT_N) * w;
        if constexpr (MODE != 1) {
            // draws whose second word a2 lies in this window: (a2 - index) odd
            const int par = static_cast<int>((p0 - first + 1) & 1);
            if (t < MT_N / 2) {
                const int64_t a2 = p0 + 2 * t + par;
                if (a2 > first && a2 <= last) {
                    const int o2 = static_cast<int>(a2 - p0);
                    const uint32_t x2 = win[cur][o2];
                    const uint32_t x1 = o2 > 0 ? win[cur][o2 - 1]
                                               : (w == w0 ? carry : win[cur ^ 1][MT_N - 1]);
                    if constexpr (MODE == 0) {
                        static_cast<double *>(out_v)[(a2 - first) >> 1] = res53(x1, x2);
                    } else {
                        const uint64_t r = (static_cast<uint64_t>(temper(x1)) << 32) | temper(x2);
                        static_cast<int64_t *>(out_v)[(a2 - first) >> 1] =
                            static_cast<int64_t>(r % range);
                    }
                }
            }
        } else {   // one draw per word of the window
            int64_t *out = static_cast<int64_t *>(out_v);
            for (int o = t; o < MT_N; o += MT_THREADS) {
                const int64_t a = p0 + o;
                if (a >= first && a <= last)
                    out[a - first] = static_cast<int64_t>(temper(win[cur][o]) % range);
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

}  // extern "C"

namespace {
// index >= 0: the index (the host knows it); < 0: mt[624] on the device.
int mt_generate(int32_t mode, const uint32_t *mt, int32_t index, int64_t n, void *out,
                uint64_t range, uint32_t *state_out, int64_t window_stride,
                const uint16_t *jump_pos, const int64_t *jump_off, int64_t n_chains_table,
                uint32_t *workspace, int64_t workspace_words, hipStream_t st, const char *what) {
    DW_REQUIRE(mode >= 0 && mode <= 2, "%s: mode must be 0, 1 or 2", what);
    DW_REQUIRE(index <= MT_N, "%s: index must be in [0, 624]", what);
    DW_REQUIRE(n >= 0 && n <= (int64_t(1) << 40), "%s: n must be in [0, 2^40]", what);
    DW_REQUIRE(window_stride >= 1, "%s: window_stride must be >= 1", what);
    DW_REQUIRE(mode == 0 || (mode == 1 && range >= 1 && range < (uint64_t(1) << 28)) ||
                   (mode == 2 && range >= (uint64_t(1) << 28) && range < (uint64_t(1) << 32)),
               "%s: randint range must be in [1, 2^28) (mode 1) or [2^28, 2^32) (mode 2)", what);
    DW_REQUIRE(mt && state_out && (out || n == 0), "%s: null pointer", what);
    const int wpd = mode == 1 ? 1 : 2;
    int64_t n_windows = 1, chains = 1;
    if (n > 0) {   // (a device index: sized for the largest, 624)
        n_windows = ((index >= 0 ? index : MT_N) + wpd * n - 1) / MT_N + 1;
        chains = (n_windows + window_stride - 1) / window_stride;
    }
    DW_REQUIRE(chains == 1 || (jump_pos && jump_off && chains <= n_chains_table),
               "%s: %lld chains of %lld windows need a jump table of that many chains "
               "(dw_mt_jump_table), have %lld", what, static_cast<long long>(chains),
               static_cast<long long>(window_stride), static_cast<long long>(n_chains_table));
    DW_REQUIRE(chains == 1 || (workspace && workspace_words >= chains * JWIN),
               "%s: the workspace needs %lld words (dw_mt_workspace_words)", what,
               static_cast<long long>(chains * JWIN));
    DW_REQUIRE(chains < (int64_t(1) << 31), "%s: too many chains", what);
    if (chains > 1) {
        hipLaunchKernelGGL(k_mt_jump, dim3(static_cast<unsigned>(chains - 1)), dim3(JUMP_THREADS),
                           0, st, mt, jump_pos, jump_off, workspace);
        DW_LAUNCH_CHECK("dw_mt/jump");
    }
    const int32_t idx_dev = index < 0 ? 1 : 0;
    const dim3 g(static_cast<unsigned>(chains)), bl(MT_THREADS);
    if (mode == 0)
        hipLaunchKernelGGL(k_mt_chains<0>, g, bl, 0, st, mt, index, idx_dev, n, out, range,
                           state_out, window_stride, workspace);
    else if (mode == 1)
        hipLaunchKernelGGL(k_mt_chains<1>, g, bl, 0, st, mt, index, idx_dev, n, out, range,
                           state_out, window_stride, workspace);
    else
        hipLaunchKernelGGL(k_mt_chains<2>, g, bl, 0, st, mt, index, idx_dev, n, out, range,
                           state_out, window_stride, workspace);
    DW_LAUNCH_CHECK("dw_mt/chains");
    return DW_OK;
}
}  // namespace

extern "C" {

int dw_mt_uniforms(const uint32_t *mt, int32_t index, int64_t n, double *out,
                   uint32_t *state_out, int64_t window_stride, const uint16_t *jump_pos,
                   const int64_t *jump_off, int64_t n_chains_table, uint32_t *workspace,
                   int64_t workspace_words, void *stream) {
    DW_REQUIRE(index >= 0, "dw_mt_uniforms: index must be in [0, 624]");
    return mt_generate(0, mt, index, n, out, 0, state_out, window_stride, jump_pos, jump_off,
                       n_chains_table, workspace, workspace_words, dw::as_stream(stream),
                       "dw_mt_uniforms");
}

int dw_mt_draw(int32_t mode, uint32_t *state, int32_t index, int64_t n, void *out,
               uint64_t range, uint32_t *scratch, int64_t window_stride,
               const uint16_t *jump_pos, const int64_t *jump_off, int64_t n_chains_table,
               uint32_t *workspace, int64_t workspace_words, void *stream) {
    DW_REQUIRE(state && scratch && state != scratch, "dw_mt_draw: state / scratch");
    hipStream_t st = dw::as_stream(stream);
    const int rc = mt_generate(mode, state, index < 0 ? -1 : index, n, out, range, scratch,
                               window_stride, jump_pos, jump_off, n_chains_table, workspace,
                               workspace_words, st, "dw_mt_draw");
    if (rc != DW_OK) return rc;
    // the state after the draws back into place (625 words; stream-ordered, capturable)
    const hipError_t e = hipMemcpyAsync(state, scratch, (MT_N + 1) * sizeof(uint32_t),
                                        hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) {
        dw::set_error("dw_mt_draw: state copy: %s", hipGetErrorString(e));
        return DW_E_HIP;
    }
    return DW_OK;
}

int64_t dw_mt_workspace_words(int64_t n_chains) { return n_chains * JWIN; }

}  // extern "C"
