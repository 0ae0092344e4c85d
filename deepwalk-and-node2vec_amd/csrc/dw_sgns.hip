// Skip-gram negative sampling on gfx950 (hot path B).
//
// Reference chain for one batch:
//   W2VCollateFunctional.__call__   torch_dataset.py:293-322  (centre, 2R contexts, left|right)
//   generate_noise_batch            utils/sampling.py:7-21     (uniform [0, V), shape (B', 2R, K))
//   SkipGram.forward x2             model.py:79-91             (gather + bmm logits)
//   NegativeSamplingLoss            loss.py:14-22              (-log clamp(sigmoid, 1e-6))
//   autograd backward               embedding_dense_backward into dense (V, d) grads
//
// One wave per centre. Lane l holds elements l, l+64, ... of every row, so each row load and
// each float atomic is one 256-byte contiguous wave-instruction per 64 elements (the full-rate
// atomic shape on MI355X). Per centre: the centre row once, then the 2R(1+K) output rows in
// chunks of CHUNK independent loads; logits by wave butterfly; the clamp mask and 1/M scale
// give the closed-form gradient; output-row gradients go straight out as atomics, the centre's
// gradient is summed in registers and leaves as ONE atomic row per centre.
#include "dw_common.h"

namespace {

constexpr int WAVE = 64;
constexpr int WAVES_PER_BLOCK = 4;
constexpr int CHUNK = 4;
constexpr uint32_t TAG_SGNS = 0x53470000u;  // 'SG'

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + expf(-x)); }

struct SgnsArgs {
    // source of centres / contexts
    const int32_t *walks;     // walks mode
    int32_t L, R;
    const int64_t *inputs;    // pairs mode
    const int64_t *targets;
    int64_t batch;            // number of centres B'
    int32_t C;                // contexts per centre
    int32_t K;
    int64_t V;
    int32_t d;
    const float *w_in, *w_out;
    float *g_in, *g_out;
    const int64_t *noise;
    uint32_t k0, k1;
    uint64_t noise_offset;
    float scale;
    double *loss_acc;
    int32_t *status;
};

template <bool FROM_WALKS>
__device__ __forceinline__ int64_t centre_id(const SgnsArgs &a, int64_t b) {
    if (FROM_WALKS) {
        const int64_t per = a.L - 2 * a.R;
        const int64_t w = b / per, i = a.R + (b - w * per);
        return a.walks[w * a.L + i];
    }
    return a.inputs[b];
}

template <bool FROM_WALKS>
__device__ __forceinline__ int64_t context_id(const SgnsArgs &a, int64_t b, int j) {
    if (FROM_WALKS) {
        const int64_t per = a.L - 2 * a.R;
        const int64_t w = b / per, i = a.R + (b - w * per);
        const int64_t pos = (j < a.R) ? (i - a.R + j) : (i + 1 + (j - a.R));
        return a.walks[w * a.L + pos];
    }
    return a.targets[b * a.C + j];
}

__device__ __forceinline__ int64_t noise_id(const SgnsArgs &a, int64_t b, int j, int k) {
    if (a.noise) return a.noise[(b * a.C + j) * a.K + k];
    const uint64_t g = a.noise_offset + static_cast<uint64_t>(b);
    const dw::U4 r = dw::philox(
        dw::U4{static_cast<uint32_t>(g), static_cast<uint32_t>(g >> 32),
               static_cast<uint32_t>(j * a.K + k), TAG_SGNS},
        a.k0, a.k1);
    return static_cast<int64_t>(dw::bounded64(r.x, r.y, static_cast<uint64_t>(a.V)));
}

// VPL = values per lane (d <= 64*VPL); MASKED when d is not exactly 64*VPL.
template <int VPL, bool MASKED, bool FROM_WALKS>
__global__ void __launch_bounds__(WAVES_PER_BLOCK *WAVE) k_sgns(SgnsArgs a) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int wv = threadIdx.x / WAVE;
    const int64_t n_waves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
    const int rows_per_ctx = 1 + a.K;
    const int n_rows = a.C * rows_per_ctx;

    bool live[VPL];
#pragma unroll
    for (int m = 0; m < VPL; ++m) live[m] = !MASKED || (lane + WAVE * m < a.d);

    float acc_pos = 0.f, acc_neg = 0.f, acc_rec = 0.f, acc_prec = 0.f;

    for (int64_t b = (int64_t)blockIdx.x * WAVES_PER_BLOCK + wv; b < a.batch; b += n_waves) {
        const int64_t cid = centre_id<FROM_WALKS>(a, b);
        if (cid < 0 || cid >= a.V) {
            if (lane == 0) dw::status_or(a.status, DW_S_BAD_INDEX);
            continue;
        }
        float c[VPL], gc[VPL];
        const float *crow = a.w_in + cid * a.d + lane;
#pragma unroll
        for (int m = 0; m < VPL; ++m) {
            c[m] = live[m] ? crow[WAVE * m] : 0.f;
            gc[m] = 0.f;
        }
        for (int r0 = 0; r0 < n_rows; r0 += CHUNK) {
            int64_t id[CHUNK];
            bool pos[CHUNK], ok[CHUNK];
            float o[CHUNK][VPL], dot[CHUNK];
#pragma unroll
            for (int u = 0; u < CHUNK; ++u) {
                const int r = r0 + u;
                ok[u] = r < n_rows;
                pos[u] = false;
                id[u] = 0;
                if (ok[u]) {
                    const int j = r / rows_per_ctx, k = r - j * rows_per_ctx - 1;
                    pos[u] = k < 0;
                    id[u] = pos[u] ? context_id<FROM_WALKS>(a, b, j) : noise_id(a, b, j, k);
                    if (id[u] < 0 || id[u] >= a.V) {
                        if (lane == 0) dw::status_or(a.status, DW_S_BAD_INDEX);
                        ok[u] = false;
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < CHUNK; ++u) {
                const float *row = a.w_out + (ok[u] ? id[u] : 0) * a.d + lane;
#pragma unroll
                for (int m = 0; m < VPL; ++m) o[u][m] = (ok[u] && live[m]) ? row[WAVE * m] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < CHUNK; ++u) {
                float s = 0.f;
#pragma unroll
                for (int m = 0; m < VPL; ++m) s += c[m] * o[u][m];
                dot[u] = s;
            }
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
                for (int u = 0; u < CHUNK; ++u) dot[u] += __shfl_xor(dot[u], off, WAVE);
            }
#pragma unroll
            for (int u = 0; u < CHUNK; ++u) {
                if (!ok[u]) continue;
                float gscal;
                if (pos[u]) {
                    // -log(clamp(sigmoid(s), 1e-6)); d/ds = sigmoid(s) - 1 where unclamped
                    const float sg = sigmoidf(dot[u]);
                    acc_pos += -logf(fmaxf(sg, 1e-6f));
                    acc_rec += (sg >= 0.5f) ? 1.f : 0.f;
                    gscal = (sg >= 1e-6f) ? (sg - 1.0f) * a.scale : 0.f;
                } else {
                    // -log(clamp(sigmoid(-t), 1e-6)); d/dt = 1 - sigmoid(-t) where unclamped
                    const float sn = sigmoidf(-dot[u]);
                    acc_neg += -logf(fmaxf(sn, 1e-6f));
                    acc_prec += (sigmoidf(dot[u]) >= 0.5f) ? 1.f : 0.f;
                    gscal = (sn >= 1e-6f) ? (1.0f - sn) * a.scale : 0.f;
                }
                if (gscal != 0.f) {
                    float *grow = a.g_out + id[u] * a.d + lane;
#pragma unroll
                    for (int m = 0; m < VPL; ++m) {
                        if (live[m]) {
                            gc[m] += gscal * o[u][m];
                            atomicAdd(grow + WAVE * m, gscal * c[m]);
                        }
                    }
                }
            }
        }
        float *gcrow = a.g_in + cid * a.d + lane;
#pragma unroll
        for (int m = 0; m < VPL; ++m)
            if (live[m]) atomicAdd(gcrow + WAVE * m, gc[m]);
    }

    // loss partials: the four scalars are wave-uniform; one double atomic per wave and value
    if (a.loss_acc && lane == 0) {
        if (acc_pos != 0.f) atomicAdd(a.loss_acc + 0, (double)acc_pos);
        if (acc_neg != 0.f) atomicAdd(a.loss_acc + 1, (double)acc_neg);
        if (acc_rec != 0.f) atomicAdd(a.loss_acc + 2, (double)acc_rec);
        if (acc_prec != 0.f) atomicAdd(a.loss_acc + 3, (double)acc_prec);
    }
}

template <bool FROM_WALKS>
int launch_sgns(const SgnsArgs &a, hipStream_t st) {
    if (a.batch == 0) return DW_OK;
    int64_t blocks = (a.batch + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
    if (blocks > 65536) blocks = 65536;
    const dim3 g((unsigned)blocks), bl(WAVES_PER_BLOCK * WAVE);
#define DW_SGNS_CASE(VPL)                                                                    \
    if (a.d <= 64 * VPL) {                                                                    \
        if (a.d == 64 * VPL)                                                                  \
            hipLaunchKernelGGL((k_sgns<VPL, false, FROM_WALKS>), g, bl, 0, st, a);           \
        else                                                                                  \
            hipLaunchKernelGGL((k_sgns<VPL, true, FROM_WALKS>), g, bl, 0, st, a);            \
        DW_LAUNCH_CHECK("dw_sgns");                                                           \
        return DW_OK;                                                                         \
    }
    DW_SGNS_CASE(1)
    DW_SGNS_CASE(2)
    DW_SGNS_CASE(4)
    DW_SGNS_CASE(8)
#undef DW_SGNS_CASE
    dw::set_error("dw_sgns: dim %d > 512 is not supported", a.d);
    return DW_E_UNSUPPORTED;
}

// ---- SkipGram.forward logits and its backward (autograd path of the reference API) ----------
__global__ void __launch_bounds__(256)
    k_logits(const int64_t *__restrict__ inputs, const int64_t *__restrict__ outputs, int64_t B,
             int32_t N, int64_t V, int32_t d, const float *__restrict__ w_in,
             const float *__restrict__ w_out, int32_t proba, float *__restrict__ logits,
             int32_t *status) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t n_waves = (int64_t)gridDim.x * (blockDim.x / WAVE);
    for (int64_t b = blockIdx.x * (int64_t)(blockDim.x / WAVE) + threadIdx.x / WAVE; b < B;
         b += n_waves) {
        const int64_t c = inputs[b];
        for (int n = 0; n < N; ++n) {
            const int64_t o = outputs[b * N + n];
            float s = 0.f;
            const bool ok = c >= 0 && c < V && o >= 0 && o < V;
            if (ok)
                for (int e = lane; e < d; e += WAVE) s += w_in[c * d + e] * w_out[o * d + e];
            s = dw::wave_sum(s);
            if (lane == 0) {
                if (!ok) dw::status_or(status, DW_S_BAD_INDEX);
                logits[b * N + n] = proba ? sigmoidf(s) : s;
            }
        }
    }
}

__global__ void __launch_bounds__(256)
    k_logits_bwd(const int64_t *__restrict__ inputs, const int64_t *__restrict__ outputs,
                 int64_t B, int32_t N, int64_t V, int32_t d, const float *__restrict__ w_in,
                 const float *__restrict__ w_out, const float *__restrict__ dl,
                 float *__restrict__ g_in, float *__restrict__ g_out, int32_t *status) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t n_waves = (int64_t)gridDim.x * (blockDim.x / WAVE);
    for (int64_t b = blockIdx.x * (int64_t)(blockDim.x / WAVE) + threadIdx.x / WAVE; b < B;
         b += n_waves) {
        const int64_t c = inputs[b];
        if (c < 0 || c >= V) {
            if (lane == 0) dw::status_or(status, DW_S_BAD_INDEX);
            continue;
        }
        for (int e0 = 0; e0 < d; e0 += WAVE) {
            const int e = e0 + lane;
            float gc = 0.f;
            const float ce = e < d ? w_in[c * d + e] : 0.f;
            for (int n = 0; n < N; ++n) {
                const int64_t o = outputs[b * N + n];
                if (o < 0 || o >= V) continue;
                const float g = dl[b * N + n];
                if (e < d) {
                    gc += g * w_out[o * d + e];
                    atomicAdd(g_out + o * d + e, g * ce);
                }
            }
            if (e < d) atomicAdd(g_in + c * d + e, gc);
        }
    }
}

}  // namespace

extern "C" {

int dw_sgns_walks(const int32_t *walks, int64_t n_walks, int32_t walk_length,
                  int32_t context_radius, int32_t neg_samples, int64_t vocab_size, int32_t dim,
                  const float *w_in, const float *w_out, float *g_in, float *g_out,
                  const int64_t *noise, uint64_t seed, uint64_t noise_offset, float grad_scale,
                  double *loss_acc, int32_t *status, void *stream) {
    DW_REQUIRE(context_radius >= 1, "dw_sgns_walks: context_radius must be >= 1");
    DW_REQUIRE(walk_length >= 2 * context_radius + 1,
               "dw_sgns_walks: walk_length %d < 2R+1 (Text is too short!)", walk_length);
    DW_REQUIRE(neg_samples >= 0 && dim >= 1 && vocab_size >= 1 && n_walks >= 0,
               "dw_sgns_walks: bad sizes");
    DW_REQUIRE(walks && w_in && w_out && g_in && g_out && status, "dw_sgns_walks: null pointer");
    SgnsArgs a{};
    a.walks = walks;
    a.L = walk_length;
    a.R = context_radius;
    a.batch = n_walks * (walk_length - 2 * context_radius);
    a.C = 2 * context_radius;
    a.K = neg_samples;
    a.V = vocab_size;
    a.d = dim;
    a.w_in = w_in;
    a.w_out = w_out;
    a.g_in = g_in;
    a.g_out = g_out;
    a.noise = noise;
    a.k0 = static_cast<uint32_t>(seed);
    a.k1 = static_cast<uint32_t>(seed >> 32);
    a.noise_offset = noise_offset;
    a.scale = grad_scale;
    a.loss_acc = loss_acc;
    a.status = status;
    return launch_sgns<true>(a, dw::as_stream(stream));
}

int dw_sgns_pairs(const int64_t *inputs, const int64_t *targets, int64_t batch, int32_t n_ctx,
                  int32_t neg_samples, int64_t vocab_size, int32_t dim,
                  const float *w_in, const float *w_out, float *g_in, float *g_out,
                  const int64_t *noise, uint64_t seed, uint64_t noise_offset, float grad_scale,
                  double *loss_acc, int32_t *status, void *stream) {
    DW_REQUIRE(n_ctx >= 1 && neg_samples >= 0 && dim >= 1 && vocab_size >= 1 && batch >= 0,
               "dw_sgns_pairs: bad sizes");
    DW_REQUIRE(inputs && targets && w_in && w_out && g_in && g_out && status,
               "dw_sgns_pairs: null pointer");
    SgnsArgs a{};
    a.inputs = inputs;
    a.targets = targets;
    a.batch = batch;
    a.C = n_ctx;
    a.K = neg_samples;
    a.V = vocab_size;
    a.d = dim;
    a.w_in = w_in;
    a.w_out = w_out;
    a.g_in = g_in;
    a.g_out = g_out;
    a.noise = noise;
    a.k0 = static_cast<uint32_t>(seed);
    a.k1 = static_cast<uint32_t>(seed >> 32);
    a.noise_offset = noise_offset;
    a.scale = grad_scale;
    a.loss_acc = loss_acc;
    a.status = status;
    return launch_sgns<false>(a, dw::as_stream(stream));
}

int dw_skipgram_logits(const int64_t *inputs, const int64_t *outputs, int64_t batch,
                       int32_t n_out, int64_t vocab_size, int32_t dim, const float *w_in,
                       const float *w_out, int32_t proba, float *logits, int32_t *status,
                       void *stream) {
    DW_REQUIRE(batch >= 0 && n_out >= 0 && dim >= 1, "dw_skipgram_logits: bad sizes");
    if (batch == 0 || n_out == 0) return DW_OK;
    DW_REQUIRE(inputs && outputs && w_in && w_out && logits && status,
               "dw_skipgram_logits: null pointer");
    int64_t blocks = (batch + 3) / 4;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_logits, dim3((unsigned)blocks), dim3(256), 0, dw::as_stream(stream),
                       inputs, outputs, batch, n_out, vocab_size, dim, w_in, w_out, proba, logits,
                       status);
    DW_LAUNCH_CHECK("dw_skipgram_logits");
    return DW_OK;
}

int dw_skipgram_logits_backward(const int64_t *inputs, const int64_t *outputs, int64_t batch,
                                int32_t n_out, int64_t vocab_size, int32_t dim,
                                const float *w_in, const float *w_out, const float *dlogits,
                                float *g_in, float *g_out, int32_t *status, void *stream) {
    DW_REQUIRE(batch >= 0 && n_out >= 0 && dim >= 1, "dw_skipgram_logits_backward: bad sizes");
    if (batch == 0 || n_out == 0) return DW_OK;
    DW_REQUIRE(inputs && outputs && w_in && w_out && dlogits && g_in && g_out && status,
               "dw_skipgram_logits_backward: null pointer");
    int64_t blocks = (batch + 3) / 4;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_logits_bwd, dim3((unsigned)blocks), dim3(256), 0, dw::as_stream(stream),
                       inputs, outputs, batch, n_out, vocab_size, dim, w_in, w_out, dlogits, g_in,
                       g_out, status);
    DW_LAUNCH_CHECK("dw_skipgram_logits_backward");
    return DW_OK;
}

}  // extern "C"
