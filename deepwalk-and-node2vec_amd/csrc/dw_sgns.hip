// Skip-gram negative sampling on gfx950 (hot path B).
//
// Reference chain for one batch:
//   W2VCollateFunctional.__call__   torch_dataset.py:293-322  (centre, 2R contexts, left|right)
//   generate_noise_batch            utils/sampling.py:7-21     (uniform [0, V), shape (B', 2R, K))
//   SkipGram.forward x2             model.py:79-91             (gather + bmm logits)
//   NegativeSamplingLoss            loss.py:14-22              (-log clamp(sigmoid, 1e-6))
//   autograd backward               embedding_dense_backward into dense (V, d) grads
//
// Pass 1, k_sgns: one wave per centre. Lane l holds elements l, l+64, ... of every row (each
// row load is one 256-byte contiguous wave-instruction per 64 elements). Per centre: the centre
// row, then its T = 2R(1+K) output rows (contexts, then each context's K negatives) in chunks of
// CHUNK independent loads; logits by a batched wave butterfly; the clamp mask and 1/M scale give
// the closed-form gradient coefficient of every row. The centre's own gradient is summed in
// registers and leaves as ONE atomic row per centre. For the output table there are two modes:
//   * atomic: g_out[row] += coef * centre, float atomics (1.3 TB/s chip-wide ceiling on MI355X;
//     the output-table scatter is ~90% of the SGNS bytes, so this mode is atomic-bound);
//   * records (workspace given): each output row's coefficient is written as a 12-byte record
//     {row, centre, coef} (coalesced), the records are radix-sorted by row (hipcub, stable), and
//     pass 2 (k_rec_gather) gathers the centre rows and sums every output row's records in
//     registers. No float atomics except where a row straddles two fixed-size chunks; the
//     gathered bytes move at read speed, not atomic speed.
#include <hipcub/hipcub.hpp>

#include "dw_common.h"

namespace {

constexpr int WAVE = 64;
constexpr int WAVES_PER_BLOCK = 4;
constexpr int CHUNK = 6;
constexpr int TMAX = 256;            // max output rows per centre in records mode
constexpr int GCH = 512;             // records per pass-2 wave chunk
constexpr int GU = 8;                // records in flight per pass-2 iteration
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
    uint32_t *rec_key;        // records mode: [batch * T]
    uint64_t *rec_val;        //   {coef bits << 32 | centre id}
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

__device__ __forceinline__ uint64_t pack_record(float coef, int64_t centre) {
    return (static_cast<uint64_t>(__float_as_uint(coef)) << 32) |
           static_cast<uint32_t>(centre);
}

// VPL = values per lane (d <= 64*VPL); MASKED when d is not exactly 64*VPL.
template <int VPL, bool MASKED, bool FROM_WALKS, bool RECORDS>
__global__ void __launch_bounds__(WAVES_PER_BLOCK *WAVE) k_sgns(SgnsArgs a) {
    __shared__ uint32_t s_key[RECORDS ? WAVES_PER_BLOCK : 1][RECORDS ? TMAX : 1];
    __shared__ uint64_t s_val[RECORDS ? WAVES_PER_BLOCK : 1][RECORDS ? TMAX : 1];
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
        const bool centre_ok = cid >= 0 && cid < a.V;
        if (!centre_ok) {
            if (lane == 0) dw::status_or(a.status, DW_S_BAD_INDEX);
            if (RECORDS) {  // keep the record array well-formed: zero-coefficient records
                for (int t = lane; t < n_rows; t += WAVE) {
                    a.rec_key[b * n_rows + t] = 0u;
                    a.rec_val[b * n_rows + t] = 0ull;
                }
            }
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
                        if (RECORDS && lane == 0) {
                            s_key[wv][r] = 0u;
                            s_val[wv][r] = 0ull;
                        }
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
#pragma unroll
                for (int m = 0; m < VPL; ++m) gc[m] += gscal * o[u][m];
                if (RECORDS) {
                    if (lane == 0) {
                        s_key[wv][r0 + u] = static_cast<uint32_t>(id[u]);
                        s_val[wv][r0 + u] = pack_record(gscal, cid);
                    }
                } else if (gscal != 0.f) {
                    float *grow = a.g_out + id[u] * a.d + lane;
#pragma unroll
                    for (int m = 0; m < VPL; ++m)
                        if (live[m]) atomicAdd(grow + WAVE * m, gscal * c[m]);
                }
            }
        }
        if (RECORDS) {  // one coalesced record store per centre
            dw::wave_lds_sync();
            for (int t = lane; t < n_rows; t += WAVE) {
                a.rec_key[b * n_rows + t] = s_key[wv][t];
                a.rec_val[b * n_rows + t] = s_val[wv][t];
            }
            dw::wave_lds_sync();
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

// Pass 2: records sorted by output row -> g_out[row] += sum coef * w_in[centre].
// Each wave owns a fixed chunk of GCH sorted records (balanced whatever the row lengths —
// hub rows hold thousands). A row wholly inside the chunk is summed in registers and added
// with a plain read-modify-write (the chunk is its only writer); the first / last row of a
// chunk may continue in the neighbouring chunk and is added with float atomics.
template <int VPL, bool MASKED>
__global__ void __launch_bounds__(WAVES_PER_BLOCK *WAVE)
    k_rec_gather(const uint32_t *__restrict__ keys, const uint64_t *__restrict__ vals,
                 int64_t n_rec, const float *__restrict__ w_in, float *__restrict__ g_out,
                 int32_t d) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
    const int64_t n_chunks = (n_rec + GCH - 1) / GCH;
    const int64_t n_waves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
    bool live[VPL];
#pragma unroll
    for (int m = 0; m < VPL; ++m) live[m] = !MASKED || (lane + WAVE * m < d);

    for (int64_t ch = (int64_t)blockIdx.x * WAVES_PER_BLOCK + wv; ch < n_chunks; ch += n_waves) {
        const int64_t e0 = ch * GCH;
        const int64_t e1 = (e0 + GCH < n_rec) ? e0 + GCH : n_rec;
        const uint32_t before = e0 > 0 ? keys[e0 - 1] : 0xFFFFFFFFu;
        const uint32_t after = e1 < n_rec ? keys[e1] : 0xFFFFFFFFu;
        uint32_t cur = keys[e0];
        float g[VPL];
#pragma unroll
        for (int m = 0; m < VPL; ++m) g[m] = 0.f;

        auto flush = [&](uint32_t row) {
            float *dst = g_out + static_cast<int64_t>(row) * d + lane;
            if (row != before && row != after) {
#pragma unroll
                for (int m = 0; m < VPL; ++m)
                    if (live[m]) dst[WAVE * m] += g[m];
            } else {
#pragma unroll
                for (int m = 0; m < VPL; ++m)
                    if (live[m]) atomicAdd(dst + WAVE * m, g[m]);
            }
        };

        for (int64_t e = e0; e < e1; e += GU) {
            uint32_t k[GU];
            float coef[GU];
            float x[GU][VPL];
#pragma unroll
            for (int u = 0; u < GU; ++u) {
                const bool in = e + u < e1;
                const uint64_t v = in ? vals[e + u] : 0ull;
                k[u] = in ? keys[e + u] : cur;
                coef[u] = in ? __uint_as_float(static_cast<uint32_t>(v >> 32)) : 0.f;
                const float *src = w_in + static_cast<int64_t>(static_cast<uint32_t>(v)) * d + lane;
#pragma unroll
                for (int m = 0; m < VPL; ++m) x[u][m] = (in && live[m]) ? src[WAVE * m] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < GU; ++u) {
                if (k[u] != cur) {
                    flush(cur);
                    cur = k[u];
#pragma unroll
                    for (int m = 0; m < VPL; ++m) g[m] = 0.f;
                }
#pragma unroll
                for (int m = 0; m < VPL; ++m) g[m] += coef[u] * x[u][m];
            }
        }
        flush(cur);
    }
}

int end_bit_for(int64_t V) {
    int bits = 1;
    while (bits < 32 && (static_cast<uint64_t>(V - 1) >> bits) != 0) ++bits;
    return bits;
}

struct Workspace {
    uint32_t *k0, *k1;
    uint64_t *v0, *v1;
    void *cub;
    size_t cub_bytes;
    size_t total;
};

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

int plan_workspace(int64_t n_rec, int64_t V, void *base, Workspace *ws, hipStream_t st) {
    size_t cub_bytes = 0;
    hipcub::DoubleBuffer<uint32_t> kb(nullptr, nullptr);
    hipcub::DoubleBuffer<uint64_t> vb(nullptr, nullptr);
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, cub_bytes, kb, vb, (int)n_rec, 0,
                                                      end_bit_for(V), st);
    if (e != hipSuccess) {
        dw::set_error("dw_sgns: hipcub size query failed: %s", hipGetErrorString(e));
        return DW_E_HIP;
    }
    const size_t kbytes = align256((size_t)n_rec * 4), vbytes = align256((size_t)n_rec * 8);
    char *p = static_cast<char *>(base);
    ws->k0 = reinterpret_cast<uint32_t *>(p);
    ws->k1 = reinterpret_cast<uint32_t *>(p + kbytes);
    ws->v0 = reinterpret_cast<uint64_t *>(p + 2 * kbytes);
    ws->v1 = reinterpret_cast<uint64_t *>(p + 2 * kbytes + vbytes);
    ws->cub = p + 2 * kbytes + 2 * vbytes;
    ws->cub_bytes = cub_bytes;
    ws->total = 2 * kbytes + 2 * vbytes + align256(cub_bytes);
    return DW_OK;
}

template <bool FROM_WALKS, bool RECORDS>
int launch_pass1(const SgnsArgs &a, hipStream_t st) {
    int64_t blocks = (a.batch + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
    if (blocks > 65536) blocks = 65536;
    const dim3 g((unsigned)blocks), bl(WAVES_PER_BLOCK * WAVE);
#define DW_SGNS_CASE(VPL)                                                                    \
    if (a.d <= 64 * VPL) {                                                                    \
        if (a.d == 64 * VPL)                                                                  \
            hipLaunchKernelGGL((k_sgns<VPL, false, FROM_WALKS, RECORDS>), g, bl, 0, st, a);  \
        else                                                                                  \
            hipLaunchKernelGGL((k_sgns<VPL, true, FROM_WALKS, RECORDS>), g, bl, 0, st, a);   \
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

int launch_pass2(const uint32_t *keys, const uint64_t *vals, int64_t n_rec, const float *w_in,
                 float *g_out, int32_t d, hipStream_t st) {
    const int64_t n_chunks = (n_rec + GCH - 1) / GCH;
    int64_t blocks = (n_chunks + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
    if (blocks < 1) blocks = 1;
    if (blocks > 65536) blocks = 65536;
    const dim3 g((unsigned)blocks), bl(WAVES_PER_BLOCK * WAVE);
#define DW_GATHER_CASE(VPL)                                                                      \
    if (d <= 64 * VPL) {                                                                          \
        if (d == 64 * VPL)                                                                        \
            hipLaunchKernelGGL((k_rec_gather<VPL, false>), g, bl, 0, st, keys, vals, n_rec, w_in, \
                               g_out, d);                                                         \
        else                                                                                      \
            hipLaunchKernelGGL((k_rec_gather<VPL, true>), g, bl, 0, st, keys, vals, n_rec, w_in,  \
                               g_out, d);                                                         \
        DW_LAUNCH_CHECK("dw_sgns/gather");                                                        \
        return DW_OK;                                                                             \
    }
    DW_GATHER_CASE(1)
    DW_GATHER_CASE(2)
    DW_GATHER_CASE(4)
    DW_GATHER_CASE(8)
#undef DW_GATHER_CASE
    return DW_E_UNSUPPORTED;
}

template <bool FROM_WALKS>
int launch_sgns(SgnsArgs a, void *workspace, size_t workspace_bytes, hipStream_t st) {
    if (a.batch == 0) return DW_OK;
    const int64_t T = (int64_t)a.C * (1 + a.K);
    if (workspace == nullptr) return launch_pass1<FROM_WALKS, false>(a, st);
    DW_REQUIRE(T <= TMAX, "dw_sgns: records mode needs 2R(1+K) <= %d (got %lld)", TMAX,
               (long long)T);
    DW_REQUIRE(a.V <= 0x7FFFFFFF, "dw_sgns: records mode needs vocab_size < 2^31");
    const int64_t n_rec = a.batch * T;
    DW_REQUIRE(n_rec < 0x7FFFFFFF, "dw_sgns: records mode needs batch*2R(1+K) < 2^31");
    Workspace ws;
    int rc = plan_workspace(n_rec, a.V, workspace, &ws, st);
    if (rc != DW_OK) return rc;
    DW_REQUIRE(workspace_bytes >= ws.total, "dw_sgns: workspace too small (%zu < %zu)",
               workspace_bytes, ws.total);
    a.rec_key = ws.k0;
    a.rec_val = ws.v0;
    rc = launch_pass1<FROM_WALKS, true>(a, st);
    if (rc != DW_OK) return rc;
    hipcub::DoubleBuffer<uint32_t> kb(ws.k0, ws.k1);
    hipcub::DoubleBuffer<uint64_t> vb(ws.v0, ws.v1);
    size_t cub_bytes = ws.cub_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(ws.cub, cub_bytes, kb, vb, (int)n_rec, 0,
                                                      end_bit_for(a.V), st);
    if (e != hipSuccess) {
        dw::set_error("dw_sgns: hipcub sort failed: %s", hipGetErrorString(e));
        return DW_E_HIP;
    }
    return launch_pass2(kb.Current(), vb.Current(), n_rec, a.w_in, a.g_out, a.d, st);
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

SgnsArgs base_args(int64_t V, int32_t dim, int32_t K, const float *w_in, const float *w_out,
                   float *g_in, float *g_out, const int64_t *noise, uint64_t seed,
                   uint64_t noise_offset, float grad_scale, double *loss_acc, int32_t *status) {
    SgnsArgs a{};
    a.K = K;
    a.V = V;
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
    return a;
}

}  // namespace

extern "C" {

int dw_sgns_workspace_bytes(int64_t n_centres, int32_t n_ctx, int32_t neg_samples,
                            int64_t vocab_size, size_t *bytes) {
    DW_REQUIRE(bytes, "dw_sgns_workspace_bytes: bytes is null");
    DW_REQUIRE(n_centres >= 0 && n_ctx >= 1 && neg_samples >= 0 && vocab_size >= 1,
               "dw_sgns_workspace_bytes: bad sizes");
    const int64_t n_rec = n_centres * n_ctx * (1 + (int64_t)neg_samples);
    DW_REQUIRE(n_rec < 0x7FFFFFFF, "dw_sgns_workspace_bytes: too many records");
    Workspace ws;
    char dummy;
    int rc = plan_workspace(n_rec > 0 ? n_rec : 1, vocab_size, &dummy, &ws, nullptr);
    if (rc != DW_OK) return rc;
    *bytes = ws.total;
    return DW_OK;
}

int dw_sgns_walks(const int32_t *walks, int64_t n_walks, int32_t walk_length,
                  int32_t context_radius, int32_t neg_samples, int64_t vocab_size, int32_t dim,
                  const float *w_in, const float *w_out, float *g_in, float *g_out,
                  const int64_t *noise, uint64_t seed, uint64_t noise_offset, float grad_scale,
                  double *loss_acc, int32_t *status, void *workspace, size_t workspace_bytes,
                  void *stream) {
    DW_REQUIRE(context_radius >= 1, "dw_sgns_walks: context_radius must be >= 1");
    DW_REQUIRE(walk_length >= 2 * context_radius + 1,
               "dw_sgns_walks: walk_length %d < 2R+1 (Text is too short!)", walk_length);
    DW_REQUIRE(neg_samples >= 0 && dim >= 1 && vocab_size >= 1 && n_walks >= 0,
               "dw_sgns_walks: bad sizes");
    DW_REQUIRE(walks && w_in && w_out && g_in && g_out && status, "dw_sgns_walks: null pointer");
    SgnsArgs a = base_args(vocab_size, dim, neg_samples, w_in, w_out, g_in, g_out, noise, seed,
                           noise_offset, grad_scale, loss_acc, status);
    a.walks = walks;
    a.L = walk_length;
    a.R = context_radius;
    a.batch = n_walks * (walk_length - 2 * context_radius);
    a.C = 2 * context_radius;
    return launch_sgns<true>(a, workspace, workspace_bytes, dw::as_stream(stream));
}

int dw_sgns_pairs(const int64_t *inputs, const int64_t *targets, int64_t batch, int32_t n_ctx,
                  int32_t neg_samples, int64_t vocab_size, int32_t dim,
                  const float *w_in, const float *w_out, float *g_in, float *g_out,
                  const int64_t *noise, uint64_t seed, uint64_t noise_offset, float grad_scale,
                  double *loss_acc, int32_t *status, void *workspace, size_t workspace_bytes,
                  void *stream) {
    DW_REQUIRE(n_ctx >= 1 && neg_samples >= 0 && dim >= 1 && vocab_size >= 1 && batch >= 0,
               "dw_sgns_pairs: bad sizes");
    DW_REQUIRE(inputs && targets && w_in && w_out && g_in && g_out && status,
               "dw_sgns_pairs: null pointer");
    SgnsArgs a = base_args(vocab_size, dim, neg_samples, w_in, w_out, g_in, g_out, noise, seed,
                           noise_offset, grad_scale, loss_acc, status);
    a.inputs = inputs;
    a.targets = targets;
    a.batch = batch;
    a.C = n_ctx;
    return launch_sgns<false>(a, workspace, workspace_bytes, dw::as_stream(stream));
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
