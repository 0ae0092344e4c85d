// Dense Adam over the embedding tables (the dominant HBM stream of one reference step).
//
// Reference: the configs instantiate torch.optim.Adam (configs/sge_sg_*.yaml `_target_`,
// config_parser/core.py:43-53); PL calls optimizer.step() + zero_grad() every batch. The
// single-tensor update (torch/optim/adam.py, amsgrad=False) is restated with the per-step
// scalars precomputed on the host in float64 and cast to float32 exactly as torch's scalar
// arguments are:
//   m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, value=1-b2);
//   denom = (v.sqrt() / bias_correction2_sqrt).add_(eps); p.addcdiv_(m, denom, value=-step_size)
// Streaming: 16-B accesses; p, g, m, v read once, p, m, v (and g=0) written once.
#include <stdlib.h>

#include "dw_common.h"

namespace {

// Every byte is touched once per step, so loads and stores are non-temporal (they neither
// allocate in L2 / the Infinity Cache nor evict the embedding rows the next SGNS pass gathers),
// and each lane keeps U = 2 float4 groups of all four tensors in flight. Measured on MI355X,
// same box, C3 tables (2 x 1,048,577 x 128): 1.75 ms vs 2.02 ms for plain loads / stores with
// one group per lane (scripts/gpu_tune.sh, DW_ADAM_VARIANT sweep of round 1).
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld(const float4 *p, bool nt) {
    if (!nt) return *p;
    const f4v x = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(p));
    return make_float4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ void st(float4 *p, float4 v, bool nt) {
    if (!nt) {
        *p = v;
        return;
    }
    const f4v x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f4v *>(p));
}

template <bool ZERO, bool NT, int U, bool NTS = NT>
__global__ void __launch_bounds__(256)
    k_adam(const float *p, float *pd, float *__restrict__ g, float *__restrict__ m,
           float *__restrict__ v, int64_t n, dw::AdamScalars s0,
           const dw_step_scalars *__restrict__ dyn) {
    // p: parameters read; pd: parameters written (== p in place, or the other buffer of a
    // double-buffered table); dyn: the bound step block's scalars replace s0 (graph replay)
    const dw::AdamScalars s = dw::step_adam(dyn, s0);
    const int64_t n4 = n >> 2;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const float4 *p4 = reinterpret_cast<const float4 *>(p);
    float4 *pd4 = reinterpret_cast<float4 *>(pd);
    float4 *g4 = reinterpret_cast<float4 *>(g);
    float4 *m4 = reinterpret_cast<float4 *>(m);
    float4 *v4 = reinterpret_cast<float4 *>(v);
    for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i0 < n4;
         i0 += stride * U) {
        float4 pp[U], gg[U], mm[U], vv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * stride;
            if (i < n4) {
                pp[u] = ld(p4 + i, NT);
                gg[u] = ld(g4 + i, NT);
                mm[u] = ld(m4 + i, NT);
                vv[u] = ld(v4 + i, NT);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * stride;
            if (i < n4) {
                // g is re-zeroed only where its bits are not all +0: a sparse step's untouched
                // rows (most of the in table at C3) need no store — the same bits either way
                const bool dirty = (__float_as_uint(gg[u].x) | __float_as_uint(gg[u].y) |
                                    __float_as_uint(gg[u].z) | __float_as_uint(gg[u].w)) != 0u;
                dw::adam_elem(pp[u].x, gg[u].x, mm[u].x, vv[u].x, s);
                dw::adam_elem(pp[u].y, gg[u].y, mm[u].y, vv[u].y, s);
                dw::adam_elem(pp[u].z, gg[u].z, mm[u].z, vv[u].z, s);
                dw::adam_elem(pp[u].w, gg[u].w, mm[u].w, vv[u].w, s);
                st(pd4 + i, pp[u], NTS);
                st(m4 + i, mm[u], NTS);
                st(v4 + i, vv[u], NTS);
                if (ZERO && dirty) st(g4 + i, make_float4(0.f, 0.f, 0.f, 0.f), NTS);
            }
        }
    }
    for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += stride) {
        float pp = p[i];
        dw::adam_elem(pp, g[i], m[i], v[i], s);
        pd[i] = pp;
        if (ZERO) g[i] = 0.f;
    }
}

// k_adam with the gradient read from a deterministic-mode accumulator (DW_EXACT_ADAM): g =
// fl(acc * 2^-frac) (dw::from_fixed, the conversion pass's rule, so the same floats), acc cleared
// (ZERO) and the float buffer not touched. One streaming pass where the conversion after pass 1
// read and wrote every centre's row with atomics.
template <bool ZERO>
__global__ void __launch_bounds__(256)
    k_adam_fixed(const float *p, float *pd, long long *__restrict__ acc, float *__restrict__ m,
                 float *__restrict__ v, int64_t n, dw::AdamScalars s0, double fi,
                 const dw_step_scalars *__restrict__ dyn) {
    const dw::AdamScalars s = dw::step_adam(dyn, s0);
    const int64_t n4 = n >> 2;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const float4 *p4 = reinterpret_cast<const float4 *>(p);
    float4 *pd4 = reinterpret_cast<float4 *>(pd);
    longlong2 *a2 = reinterpret_cast<longlong2 *>(acc);
    float4 *m4 = reinterpret_cast<float4 *>(m);
    float4 *v4 = reinterpret_cast<float4 *>(v);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 pp = ld(p4 + i, true), mm = ld(m4 + i, true), vv = ld(v4 + i, true);
        const longlong2 a0 = a2[2 * i], a1 = a2[2 * i + 1];
        float g0 = dw::from_fixed(a0.x, fi), g1 = dw::from_fixed(a0.y, fi);
        float g2 = dw::from_fixed(a1.x, fi), g3 = dw::from_fixed(a1.y, fi);
        dw::adam_elem(pp.x, g0, mm.x, vv.x, s);
        dw::adam_elem(pp.y, g1, mm.y, vv.y, s);
        dw::adam_elem(pp.z, g2, mm.z, vv.z, s);
        dw::adam_elem(pp.w, g3, mm.w, vv.w, s);
        st(pd4 + i, pp, true);
        st(m4 + i, mm, true);
        st(v4 + i, vv, true);
        // (cleared only where a sum was left: most rows are no centre of the step, and their
        // zeros need no store — a third of the update's writes)
        if (ZERO && ((a0.x | a0.y | a1.x | a1.y) != 0)) {
            a2[2 * i] = make_longlong2(0, 0);
            a2[2 * i + 1] = make_longlong2(0, 0);
        }
    }
    for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += stride) {
        float pp = p[i], gg = dw::from_fixed(acc[i], fi);
        dw::adam_elem(pp, gg, m[i], v[i], s);
        pd[i] = pp;
        if (ZERO) acc[i] = 0;
    }
}

// ---- lazy exact Adam over selected rows (the touched-row in-table exchange, N > 1) ------------
// A row that no centre of a batch touched has g = 0 for that step, and torch's update with
// g = 0 is a fixed recurrence in (p, m, v) driven by the step's scalars. OwnerLazyTables defers
// those updates and replays them here, one step at a time through the same adam_elem, when the
// row is next read or at a flush: every element goes through the same fp32 operations in the
// same order as under the dense update, so the tables are bit-for-bit the dense ones.
//   hist[8 s + k]: step s's scalars (AdamScalars order; [7] = RN(1 / bc2s), 0: divide), s >= 1;
//                  row 0: the box header (dw::hist_box_from)
//   last[r]:       the step up to which row r's (p, m, v) are current
using dw::hist_at;

// One block per row, one element per thread (blockDim = 64 * ceil(d / 64)): the replays are
// ALU-bound dependent chains (correctly rounded sqrt and two divisions per element-step), so the
// row is spread over as many waves as it has 64-element pieces — at C3's 64-walk batch the
// in-table catch-up replays ~234 steps on 4,480 rows, and 2 waves per row fill the SIMDs where
// one wave per row (two rows per trip) left them latency-bound. Every wave reads last[r] before
// the barrier; thread 0 writes it after. STEP: replay the missed steps up to step - 1, then
// apply `step` with the row's gradient g_rows[i]; else replay up to `step`. The step loop is
// uniform: lanes past d carry zeros and are not stored.
// E = 2 (even d): two adjacent elements per thread (8-B accesses), replayed as pairs on the
// packed fp32 instructions (dw::replay_g0 with N = 2): half the threads, half the issue slots.
// BY_ROW (with STEP): the gradient is the table's own row g_rows[r] (the dense gradient buffer),
// cleared as it is used — one rank's touched in rows, with no gather in between.
template <bool STEP, bool P_ONLY = false, int E = 1, bool BY_ROW = false>
__global__ void __launch_bounds__(512)
    k_rows_adam(float *__restrict__ p, float *__restrict__ m, float *__restrict__ v,
                int32_t *__restrict__ last, uint8_t *__restrict__ pend, int64_t n_table, int32_t d,
                const uint32_t *__restrict__ rows, const int64_t *__restrict__ n_dev,
                int64_t n_max, float *__restrict__ g_rows, const float *__restrict__ hist,
                int32_t step_arg, const dw_step_scalars *__restrict__ dyn, int32_t delta) {
    const int32_t step = dw::eff_step(dyn, delta, step_arg);   // graph replay: from the block
    const int e = threadIdx.x * E;
    const bool live = e < d;
    int64_t n = n_max;
    if (n_dev) {
        const int64_t c = *n_dev;
        n = c < n_max ? c : n_max;
    }
    const int32_t upto = STEP ? step - 1 : step;
    const int32_t box_from = dw::hist_box_from(hist);
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const int64_t r = rows ? static_cast<int64_t>(rows[i]) : i;
        // an out-of-range centre is reported by the SGNS pass
        const int32_t from = r < n_table ? __builtin_amdgcn_readfirstlane(last[r]) : step;
        // a row the lazy out step left pending: p lags m and v by the parameter half of `from`
        const bool pd = pend && r < n_table && __builtin_amdgcn_readfirstlane(pend[r]) != 0;
        __syncthreads();   // every wave has read last[r] before thread 0 advances it
        if (from >= (STEP ? step : upto) && !pd) continue;   // already current (or stepped)
        const int64_t o = r * d + e;
        const int64_t og = (BY_ROW ? r : i) * d + e;   // the gradient row
        float pr[E], mr[E], vr[E], gg[E];
        if constexpr (E == 2) {   // (d even: o is 8-B aligned)
            const float2 zero = make_float2(0.f, 0.f);
            const float2 p2 = live ? *reinterpret_cast<const float2 *>(p + o) : zero;
            const float2 m2 = live ? *reinterpret_cast<const float2 *>(m + o) : zero;
            const float2 v2 = live ? *reinterpret_cast<const float2 *>(v + o) : zero;
            const float2 g2 = (STEP && live) ? *reinterpret_cast<const float2 *>(g_rows + og)
                                             : zero;
            if (BY_ROW && live) *reinterpret_cast<float2 *>(g_rows + og) = zero;
            pr[0] = p2.x, pr[1] = p2.y, mr[0] = m2.x, mr[1] = m2.y;
            vr[0] = v2.x, vr[1] = v2.y, gg[0] = g2.x, gg[1] = g2.y;
        } else {
            pr[0] = live ? p[o] : 0.f;
            mr[0] = live ? m[o] : 0.f;
            vr[0] = live ? v[o] : 0.f;
            gg[0] = (STEP && live) ? g_rows[og] : 0.f;
            if (BY_ROW && live) g_rows[og] = 0.f;
        }
        if (pd) dw::settle_pending(pr, mr, vr, hist, from, box_from);
        dw::replay_g0<E, true>(pr, mr, vr, hist, from, upto, box_from);
        if (STEP) {
            const dw::AdamScalars hs = hist_at(hist, step);
#pragma unroll
            for (int k = 0; k < E; ++k) dw::adam_elem(pr[k], gg[k], mr[k], vr[k], hs);
        }
        if (live) {
            if constexpr (E == 2) {
                *reinterpret_cast<float2 *>(p + o) = make_float2(pr[0], pr[1]);
                if (!P_ONLY) {
                    *reinterpret_cast<float2 *>(m + o) = make_float2(mr[0], mr[1]);
                    *reinterpret_cast<float2 *>(v + o) = make_float2(vr[0], vr[1]);
                }
            } else {
                p[o] = pr[0];
                if (!P_ONLY) {
                    m[o] = mr[0];
                    v[o] = vr[0];
                }
            }
        }
        if (e == 0 && !P_ONLY) {
            last[r] = STEP ? step : upto;
            if (pd) pend[r] = 0;
        }
    }
}

// out[i] = table[rows[i]] (one wave per row); zero: the source rows are cleared in the same pass
__global__ void __launch_bounds__(256)
    k_rows_gather(float *__restrict__ table, int64_t n_table, int32_t d,
                  const uint32_t *__restrict__ rows, const int64_t *__restrict__ n_dev,
                  int64_t n_max, float *__restrict__ out, int32_t zero) {
    const int lane = threadIdx.x & 63;
    int64_t n = n_max;
    if (n_dev) {
        const int64_t c = *n_dev;
        n = c < n_max ? c : n_max;
    }
    const int64_t n_waves = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t i = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; i < n;
         i += n_waves) {
        const int64_t r = static_cast<int64_t>(rows[i]);
        const bool ok = r < n_table;
        for (int64_t e = lane; e < d; e += 64) {
            out[i * d + e] = ok ? table[r * d + e] : 0.f;
            if (zero && ok) table[r * d + e] = 0.f;
        }
    }
}

__global__ void __launch_bounds__(256)
    k_scale(float *__restrict__ x, int64_t n, float alpha, const float *__restrict__ alpha_dev) {
    if (alpha_dev) alpha *= *alpha_dev;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride)
        x[i] *= alpha;
}

}  // namespace

// STREAM copy (the "measured HBM roofline" of SURVEY.md §8d / BASELINE.md): dst = src. Each
// block copies one tile of 256 x 4 float4 (all four loads in flight before the stores) with
// non-temporal loads and stores, and the grid covers the array. Of the shapes measured on MI355X
// (scripts/microbench/copy_rates.hip, profiles/r03_copy_rates.jsonl) this one is the fastest:
// 6.17 TB/s for 2 GiB, against 4.62 for a grid-stride loop of 8 blocks per CU (the round-3
// first version) and 4.96 for hipMemcpyAsync. bench.py times it once per run and reports the
// SGNS step against it beside the 8 TB/s spec figure.
__global__ void __launch_bounds__(256)
    k_stream_copy(const float4 *__restrict__ src, float4 *__restrict__ dst, int64_t n4) {
    constexpr int U = 4;
    const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
    float4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + u * 256;
        if (i < n4) {
            r[u].x = __builtin_nontemporal_load(&src[i].x);
            r[u].y = __builtin_nontemporal_load(&src[i].y);
            r[u].z = __builtin_nontemporal_load(&src[i].z);
            r[u].w = __builtin_nontemporal_load(&src[i].w);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + u * 256;
        if (i < n4) {
            __builtin_nontemporal_store(r[u].x, &dst[i].x);
            __builtin_nontemporal_store(r[u].y, &dst[i].y);
            __builtin_nontemporal_store(r[u].z, &dst[i].z);
            __builtin_nontemporal_store(r[u].w, &dst[i].w);
        }
    }
}

extern "C" {

int dw_stream_copy(const void *src, void *dst, int64_t bytes, void *stream) {
    DW_REQUIRE(bytes >= 0 && bytes % 16 == 0, "dw_stream_copy: bytes must be a multiple of 16");
    if (bytes == 0) return DW_OK;
    DW_REQUIRE(src && dst, "dw_stream_copy: null pointer");
    DW_REQUIRE((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) % 16 == 0,
               "dw_stream_copy: buffers must be 16-B aligned");
    const int64_t n4 = bytes / 16;
    const int64_t blocks = (n4 + 1023) / 1024;
    DW_REQUIRE(blocks <= 0x7FFFFFFF, "dw_stream_copy: %lld bytes is too large", (long long)bytes);
    hipLaunchKernelGGL(k_stream_copy, dim3((unsigned)blocks), dim3(256), 0, dw::as_stream(stream),
                       reinterpret_cast<const float4 *>(src), reinterpret_cast<float4 *>(dst), n4);
    DW_LAUNCH_CHECK("dw_stream_copy");
    return DW_OK;
}

int dw_adam_dense_to(const float *param_src, float *param_dst, float *grad, float *exp_avg,
                     float *exp_avg_sq, int64_t n_elem, float one_minus_beta1, float beta2,
                     float one_minus_beta2, float bias_correction2_sqrt, float neg_step_size,
                     float eps, float weight_decay, int32_t zero_grad, int64_t max_blocks,
                     void *stream) {
    DW_REQUIRE(n_elem >= 0, "dw_adam_dense: negative size");
    if (n_elem == 0) return DW_OK;
    DW_REQUIRE(param_src && param_dst && grad && exp_avg && exp_avg_sq,
               "dw_adam_dense: null pointer");
    DW_REQUIRE(((uintptr_t)param_src | (uintptr_t)param_dst | (uintptr_t)grad |
                (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0,
               "dw_adam_dense: buffers must be 16-byte aligned");
    DW_REQUIRE(bias_correction2_sqrt > 0.f, "dw_adam_dense: bias_correction2_sqrt must be > 0");
    dw::AdamScalars s{one_minus_beta1, beta2,         one_minus_beta2, bias_correction2_sqrt,
                      neg_step_size,   eps,           weight_decay,    1.0f / bias_correction2_sqrt};
    int64_t blocks = ((n_elem >> 2) + 255) / 256;
    if (blocks < 1) blocks = 1;
    if (blocks > 8192) blocks = 8192;  // 256 CUs x 8 resident blocks, grid-stride beyond
    if (max_blocks > 0 && blocks > max_blocks) blocks = max_blocks;
    {   // the deterministic mode's fused conversion (DW_EXACT_ADAM): the sums from the accumulator
        dw::Fixed fx;
        int64_t fn = 0;
        int32_t ffl = 0;
        if (dw::exact_lookup(grad, &fx, &fn, &ffl) && (ffl & DW_EXACT_ADAM)) {
            DW_REQUIRE(fn >= n_elem, "dw_adam_dense: the accumulator registered for grad holds "
                       "%lld elements, the update covers %lld", (long long)fn, (long long)n_elem);
            DW_REQUIRE(((uintptr_t)fx.acc % 16) == 0, "dw_adam_dense: accumulator alignment");
            auto *acc = reinterpret_cast<long long *>(fx.acc);
            if (zero_grad)
                hipLaunchKernelGGL(k_adam_fixed<true>, dim3((unsigned)blocks), dim3(256), 0,
                                   dw::as_stream(stream), param_src, param_dst, acc, exp_avg,
                                   exp_avg_sq, n_elem, s, fx.fi, dw::bound_step_scalars());
            else
                hipLaunchKernelGGL(k_adam_fixed<false>, dim3((unsigned)blocks), dim3(256), 0,
                                   dw::as_stream(stream), param_src, param_dst, acc, exp_avg,
                                   exp_avg_sq, n_elem, s, fx.fi, dw::bound_step_scalars());
            DW_LAUNCH_CHECK("dw_adam_dense/fixed");
            return DW_OK;
        }
    }
    if (zero_grad)
        hipLaunchKernelGGL((k_adam<true, true, 2>), dim3((unsigned)blocks), dim3(256), 0,
                           dw::as_stream(stream), param_src, param_dst, grad, exp_avg,
                           exp_avg_sq, n_elem, s, dw::bound_step_scalars());
    else
        hipLaunchKernelGGL((k_adam<false, true, 2>), dim3((unsigned)blocks), dim3(256), 0,
                           dw::as_stream(stream), param_src, param_dst, grad, exp_avg,
                           exp_avg_sq, n_elem, s, dw::bound_step_scalars());
    DW_LAUNCH_CHECK("dw_adam_dense");
    return DW_OK;
}

int dw_adam_dense(float *param, float *grad, float *exp_avg, float *exp_avg_sq, int64_t n_elem,
                  float one_minus_beta1, float beta2, float one_minus_beta2,
                  float bias_correction2_sqrt, float neg_step_size, float eps,
                  float weight_decay, int32_t zero_grad, void *stream) {
    return dw_adam_dense_to(param, param, grad, exp_avg, exp_avg_sq, n_elem, one_minus_beta1,
                            beta2, one_minus_beta2, bias_correction2_sqrt, neg_step_size, eps,
                            weight_decay, zero_grad, 0, stream);
}

}  // extern "C"

int dw::adam_rows_launch(float *param, float *exp_avg, float *exp_avg_sq, int32_t *last_step,
                         uint8_t *pending, int64_t n_table_rows, int32_t dim, const uint32_t *rows,
                         const int64_t *n_rows_dev, int64_t n_rows_max, float *grad_rows,
                         const float *hist, int32_t step, bool p_only, hipStream_t st,
                         bool grad_by_row) {
    DW_REQUIRE(n_table_rows >= 0 && dim >= 1 && n_rows_max >= 0 && step >= 0,
               "dw_adam_rows: bad sizes");
    if (n_rows_max == 0) return DW_OK;
    DW_REQUIRE(param && exp_avg && exp_avg_sq && last_step && hist, "dw_adam_rows: null pointer");
    DW_REQUIRE(rows || !n_rows_dev, "dw_adam_rows: a device row count needs a row list");
    DW_REQUIRE(!grad_rows || step >= 1, "dw_adam_rows: a gradient step needs step >= 1");
    DW_REQUIRE(dim <= 512, "dw_adam_rows: dim > 512 is not supported");
    const dw_step_scalars *dyn = nullptr;
    int32_t delta = 0;
    const int rc = dw::bound_step_rel(step, &dyn, &delta, "dw_adam_rows");
    if (rc != DW_OK) return rc;
    int64_t blocks = n_rows_max;   // one block per row (grid-stride beyond the cap)
    if (blocks > 65536) blocks = 65536;
    DW_REQUIRE(!(p_only && grad_rows), "dw_adam_rows: p_only replays carry no gradient step");
    DW_REQUIRE(!(p_only && pending), "dw_adam_rows: p_only replays do not settle pending rows");
    DW_REQUIRE(!grad_by_row || grad_rows, "dw_adam_rows: grad_by_row needs the gradient table");
    // a pending row current to `step` would be settled and then stepped a second time
    DW_REQUIRE(!(pending && grad_rows), "dw_adam_rows: pending rows are settled without a "
               "gradient step (flush); step them through the rows-major out step");
    // even d: two elements per thread on the packed instructions
    const bool pair = dim % 2 == 0;
    const int threads = pair ? 64 * ((dim / 2 + 63) / 64) : 64 * ((dim + 63) / 64);
#define DW_ROWS_ADAM(STEP_, PONLY_, BYROW_)                                                      \
    do {                                                                                        \
        if (pair)                                                                               \
            hipLaunchKernelGGL((k_rows_adam<STEP_, PONLY_, 2, BYROW_>), dim3((unsigned)blocks), \
                               dim3(threads), 0, st, param, exp_avg, exp_avg_sq, last_step,     \
                               pending, n_table_rows, dim, rows, n_rows_dev, n_rows_max,        \
                               grad_rows, hist,                                                 \
                               step, dyn, delta);                                               \
        else                                                                                    \
            hipLaunchKernelGGL((k_rows_adam<STEP_, PONLY_, 1, BYROW_>), dim3((unsigned)blocks), \
                               dim3(threads), 0, st, param, exp_avg, exp_avg_sq, last_step,     \
                               pending, n_table_rows, dim, rows, n_rows_dev, n_rows_max,        \
                               grad_rows, hist,                                                 \
                               step, dyn, delta);                                               \
    } while (0)
    if (grad_rows && grad_by_row)
        DW_ROWS_ADAM(true, false, true);
    else if (grad_rows)
        DW_ROWS_ADAM(true, false, false);
    else if (p_only)
        DW_ROWS_ADAM(false, true, false);
    else
        DW_ROWS_ADAM(false, false, false);
#undef DW_ROWS_ADAM
    DW_LAUNCH_CHECK("dw_adam_rows");
    return DW_OK;
}

extern "C" {

int dw_adam_rows(float *param, float *exp_avg, float *exp_avg_sq, int32_t *last_step,
                 uint8_t *pending, int64_t n_table_rows, int32_t dim, const uint32_t *rows,
                 const int64_t *n_rows_dev, int64_t n_rows_max, float *grad_rows,
                 int32_t grad_by_row, const float *hist, int32_t step, void *stream) {
    return dw::adam_rows_launch(param, exp_avg, exp_avg_sq, last_step, pending, n_table_rows,
                                dim, rows, n_rows_dev, n_rows_max, grad_rows, hist, step, false,
                                dw::as_stream(stream), grad_by_row != 0);
}

int dw_rows_gather(float *table, int64_t n_table_rows, int32_t dim, const uint32_t *rows,
                   const int64_t *n_rows_dev, int64_t n_rows_max, float *out,
                   int32_t zero_source, void *stream) {
    DW_REQUIRE(n_table_rows >= 0 && dim >= 1 && n_rows_max >= 0, "dw_rows_gather: bad sizes");
    if (n_rows_max == 0) return DW_OK;
    DW_REQUIRE(table && rows && out, "dw_rows_gather: null pointer");
    int64_t blocks = (n_rows_max + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_rows_gather, dim3((unsigned)blocks), dim3(256), 0, dw::as_stream(stream),
                       table, n_table_rows, dim, rows, n_rows_dev, n_rows_max, out, zero_source);
    DW_LAUNCH_CHECK("dw_rows_gather");
    return DW_OK;
}

int dw_scale(float *x, int64_t n_elem, float alpha, const float *alpha_dev, void *stream) {
    DW_REQUIRE(n_elem >= 0, "dw_scale: negative size");
    if (n_elem == 0) return DW_OK;
    DW_REQUIRE(x, "dw_scale: null pointer");
    int64_t blocks = (n_elem + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_scale, dim3((unsigned)blocks), dim3(256), 0, dw::as_stream(stream), x,
                       n_elem, alpha, alpha_dev);
    DW_LAUNCH_CHECK("dw_scale");
    return DW_OK;
}

}  // extern "C"
