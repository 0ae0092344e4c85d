// Internal helpers shared by the gfx950 kernels of libdw_hip.so (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/dw_hip.h"

namespace dw {

// ---- error reporting across the C ABI ---------------------------------------------------------
void set_error(const char *fmt, ...);

// The dw_step_scalars block bound on this host thread (dw_step_scalars_bind), or NULL.
const dw_step_scalars *bound_step_scalars();

// Lazy-Adam launches (dw_adam_rows, dw_sgns_owner_out_catch_up, dw_sgns_owner_pass2_lazy) take an
// Adam step number. With a block bound by dw_step_scalars_bind_at(dev, host_step) their `step`
// argument is relative to it: the kernels use dyn->step + (step - host_step), read on the
// device. Returns DW_OK and sets *dyn / *delta (dyn NULL: nothing bound, use `step`), or
// DW_E_INVALID_ARG when a block is bound without a host step (dw_step_scalars_bind): a captured
// lazy step would otherwise replay a frozen step number.
int bound_step_rel(int64_t step, const dw_step_scalars **dyn, int32_t *delta, const char *what);

// The step a lazy kernel applies: the bound block's (plus the launch's delta) or the launch's.
__device__ __forceinline__ int32_t eff_step(const dw_step_scalars *dyn, int32_t delta,
                                            int32_t step) {
    return dyn ? static_cast<int32_t>(dyn->step) + delta : step;
}

#define DW_REQUIRE(cond, ...)                 \
    do {                                      \
        if (!(cond)) {                        \
            ::dw::set_error(__VA_ARGS__);     \
            return DW_E_INVALID_ARG;          \
        }                                     \
    } while (0)

#define DW_LAUNCH_CHECK(what)                                                         \
    do {                                                                              \
        hipError_t e_ = hipGetLastError();                                            \
        if (e_ != hipSuccess) {                                                       \
            ::dw::set_error("%s: HIP launch failed: %s", what, hipGetErrorString(e_)); \
            return DW_E_HIP;                                                          \
        }                                                                             \
    } while (0)

static inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// ---- Philox4x32-10 (Salmon et al., SC'11), the device RNG of every fast-mode kernel ----------
// Restated bit-for-bit on the host in oracle/philox.py (test infrastructure).
struct U4 {
    uint32_t x, y, z, w;
};

template <int ROUNDS = 10>
__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
        const uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
        const uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += W0;
        k1 += W1;
    }
    return c;
}

// Stream tags keep the counter spaces of different consumers disjoint.
constexpr uint32_t TAG_DEEPWALK = 0x44570000u;   // 'DW'
constexpr uint32_t TAG_NODE2VEC = 0x4E320000u;   // 'N2'
constexpr uint32_t TAG_N2V_POS = 0x4E500000u;    // 'NP' (node2vec over the position index)

// Uniform index in [0, n) from 32 random bits (multiply-high; bias <= n / 2^32).
__device__ __forceinline__ uint32_t bounded32(uint32_t r, uint32_t n) { return __umulhi(r, n); }

// Uniform index in [0, n) from 64 random bits (bias <= n / 2^64) — torch.randint(0, V) analogue.
__device__ __forceinline__ uint64_t bounded64(uint32_t lo, uint32_t hi, uint64_t n) {
    const uint64_t r = (static_cast<uint64_t>(hi) << 32) | lo;
    return __umul64hi(r, n);
}

// Per-row adjacency hash (dw_adj_hash_*): buckets of 16 int32 slots for a row of degree `deg`
// (none up to DW_ADJ_HASH_MIN_DEG, else load <= 3/4), and the home bucket of neighbour x.
__host__ __device__ __forceinline__ int64_t adj_buckets(int64_t deg) {
    return deg > DW_ADJ_HASH_MIN_DEG ? (4 * deg + 47) / 48 : 0;
}
__device__ __forceinline__ uint32_t adj_bucket(int32_t x, uint32_t nb) {
    return static_cast<uint32_t>(
        (static_cast<uint64_t>(static_cast<uint32_t>(x) * 0x9E3779B1u) * nb) >> 32);
}

__device__ __forceinline__ void status_or(int32_t *status, int32_t bits) {
    if (status) atomicOr(status, bits);
}

// Wave-level LDS visibility for a wave that owns a private LDS slice (no s_barrier needed).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

__device__ __forceinline__ double wave_sum_d(double x) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

// torch.optim.Adam single-tensor update of one element (dw_adam.hip; also fused into the SGNS
// output-table pass). Scalars precomputed on the host in float64, cast to float32.
struct AdamScalars {
    float w1, b2, omb2, bc2s, nstep, eps, wd;
    float rbc2s = 0.f;   // RN(1 / bc2s) from the host (0: divide)
};

// sqrt(v) / bias_correction2_sqrt, bit for bit the IEEE quotient: with y = RN(1 / c) computed on
// the host, q = x y, the remainder r = fma(-c, q, x) is exact and fma(r, y, q) is the correctly
// rounded x / c (Markstein) for x in [2^-64, 2^64] — proved on MI355X for every fp32 mantissa
// and every step's c at beta2 .999 and .99 (1.53e11 checks, 0 mismatches: scripts/microbench/
// div_proof.py, profiles/r05_div_proof.jsonl); the host writes y into the history only for those
// betas (sharding.RECIPROCAL_PROVEN_BETA2), else 0. Three operations for the ~12 of the IEEE
// sequence (its rcp is quarter rate): the lazy replays are ALU-bound on these steps. Outside the
// range, or without y, the wave divides (the same bits either way).
__device__ __forceinline__ float div_bc2s(float x, const AdamScalars &s) {
#pragma clang fp contract(off)
    const bool ok = s.rbc2s != 0.f && ((x >= 0x1p-64f && x <= 0x1p64f) || x == 0.f);
    if (__all(ok)) {
        const float q = x * s.rbc2s;
        const float r = fmaf(-s.bc2s, q, x);
        return fmaf(r, s.rbc2s, q);
    }
    return x / s.bc2s;
}

// adam_elem in its two halves: the moments (adam_mv: m and v from g, weight decay reading p as
// it was before the step) and the parameter (adam_p: p from the new m and v). The lazy out step
// (dw_sgns_owner_out_rows) applies the first at step s and leaves the second pending until the
// row is next read (dw::settle_pending): the same operations on the same values, the same bits.
__device__ __forceinline__ void adam_mv(float p, float &g, float &m, float &v,
                                        const AdamScalars &s) {
#pragma clang fp contract(off)
    float gg = g;
    if (s.wd != 0.f) gg = gg + s.wd * p;
    m = fmaf(s.w1, gg - m, m);  // lerp with weight < 0.5: self + weight * (end - self)
    v = v * s.b2;
    v = v + s.omb2 * gg * gg;
}

__device__ __forceinline__ void adam_p(float &p, float m, float v, const AdamScalars &s) {
#pragma clang fp contract(off)
    const float denom = div_bc2s(sqrtf(v), s) + s.eps;
    p = p + s.nstep * (m / denom);
}

__device__ __forceinline__ void adam_elem(float &p, float &g, float &m, float &v,
                                          const AdamScalars &s) {
    // No implicit FMA contraction: each element rounds the same way whichever unrolled slot,
    // grid size or fused kernel (k_rec_gather) updates it; the lerp's fmaf is explicit.
    adam_mv(p, g, m, v, s);
    adam_p(p, m, v, s);
}

// adam_elem with g = 0 when weight_decay == 0 (the lazy replays' deferred steps; callers test
// wd once per step, uniformly). The same IEEE operations give the same bits: gg - m is -m
// exactly (for m = +-0 both forms make fmaf's result +0), omb2 * 0 * 0 is +0 and v + (+0) is v
// for every v the update can hold (v >= +0, or NaN / inf) — minus the dead operations and the
// per-lane weight-decay select, which the replay loops, ALU-bound, otherwise pay every step.
__device__ __forceinline__ void adam_elem_g0(float &p, float &m, float &v, const AdamScalars &s) {
#pragma clang fp contract(off)
    m = fmaf(s.w1, -m, m);
    v = v * s.b2;
    const float denom = div_bc2s(sqrtf(v), s) + s.eps;
    p = p + s.nstep * (m / denom);
}

// Row s of a per-step Adam scalar history ([steps][8] fp32; the lazy exact Adam's replays).
__device__ __forceinline__ AdamScalars hist_at(const float *__restrict__ hist, int64_t s) {
    const float *h = hist + 8 * s;
    return AdamScalars{h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]};
}

// ---- the g = 0 replay inside a box where sqrt and division need no range scaling ----------------
// sqrtf and the IEEE division compile to range-scaled sequences: sqrtf scales x < 2^-96 by 2^32
// (and back) and selects x itself for +-0 / inf / NaN; the division runs v_div_scale on both
// operands, v_div_fmas and v_div_fixup around the reciprocal's Newton / Markstein steps. Inside
// the box below no operand is scaled (v_div_scale returns it unchanged, v_div_fmas is a plain fma,
// v_div_fixup passes the quotient through), so the unscaled steps are the same operations on the
// same values — the same bits — for ~30 VALU slots per element-step instead of ~45 (the lazy
// replays run at the VALU's issue rate). Checked on MI355X for every x in the box's sqrt range
// and 2^32 random quotients (scripts/microbench/box_check.hip), and by the lazy-vs-dense tests.
__device__ __forceinline__ float sqrt_box(float x) {   // x = +0 or x in [2^-96, 2^20]
#pragma clang fp contract(off)
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u);
    const float su = __uint_as_float(__float_as_uint(s) + 1u);
    const float rd = fmaf(-sd, s, x), ru = fmaf(-su, s, x);
    float t = rd <= 0.f ? sd : s;
    return ru > 0.f ? su : t;
}

__device__ __forceinline__ float div_box(float n, float d) {   // |n| in [2^-100, 2^60] or n = +0,
#pragma clang fp contract(off)                                  // d in [2^-27, 2^21]
    float r = __builtin_amdgcn_rcpf(d);
    float e = fmaf(-d, r, 1.0f);
    r = fmaf(e, r, r);
    float q = n * r;
    e = fmaf(-d, q, n);
    q = fmaf(e, r, q);
    e = fmaf(-d, q, n);
    return fmaf(e, r, q);
}

// A step whose scalars keep every replayed operand in the box: weight_decay +0 (the g = 0
// form), the reciprocal present, eps in [2^-27, 1], bc2s in [2^-10, 1], w1 and b2 in [0, 1] —
// then |m| and v only shrink, sqrt(v) <= 2^10 when v <= 2^20, and the denominator
// sqrt(v) / bc2s + eps lies in [2^-27, 2^21). The host tests its rows when it writes them and
// keeps the answer in the history's row 0, which no step uses (include/dw_hip.h,
// DW_HIST_BOX_TAG): [0] the tag's bits, [1] the bits of the int32 step from which every written
// row is in the box. Anything else there: no step is taken to be in the box.
__device__ __forceinline__ int32_t hist_box_from(const float *__restrict__ hist) {
    typedef __attribute__((address_space(4))) const uint32_t const_u32;
    const const_u32 *h0 = (const const_u32 *)hist;
    return h0[0] == DW_HIST_BOX_TAG ? static_cast<int32_t>(h0[1]) : INT32_MAX;
}

__device__ __forceinline__ void adam_elem_g0_box(float &p, float &m, float &v, const AdamScalars &s) {
#pragma clang fp contract(off)
    m = fmaf(s.w1, -m, m);
    v = v * s.b2;
    const float x = sqrt_box(v);
    const float q = x * s.rbc2s;
    const float c = fmaf(-s.bc2s, q, x);
    const float denom = fmaf(c, s.rbc2s, q) + s.eps;
    p = p + s.nstep * div_box(m, denom);
}

// The box step on two elements at once: the same IEEE operations per element as
// adam_elem_g0_box — the multiplies, adds and fmas as gfx950's packed fp32 instructions
// (v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32: two elements per lane and issue slot, each
// rounded as the scalar instruction rounds it), the sqrt and reciprocal seeds and the sqrt's
// rounding selects per element. ~18 issue slots per element-step instead of ~30: the replays
// are ALU-bound (every row's deferred steps are eventually replayed, ~V x d element-steps per
// training step in the steady state of the lazy exact Adam).
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 sqrt_box2(f32x2 x) {
#pragma clang fp contract(off)
    f32x2 s;
    s.x = __builtin_amdgcn_sqrtf(x.x);
    s.y = __builtin_amdgcn_sqrtf(x.y);
    f32x2 sd, su;
    sd.x = __uint_as_float(__float_as_uint(s.x) - 1u);
    sd.y = __uint_as_float(__float_as_uint(s.y) - 1u);
    su.x = __uint_as_float(__float_as_uint(s.x) + 1u);
    su.y = __uint_as_float(__float_as_uint(s.y) + 1u);
    const f32x2 rd = __builtin_elementwise_fma(-sd, s, x);
    const f32x2 ru = __builtin_elementwise_fma(-su, s, x);
    f32x2 r;
    r.x = ru.x > 0.f ? su.x : (rd.x <= 0.f ? sd.x : s.x);
    r.y = ru.y > 0.f ? su.y : (rd.y <= 0.f ? sd.y : s.y);
    return r;
}

__device__ __forceinline__ f32x2 div_box2(f32x2 n, f32x2 d) {
#pragma clang fp contract(off)
    f32x2 r;
    r.x = __builtin_amdgcn_rcpf(d.x);
    r.y = __builtin_amdgcn_rcpf(d.y);
    const f32x2 one = {1.0f, 1.0f};
    f32x2 e = __builtin_elementwise_fma(-d, r, one);
    r = __builtin_elementwise_fma(e, r, r);
    f32x2 q = n * r;
    e = __builtin_elementwise_fma(-d, q, n);
    q = __builtin_elementwise_fma(e, r, q);
    e = __builtin_elementwise_fma(-d, q, n);
    return __builtin_elementwise_fma(e, r, q);
}

__device__ __forceinline__ void adam_elem_g0_box2(f32x2 &p, f32x2 &m, f32x2 &v,
                                                  const AdamScalars &s, f32x2 &x) {
#pragma clang fp contract(off)
    const f32x2 w1 = {s.w1, s.w1}, b2 = {s.b2, s.b2}, rb = {s.rbc2s, s.rbc2s};
    const f32x2 bc = {s.bc2s, s.bc2s}, eps = {s.eps, s.eps}, ns = {s.nstep, s.nstep};
    m = __builtin_elementwise_fma(w1, -m, m);
    v = v * b2;
    x = sqrt_box2(v);
    const f32x2 q = x * rb;
    const f32x2 c = __builtin_elementwise_fma(-bc, q, x);
    const f32x2 denom = __builtin_elementwise_fma(c, rb, q) + eps;
    p = p + ns * div_box2(m, denom);
}

// ---- frozen parameters: the tail of a long g = 0 replay where p can no longer move -------------
// Over g = 0 steps m shrinks by (1 - beta1) and sqrt(v) by only sqrt(beta2) per step, so after
// enough of them every update y_j = RN(nstep_j RN(m_j / denom_j)) is below half the spacing of p
// around p and p + y_j rounds back to p: the remaining steps change m and v only. The host
// certifies the history's box rows (sharding.hist_header, row 0): [2] F = max |nstep| over them,
// [3] their eps, constant, with (1 - beta1)(1 + 2^-20) <= sqrt(beta2) on every row — else F = inf
// (never frozen). Then for every later step j, |m_j| / denom_j <= |m_k| / max(x_k, eps) (m
// shrinks at least as fast as x = RN(sqrt(v)) while x > eps; denom_j >= max(x_j, eps), and a
// subnormal m_j is below 2^-126 / eps), so |y_j| <= F |m_k| / max(x_k, eps) (1 + 2^-24)^3, and
// p is frozen once that is below |p| 2^-26 (< half the spacing below |p|) — tested with margins
// in fp32 (frozen_el). m = +-0 freezes p too (y is a signed zero), except p = -0 with m = -0.
// The same bits as the full steps (tests/test_gpu_owner.py::test_rows_adam_long_lag_bit_exact).
struct Freeze {
    float F, eps;
};

__device__ __forceinline__ Freeze hist_freeze(const float *__restrict__ hist) {
    typedef __attribute__((address_space(4))) const uint32_t const_u32;
    const const_u32 *h0 = (const const_u32 *)hist;
    if (h0[0] != DW_HIST_BOX_TAG) return Freeze{__builtin_huge_valf(), 0.f};
    return Freeze{__uint_as_float(h0[2]), __uint_as_float(h0[3])};
}

// The history's constant betas (row 0 [4] = 1 - beta1, [5] = beta2, from sharding.hist_header:
// every box row has the same), or ok = false (NaN there: the betas changed along the run).
struct Betas {
    float w1, b2;
    bool ok;
};

__device__ __forceinline__ Betas hist_betas(const float *__restrict__ hist) {
    typedef __attribute__((address_space(4))) const uint32_t const_u32;
    const const_u32 *h0 = (const const_u32 *)hist;
    const float w1 = __uint_as_float(h0[4]), b2 = __uint_as_float(h0[5]);
    return Betas{w1, b2, h0[0] == DW_HIST_BOX_TAG && w1 == w1 && b2 == b2};
}

__device__ __forceinline__ bool frozen_el(float p, float m, float x, const Freeze &fz) {
#pragma clang fp contract(off)
    const uint32_t mb = __float_as_uint(m), pb = __float_as_uint(p);
    if ((mb & 0x7FFFFFFFu) == 0u) return !(pb == 0x80000000u && mb == 0x80000000u);
    const float ap = fabsf(p);
    const float rhs = ap * fmaxf(x, fz.eps) * 0x1p-26f;
    return fz.F * fabsf(m) * (1.0f + 0x1p-18f) < rhs && rhs >= 0x1p-100f &&
           ap * 0x1p-26f > fz.F * 0x1p-97f;
}

// The history read as constant memory: the scalar unit loads the step's scalars (uniform) and
// tests them, where a generic pointer after the kernel's own stores gets vector loads.
typedef __attribute__((address_space(4))) const float const_float;
__device__ __forceinline__ AdamScalars hist_at_const(const const_float *h8) {
    return AdamScalars{h8[0], h8[1], h8[2], h8[3], h8[4], h8[5], h8[6], h8[7]};
}

// Replays steps from + 1 .. upto with g = 0 on N elements per lane, bit for bit adam_elem_g0 /
// adam_elem. Steps from box_from on (hist_box_from: read once per launch) are in the box; |m|
// and v are non-increasing over them, so the box holds for every step of a run when it holds at
// both ends: at the start v <= 2^20 and |m| <= 2^60, at the end v >= 2^-96 unless v started +0
// (it stays +0) and |m| >= 2^-100 unless m started +0 (likewise). A row with an earlier step
// replays on the scaled path, as does a wave whose run ends outside the box (from its saved
// state). The run tests nothing per step: a test per step, on the scalar unit or not, made the
// replays slower than the scaled path they replace (scripts/microbench/replay_bench.hip).
// FREEZE: test every 8 steps whether p is frozen for the rest of the run (frozen_el) and then
// step m and v alone — for the long replays (dw_adam_rows: the in table's catch-ups, ~234 missed
// steps a row at C3's 64-walk batch, and the flushes); the short ones (the out rows' ~4) keep the
// plain loop and its registers.
template <int N, bool FREEZE = false>
__device__ __forceinline__ void replay_g0(float (&p)[N], float (&m)[N], float (&v)[N],
                                          const float *__restrict__ hist, int32_t from,
                                          int32_t upto, int32_t box_from) {
    if (from >= upto) return;
    bool start = from + 1 >= box_from;
#pragma unroll
    for (int k = 0; k < N; ++k) start = start && v[k] <= 0x1p20f && fabsf(m[k]) <= 0x1p60f;
    if (__all(start)) {
        float p0[N], m0[N], v0[N];
#pragma unroll
        for (int k = 0; k < N; ++k) {
            p0[k] = p[k];
            m0[k] = m[k];
            v0[k] = v[k];
        }
        const const_float *hc = (const const_float *)hist;
        float mc[N], vc[N];   // m, v after the last full step (the box test's end values)
        if constexpr (N % 2 == 0) {   // element pairs on the packed fp32 instructions
            f32x2 P[N / 2], M[N / 2], W[N / 2], X[N / 2];
#pragma unroll
            for (int k = 0; k < N / 2; ++k) {
                P[k] = f32x2{p[2 * k], p[2 * k + 1]};
                M[k] = f32x2{m[2 * k], m[2 * k + 1]};
                W[k] = f32x2{v[2 * k], v[2 * k + 1]};
            }
            const Freeze fz = hist_freeze(hist);
            bool frozen = false;
            int32_t s = from + 1;
            for (; s <= upto; ++s) {
                const AdamScalars h = hist_at_const(hc + 8 * static_cast<int64_t>(s));
#pragma unroll
                for (int k = 0; k < N / 2; ++k) adam_elem_g0_box2(P[k], M[k], W[k], h, X[k]);
                if (FREEZE && ((s - from) & 7) == 0 && s < upto) {   // every 8: p frozen for good?
                    bool f = true;
#pragma unroll
                    for (int k = 0; k < N / 2; ++k)
                        f = f && frozen_el(P[k].x, M[k].x, X[k].x, fz) &&
                            frozen_el(P[k].y, M[k].y, X[k].y, fz);
                    if (__all(f)) {
                        frozen = true;
                        ++s;
                        break;
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < N / 2; ++k) {
                mc[2 * k] = M[k].x;
                mc[2 * k + 1] = M[k].y;
                vc[2 * k] = W[k].x;
                vc[2 * k + 1] = W[k].y;
            }
            if (frozen) {   // the remaining steps move m and v only (the same operations)
                const Betas hb = hist_betas(hist);
                if (hb.ok) {
                    // constant betas: no per-step history loads (a steady-state catch-up replays
                    // thousands of frozen steps a row), 8 steps a trip; once m is +0 in every
                    // lane it stays +0 (fma(w1, -0, +0) = +0; a -0 becomes +0 in one step, so
                    // only +0 ends the m updates) and v steps alone
                    const f32x2 w1 = {hb.w1, hb.w1}, b2 = {hb.b2, hb.b2};
                    bool mzero = false;
                    while (s <= upto) {
                        bool z = true;
#pragma unroll
                        for (int k = 0; k < N / 2; ++k)
                            z = z && (__float_as_uint(M[k].x) | __float_as_uint(M[k].y)) == 0u;
                        if (__all(z)) {
                            mzero = true;
                            break;
                        }
                        if (upto - s >= 7) {
#pragma unroll
                            for (int u = 0; u < 8; ++u) {
#pragma unroll
                                for (int k = 0; k < N / 2; ++k) {
                                    M[k] = __builtin_elementwise_fma(w1, -M[k], M[k]);
                                    W[k] = W[k] * b2;
                                }
                            }
                            s += 8;
                        } else {
                            for (; s <= upto; ++s) {
#pragma unroll
                                for (int k = 0; k < N / 2; ++k) {
                                    M[k] = __builtin_elementwise_fma(w1, -M[k], M[k]);
                                    W[k] = W[k] * b2;
                                }
                            }
                        }
                    }
                    if (mzero) {
                        for (; upto - s >= 7; s += 8) {
#pragma unroll
                            for (int u = 0; u < 8; ++u) {
#pragma unroll
                                for (int k = 0; k < N / 2; ++k) W[k] = W[k] * b2;
                            }
                        }
                        for (; s <= upto; ++s) {
#pragma unroll
                            for (int k = 0; k < N / 2; ++k) W[k] = W[k] * b2;
                        }
                    }
                } else {
                    for (; s <= upto; ++s) {
                        const float w1s = hc[8 * static_cast<int64_t>(s)];
                        const float b2s = hc[8 * static_cast<int64_t>(s) + 1];
                        const f32x2 w1 = {w1s, w1s}, b2 = {b2s, b2s};
#pragma unroll
                        for (int k = 0; k < N / 2; ++k) {
                            M[k] = __builtin_elementwise_fma(w1, -M[k], M[k]);
                            W[k] = W[k] * b2;
                        }
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < N / 2; ++k) {
                p[2 * k] = P[k].x;
                p[2 * k + 1] = P[k].y;
                m[2 * k] = M[k].x;
                m[2 * k + 1] = M[k].y;
                v[2 * k] = W[k].x;
                v[2 * k + 1] = W[k].y;
            }
        } else {
            for (int32_t s = from + 1; s <= upto; ++s) {
                const AdamScalars h = hist_at_const(hc + 8 * static_cast<int64_t>(s));
#pragma unroll
                for (int k = 0; k < N; ++k) adam_elem_g0_box(p[k], m[k], v[k], h);
            }
#pragma unroll
            for (int k = 0; k < N; ++k) {
                mc[k] = m[k];
                vc[k] = v[k];
            }
        }
        bool end = true;
#pragma unroll
        for (int k = 0; k < N; ++k)
            end = end && (__float_as_uint(v0[k]) == 0u || vc[k] >= 0x1p-96f) &&
                  (__float_as_uint(m0[k]) == 0u || fabsf(mc[k]) >= 0x1p-100f);
        if (__all(end)) return;
#pragma unroll
        for (int k = 0; k < N; ++k) {
            p[k] = p0[k];
            m[k] = m0[k];
            v[k] = v0[k];
        }
    }
    for (int32_t s = from + 1; s <= upto; ++s) {
        const AdamScalars h = hist_at(hist, s);
        if (h.wd == 0.f) {
#pragma unroll
            for (int k = 0; k < N; ++k) adam_elem_g0(p[k], m[k], v[k], h);
        } else {
#pragma unroll
            for (int k = 0; k < N; ++k) {
                float z = 0.f;
                adam_elem(p[k], z, m[k], v[k], h);
            }
        }
    }
}

// A row left pending by the lazy out step (m, v at step `at`, p at at - 1): the parameter half
// of step `at` (adam_p with that step's scalars), which makes the row current to `at`. When the
// step is in the box (at >= box_from: its scalars certified by the host) and every element's
// operands are — v +0 or in [2^-96, 2^20], m +0 or |m| in [2^-100, 2^60], so the denominator
// lies in [2^-27, 2^21) — the unscaled sqrt and division (the box replay's, packed two elements
// per instruction) give the same bits for about half the issue slots: nearly every row the
// rows-major step touches was left pending by an earlier step.
template <int N>
__device__ __forceinline__ void settle_pending(float (&p)[N], const float (&m)[N],
                                               const float (&v)[N],
                                               const float *__restrict__ hist, int32_t at,
                                               int32_t box_from = INT32_MAX) {
#pragma clang fp contract(off)
    // (the scalars through the scalar unit: a vector load here would make the wave wait for
    // every load issued before it — vector loads return in order)
    const AdamScalars h = hist_at_const((const const_float *)hist + 8 * static_cast<int64_t>(at));
    bool ok = at >= box_from;
#pragma unroll
    for (int k = 0; k < N; ++k)
        ok = ok &&
             (__float_as_uint(v[k]) == 0u || (v[k] >= 0x1p-96f && v[k] <= 0x1p20f)) &&
             (__float_as_uint(m[k]) == 0u ||
              (fabsf(m[k]) >= 0x1p-100f && fabsf(m[k]) <= 0x1p60f));
    if (__all(ok)) {
        if constexpr (N % 2 == 0) {
            const f32x2 rb = {h.rbc2s, h.rbc2s}, bc = {h.bc2s, h.bc2s};
            const f32x2 eps = {h.eps, h.eps}, ns = {h.nstep, h.nstep};
#pragma unroll
            for (int k = 0; k < N / 2; ++k) {
                const f32x2 M = {m[2 * k], m[2 * k + 1]};
                const f32x2 x = sqrt_box2(f32x2{v[2 * k], v[2 * k + 1]});
                const f32x2 q = x * rb;
                const f32x2 c = __builtin_elementwise_fma(-bc, q, x);
                const f32x2 denom = __builtin_elementwise_fma(c, rb, q) + eps;
                const f32x2 P = f32x2{p[2 * k], p[2 * k + 1]} + ns * div_box2(M, denom);
                p[2 * k] = P.x;
                p[2 * k + 1] = P.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < N; ++k) {
                const float x = sqrt_box(v[k]);
                const float q = x * h.rbc2s;
                const float c = fmaf(-h.bc2s, q, x);
                const float denom = fmaf(c, h.rbc2s, q) + h.eps;
                p[k] = p[k] + h.nstep * div_box(m[k], denom);
            }
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < N; ++k) adam_p(p[k], m[k], v[k], h);
}

// The Adam scalars a kernel uses: the bound step block's when there is one (graph replay),
// else the launch's by-value ones.
__device__ __forceinline__ AdamScalars step_adam(const dw_step_scalars *dyn,
                                                 const AdamScalars &s) {
    if (!dyn) return s;
    const float *h = dyn->adam;
    return AdamScalars{h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]};
}

// dw_adam_rows (dw_adam.hip) with p_only: the replayed g = 0 steps go back to memory as p alone
// (m, v and last[] untouched) — the lazy out slice's catch-up before pass 1, whose lazy gather
// then replays m and v itself (their g = 0 recurrences are a multiply each) before the step.
int adam_rows_launch(float *param, float *exp_avg, float *exp_avg_sq, int32_t *last_step,
                     uint8_t *pending, int64_t n_table_rows, int32_t dim, const uint32_t *rows,
                     const int64_t *n_rows_dev, int64_t n_rows_max, float *grad_rows,
                     const float *hist, int32_t step, bool p_only, hipStream_t stream,
                     bool grad_by_row = false);

// ---- deterministic accumulation (dw_exact_register) -----------------------------------------
// A gradient term t (fp32) enters an int64 accumulator as round(t * 2^frac): integer sums are
// associative, so the accumulated value is independent of the order of the atomics and of how
// the terms are split over waves, chunks or ranks. One f64 product (exact: a power of two) and
// the 1.5 * 2^52 magic addition round to the nearest integer; valid while |t| 2^frac < 2^51
// (`range` records a term past it: DW_S_FIXED_RANGE).
struct Fixed {
    int64_t *acc;       // the accumulator of the launch's gradient buffer (NULL: float path)
    double fs, fi;      // 2^frac, 2^-frac
};

__device__ __forceinline__ int64_t to_fixed(float t, double fs, bool &range) {
    const double y = static_cast<double>(t) * fs;
    range = range || !(fabs(y) < 0x1p51);
    const double r = y + 6755399441055744.0;
    return __double_as_longlong(r) - 0x4338000000000000LL;
}

// to_fixed in three issue slots per term: a run of terms adds the raw bits of fma(t, fs, M)
// (M = 1.5 * 2^52: the same double as to_fixed's r, since t * fs is exact) and the run's
// n * bits(M) is subtracted once (fixed_finish) — the same integers, with the int64 sums
// wrapping harmlessly; the range test runs once on the run's largest |t| (fixed_range).
__device__ __forceinline__ int64_t fixed_bits(float t, double fs) {
    return __double_as_longlong(fma(static_cast<double>(t), fs, 6755399441055744.0));
}
__device__ __forceinline__ int64_t fixed_finish(int64_t acc, int64_t n_terms) {
    return static_cast<int64_t>(static_cast<uint64_t>(acc) -
                                static_cast<uint64_t>(n_terms) * 0x4338000000000000ULL);
}
// The run's largest |t| is tracked as its bit pattern (fixed_track): an unsigned max orders NaN
// above +inf above every finite |t|, so a NaN term is kept (fmaxf would drop it) and fails the
// range test like an infinite or too large one.
__device__ __forceinline__ uint32_t fixed_track(uint32_t tbits, float t) {
    const uint32_t b = __float_as_uint(t) & 0x7FFFFFFFu;
    return b > tbits ? b : tbits;
}
__device__ __forceinline__ bool fixed_range(uint32_t tbits, double fs) {
    return !(static_cast<double>(__uint_as_float(tbits)) * fs < 0x1p51);
}

__device__ __forceinline__ float from_fixed(int64_t a, double fi) {
    return static_cast<float>(static_cast<double>(a) * fi);
}

// The accumulator registered for gradient buffer g (dw_exact_register): 1 and its Fixed, size
// and flags, or 0 (dw_sgns.hip).
int exact_lookup(const float *g, Fixed *fx, int64_t *n, int32_t *flags);

__device__ __forceinline__ void fixed_add(int64_t *dst, int64_t v) {
    if (v) atomicAdd(reinterpret_cast<unsigned long long *>(dst), static_cast<unsigned long long>(v));
}

}  // namespace dw
