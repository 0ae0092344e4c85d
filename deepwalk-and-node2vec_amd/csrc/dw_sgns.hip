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
//     {row, centre, coef} (coalesced), the records are radix-sorted by row (rocprim onesweep,
//     stable, 11-bit digits), and
//     pass 2 (k_rec_gather) gathers the centre rows and sums every output row's records in
//     registers. No float atomics except where a row straddles two fixed-size chunks; the
//     gathered bytes move at read speed, not atomic speed.
#include <stdlib.h>

#include <cmath>
#include <mutex>
#include <unordered_map>
#include <vector>

#include <rocprim/block/block_radix_sort.hpp>
#include <rocprim/block/block_scan.hpp>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>

#include "dw_common.h"

namespace {

constexpr int WAVE = 64;
constexpr int WAVES_PER_BLOCK = 4;
constexpr int CHUNK = 12;            // output rows in flight per wave
constexpr int TMAX = 256;            // max output rows per centre in records mode
constexpr int GCH = 512;             // records per pass-2 wave chunk (large batches; pass2_chunk)
constexpr int GU = 8;                // records in flight per pass-2 iteration
constexpr uint32_t TAG_SGNS = 0x53470000u;  // 'SG'

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + expf(-x)); }

// Loss terms and gradient coefficient of one output row (loss.py:14-22 + its autograd):
//   positive row: -log(clamp(sigmoid(x), 1e-6)),  d/dx = sigmoid(x) - 1  where unclamped;
//   negative row: -log(clamp(sigmoid(-x), 1e-6)), d/dx = 1 - sigmoid(-x) where unclamped;
// recall counts positives with sigmoid(x) >= 0.5, the precision tally negatives with it.
// One exp(-|x|) and one reciprocal give sigmoid(|x|) and sigmoid(-|x|) together (finite for
// every x); the hardware exp / rcp / log (a few ulp) keep the per-row dependency chain short —
// this chain, not memory, bounded pass 1 with the libm versions. The (s - 1) / (1 - s) forms
// keep the reference's rounding structure.
__device__ __forceinline__ float row_coef(float x, bool pos, float scale, float &acc_pos,
                                          float &acc_neg, float &acc_rec, float &acc_prec) {
    const float e = __expf(-fabsf(x));
    const float hi = __builtin_amdgcn_rcpf(1.0f + e);  // sigmoid(|x|)
    const float lo = e * hi;                            // sigmoid(-|x|)
    const float sp = x >= 0.f ? hi : lo;                // sigmoid(x)
    const float sy = pos ? sp : (x >= 0.f ? lo : hi);   // sigmoid(x) / sigmoid(-x)
    const float loss = -__logf(fmaxf(sy, 1e-6f));
    const float hit = sp >= 0.5f ? 1.f : 0.f;
    if (pos) {
        acc_pos += loss;
        acc_rec += hit;
    } else {
        acc_neg += loss;
        acc_prec += hit;
    }
    return sy >= 1e-6f ? (pos ? sy - 1.0f : 1.0f - sy) * scale : 0.f;
}

// Loss sums leave each block as ONE fp64 atomic per term. The four terms share one cache line,
// so same-address atomics serialise on a single L2 channel (~9 ns each measured on MI355X):
// one per wave over ~10^5 waves cost ~5 ms per batch, more than the whole row traffic. The
// launchers also cap the grid (grid-stride loops), so a batch issues a few thousand.
// Every thread of the block must reach this (no early exits in the kernels).
__device__ void flush_loss(double *acc, float p, float n, float r, float pr) {
    __shared__ float s_loss[WAVES_PER_BLOCK][4];
    p = dw::wave_sum(p);
    n = dw::wave_sum(n);
    r = dw::wave_sum(r);
    pr = dw::wave_sum(pr);
    const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
    if (lane == 0) {
        s_loss[wv][0] = p;
        s_loss[wv][1] = n;
        s_loss[wv][2] = r;
        s_loss[wv][3] = pr;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        double t = 0.0;
        for (int w = 0; w < WAVES_PER_BLOCK; ++w) t += s_loss[w][threadIdx.x];
        if (t != 0.0) atomicAdd(acc + threadIdx.x, t);
    }
}

// Pooled input vector of row b for lane element e: the mean of P input rows (P = 1: the
// centre row itself) — torch.mean over dim 1 (model.py:104), a sequential sum then / P.
__device__ __forceinline__ float pooled(const int64_t *__restrict__ inputs, int64_t b, int32_t P,
                                        const float *__restrict__ w_in, int32_t d, int e) {
    if (P == 1) return w_in[inputs[b] * d + e];
    float h = 0.f;
    for (int p = 0; p < P; ++p) h += w_in[inputs[b * P + p] * d + e];
    return h / static_cast<float>(P);
}

__device__ __forceinline__ bool inputs_ok(const int64_t *__restrict__ inputs, int64_t b,
                                          int32_t P, int64_t V) {
    bool ok = true;
    for (int p = 0; p < P; ++p) {
        const int64_t c = inputs[b * P + p];
        ok = ok && c >= 0 && c < V;
    }
    return ok;
}

struct SgnsArgs {
    // source of centres / contexts
    const int32_t *walks;     // walks mode
    int32_t L, R;
    const int64_t *inputs;    // pairs mode: [batch, n_in] (n_in > 1: mean-pooled, CBOW)
    int32_t n_in;
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
    // owner-computes form (dw_sgns_owner_pass1): only output rows o with o % n_owners == owner,
    // addressed as local row o / n_owners of w_out; wave g appends its records to its own region
    // [g * region, (g+1) * region) of rec_key / rec_val and leaves the count in rec_counts[g]
    int32_t owner, n_owners;
    int32_t own_shift;        //   log2(n_owners) when a power of two (mask / shift), else -1
    uint32_t *rec_counts;
    uint32_t *count_out;      //   n_owners == 1: the records are dense; their count goes here
    int64_t region;
    // placed records (one owner or many, after k_out_claim): slot (b, t)'s record goes to
    // place_off[row] + place_rank[b * T + t]; no regions, no compaction, no sort
    const uint32_t *place_rank = nullptr, *place_off = nullptr;
    const uint32_t *occ;      // centres in node order (k_occ_keys + sort): wave g takes
    int64_t occ_per_wave;     //   occ[g * occ_per_wave, (g+1) * occ_per_wave)
    const dw_step_scalars *dyn;   // bound step block (graph replay): noise_offset from it
    dw::Fixed fx_in{};        // deterministic mode: g_in's int64 accumulator (dw_exact_register)
};

#ifndef DW_NOISE_ROUNDS
#define DW_NOISE_ROUNDS 10  // (timing experiments only: any other value changes the stream)
#endif
// Device negatives (noise == NULL): centre b's negative n = j*K + k comes from Philox call
// m = n / 2 with counter (g, m, TAG_SGNS), g = noise_offset + b — words (x, y) for even n,
// (z, w) for odd n, each through bounded64 (uniform over [0, V) like torch.randint;
// oracle/philox.py device_noise). One call serves two negatives.
__device__ __forceinline__ dw::U4 noise_pair(const SgnsArgs &a, int64_t b, int m) {
    const uint64_t g = (a.dyn ? a.dyn->noise_offset : a.noise_offset) + static_cast<uint64_t>(b);
    return dw::philox<DW_NOISE_ROUNDS>(
        dw::U4{static_cast<uint32_t>(g), static_cast<uint32_t>(g >> 32), static_cast<uint32_t>(m),
               TAG_SGNS},
        a.k0, a.k1);
}

__device__ __forceinline__ int64_t noise_id(const SgnsArgs &a, int64_t b, int j, int k) {
    if (a.noise) return a.noise[(b * a.C + j) * a.K + k];
    const int n = j * a.K + k;
    const dw::U4 r = noise_pair(a, b, n >> 1);
    const uint64_t V = static_cast<uint64_t>(a.V);
    return static_cast<int64_t>((n & 1) ? dw::bounded64(r.z, r.w, V) : dw::bounded64(r.x, r.y, V));
}

__device__ __forceinline__ uint64_t pack_record(float coef, int64_t centre) {
    return (static_cast<uint64_t>(__float_as_uint(coef)) << 32) |
           static_cast<uint32_t>(centre);
}

// Output row t of centre b (t < T = C(1+K)): t = j(1+K) is context j, t = j(1+K)+1+k is the
// k-th negative of context j (the reference's (B', 2R) / (B', 2R, K) orders).
template <bool FROM_WALKS>
__device__ __forceinline__ int64_t row_id(const SgnsArgs &a, int64_t b, const int32_t *walk,
                                          int64_t i, int t) {
    const int rows_per_ctx = 1 + a.K;
    const int j = t / rows_per_ctx, k = t - j * rows_per_ctx - 1;
    if (k < 0) {
        if (FROM_WALKS) return walk[(j < a.R) ? (i - a.R + j) : (i + 1 + (j - a.R))];
        return a.targets[b * a.C + j];
    }
    return noise_id(a, b, j, k);
}

// VPL = values per lane (d <= 64*VPL); MASKED when d is not exactly 64*VPL.
// Work split inside a wave: every lane loads / draws the id of ONE output row (lane t <-> row
// g0 + t of the current group of 64 rows), so the Philox negatives cost one draw per lane, not
// one per row per lane; the row loop reads the ids back with v_readlane. After each chunk's
// butterfly every lane holds every logit; lane t evaluates sigmoid / log / the clamp mask for
// its own row only and the coefficients are read back per row. Records are written by the
// owning lane (coalesced), so no LDS staging is needed.
// EXACT (records only, no pooling): each centre-gradient term enters g_in's int64 accumulator
// as a fixed-point integer (dw::to_fixed) — the sum independent of the atomics' order.
template <int VPL, bool MASKED, bool FROM_WALKS, bool RECORDS, int CH, bool EXACT = false>
__global__ void __launch_bounds__(WAVES_PER_BLOCK *WAVE) k_sgns(SgnsArgs a) {
    static_assert(!EXACT || RECORDS, "the exact form writes records");
    bool range = false;   // EXACT: a term past the fixed-point range
    const int lane = threadIdx.x & (WAVE - 1);
    const int wv = threadIdx.x / WAVE;
    const int64_t n_waves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
    const int rows_per_ctx = 1 + a.K;
    const int n_rows = a.C * rows_per_ctx;

    bool live[VPL];
#pragma unroll
    for (int m = 0; m < VPL; ++m) live[m] = !MASKED || (lane + WAVE * m < a.d);

    // per-lane loss / metric partials (reduced across the wave once, at the end)
    float acc_pos = 0.f, acc_neg = 0.f, acc_rec = 0.f, acc_prec = 0.f;

    for (int64_t b = (int64_t)blockIdx.x * WAVES_PER_BLOCK + wv; b < a.batch; b += n_waves) {
        const int32_t *walk = nullptr;
        int64_t i = 0, cid;
        if (FROM_WALKS) {
            const int64_t per = a.L - 2 * a.R;
            const int64_t w = b / per;
            i = a.R + (b - w * per);
            walk = a.walks + w * a.L;
            cid = walk[i];
        } else {
            cid = a.inputs[b * a.n_in];
        }
        const bool pool = !FROM_WALKS && a.n_in > 1;  // CBOW: mean of n_in input rows
        const bool centre_ok =
            pool ? inputs_ok(a.inputs, b, a.n_in, a.V) : (cid >= 0 && cid < a.V);
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
        int64_t gx[VPL];
        const float *crow = a.w_in + cid * a.d + lane;
#pragma unroll
        for (int m = 0; m < VPL; ++m) {
            c[m] = !live[m] ? 0.f
                   : pool   ? pooled(a.inputs, b, a.n_in, a.w_in, a.d, lane + WAVE * m)
                            : crow[WAVE * m];
            gc[m] = 0.f;
            gx[m] = 0;
        }
        for (int g0 = 0; g0 < n_rows; g0 += WAVE) {
            const int g_rows = (n_rows - g0 < WAVE) ? n_rows - g0 : WAVE;
            // this lane's output row: id, kind, validity
            const int t = g0 + lane;
            int32_t my_id = 0;
            bool my_ok = false;
            const bool my_pos = (t % rows_per_ctx) == 0;
            if (lane < g_rows) {
                const int64_t id = row_id<FROM_WALKS>(a, b, walk, i, t);
                my_ok = id >= 0 && id < a.V;
                if (!my_ok) dw::status_or(a.status, DW_S_BAD_INDEX);
                my_id = my_ok ? static_cast<int32_t>(id) : 0;
            }
            float my_coef = 0.f;
            for (int r0 = 0; r0 < g_rows; r0 += CH) {
                int32_t id[CH];
                float o[CH][VPL], dot[CH];
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    const int src = (r0 + u < g_rows) ? r0 + u : 0;
                    id[u] = __builtin_amdgcn_readlane(my_id, src);
                }
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    const bool in = r0 + u < g_rows;
                    const float *row = a.w_out + static_cast<int64_t>(id[u]) * a.d + lane;
#pragma unroll
                    for (int m = 0; m < VPL; ++m) o[u][m] = (in && live[m]) ? row[WAVE * m] : 0.f;
                }
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    float s = 0.f;
#pragma unroll
                    for (int m = 0; m < VPL; ++m) s += c[m] * o[u][m];
                    dot[u] = s;
                }
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
                    for (int u = 0; u < CH; ++u) dot[u] += __shfl_xor(dot[u], off, WAVE);
                }
                // lane r0+u owns row r0+u of this chunk: its logit, loss terms and coefficient
                float x = 0.f;
#pragma unroll
                for (int u = 0; u < CH; ++u)
                    if (lane == r0 + u) x = dot[u];
                const bool mine = lane >= r0 && lane < r0 + CH && lane < g_rows && my_ok;
                float coef = 0.f;
                if (mine) {
                    coef = row_coef(x, my_pos, a.scale, acc_pos, acc_neg, acc_rec, acc_prec);
                    my_coef = coef;
                }
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    if (r0 + u >= g_rows) continue;
                    const float gs =
                        __int_as_float(__builtin_amdgcn_readlane(__float_as_int(coef), r0 + u));
#pragma unroll
                    for (int m = 0; m < VPL; ++m) {
                        if constexpr (EXACT)
                            gx[m] += dw::to_fixed(gs * o[u][m], a.fx_in.fs, range);
                        else
                            gc[m] += gs * o[u][m];
                    }
                    if (!RECORDS && gs != 0.f) {
                        float *grow = a.g_out + static_cast<int64_t>(id[u]) * a.d + lane;
#pragma unroll
                        for (int m = 0; m < VPL; ++m)
                            if (live[m]) atomicAdd(grow + WAVE * m, gs * c[m]);
                    }
                }
            }
            if (RECORDS && lane < g_rows) {  // lane t writes row t's record (coalesced)
                a.rec_key[b * n_rows + t] = static_cast<uint32_t>(my_id);
                a.rec_val[b * n_rows + t] = pack_record(my_ok ? my_coef : 0.f, cid);
            }
        }
        if (pool) {  // mean backward: each pooled input row receives gc / n_in
            for (int p = 0; p < a.n_in; ++p) {
                float *grow = a.g_in + a.inputs[b * a.n_in + p] * a.d + lane;
#pragma unroll
                for (int m = 0; m < VPL; ++m)
                    if (live[m]) atomicAdd(grow + WAVE * m, gc[m] / static_cast<float>(a.n_in));
            }
        } else if constexpr (EXACT) {
            int64_t *gxrow = a.fx_in.acc + cid * a.d + lane;
#pragma unroll
            for (int m = 0; m < VPL; ++m)
                if (live[m]) dw::fixed_add(gxrow + WAVE * m, gx[m]);
        } else {
            float *gcrow = a.g_in + cid * a.d + lane;
#pragma unroll
            for (int m = 0; m < VPL; ++m)
                if (live[m]) atomicAdd(gcrow + WAVE * m, gc[m]);
        }
    }
    if constexpr (EXACT)
        if (__ballot(range) && lane == 0) dw::status_or(a.status, DW_S_FIXED_RANGE);

    // loss partials: wave-reduce the per-lane sums, one double atomic per wave and value
    if (a.loss_acc) flush_loss(a.loss_acc, acc_pos, acc_neg, acc_rec, acc_prec);
}

// ---- pass 1, 16-lane-group form (records mode, d = 64 * F4, T <= 64) -------------------------
// One centre per 16-lane group, four centres per wave: lane gl of group q holds elements
// [4gl + 64f, 4gl + 64f + 4) of every row (float4 loads: one wave-instruction moves 1 KiB =
// four 256-B row pieces), so a logit is 4*F4 FMAs and a 16-lane DPP row-rotate reduction
// (no LDS permutes). Each group's 2R(1+K) row ids are drawn once into LDS (lane gl draws rows
// gl, gl+16, ...); per chunk of CHR rows the group loads CHR rows, lanes gl < CHR evaluate the
// loss / clamp mask / coefficient of row gl (one transcendental pass per chunk, not per row)
// and the coefficients come back by ds_bpermute. The centre gradient is staged in LDS and
// added as full 256-B wave-instruction atomics; records are written by their owning lanes.
constexpr int G16_TMAX = 64;
#ifndef G16_MIN_WAVES
#define G16_MIN_WAVES 4  // waves per SIMD the register allocation must allow (no spills)
#endif

template <int N>
__device__ __forceinline__ float row_ror(float x) {  // lane i <- lane (i +- N) mod 16 of its row
    return __int_as_float(
        __builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x120 + N, 0xF, 0xF, false));
}

__device__ __forceinline__ float row_sum16(float x) {
    x += row_ror<8>(x);
    x += row_ror<4>(x);
    x += row_ror<2>(x);
    x += row_ror<1>(x);
    return x;
}

// OWNER (dw_sgns_owner_pass1, N > 1): the group keeps only the output rows this rank owns
// (o % n_owners == owner), compacted to the front of its id list in slot order (s_t keeps each
// one's slot t for the positive / negative rule), so the chunk loop gathers ~T / n_owners rows
// from the rank's local slice of the out table. Each wave appends its records to a region of
// its own (sized for every slot of its iterations), counted in a register: no atomics (a
// shared counter took one same-address atomic per wave iteration — ~12 ns each, serialised:
// 14 ms per pass at 8 owners); k_rec_compact packs the regions afterwards.
// Every rank forms every centre of the global batch, so at W owners the centre-gradient atomics
// grow W-fold (2.35 GB per pass at W = 8, C3). The owner form therefore takes the centres in
// node order (a sorted occurrence list, contiguous per wave): consecutive occurrences of one
// node are summed in registers (pend) and leave as ONE atomic row per run.
// EXACT: the centre-gradient terms enter g_in's int64 accumulator as fixed-point integers
// (dw::to_fixed), each lane adding its 4 F4 elements of its group's centre straight from
// registers (no LDS staging, no run summing: integer sums need no order).
// COEFIN (the rows-major step, after k_out_rows; one owner or many, placed records): slot
// b T + t's coefficient is already in ((float *) rec_val)[b T + t] and its row holds its
// pre-step values p^{s-1} (k_out_rows leaves the rows it steps pending: m and v at step s, the
// parameter half deferred): only the centre gradient is formed — the same FMAs in the same
// order as the full pass.
template <int F4, bool FROM_WALKS, int CHR, bool OWNER, bool EXACT = false, bool COEFIN = false>
__global__ void __launch_bounds__(WAVES_PER_BLOCK *WAVE, CHR >= 8 ? 3 : G16_MIN_WAVES)
    k_sgns_g16(SgnsArgs a) {
    static_assert(!COEFIN || OWNER, "the coefficients-in form is the owner path's");
    constexpr int D = 64 * F4;
    __shared__ int32_t s_id[WAVES_PER_BLOCK][4][G16_TMAX];
    __shared__ float s_coef[WAVES_PER_BLOCK][4][G16_TMAX];
    __shared__ uint8_t s_t[WAVES_PER_BLOCK][4][OWNER ? G16_TMAX : 1];
    __shared__ float4 s_g[WAVES_PER_BLOCK][4][EXACT ? 1 : 16 * F4];
    __shared__ int64_t s_gx[WAVES_PER_BLOCK][EXACT ? D : 1];   // EXACT: one centre's sums
    bool range = false;   // EXACT: a term past the fixed-point range
    uint32_t tmax = 0u;   // EXACT: the largest |term|'s bits (the range test, once at the end)
    const int lane = threadIdx.x & (WAVE - 1);
    const int wv = threadIdx.x / WAVE;
    const int q = lane >> 4, gl = lane & 15;
    const int rows_per_ctx = 1 + a.K;
    const int T = a.C * rows_per_ctx;
    const int64_t n_slots = (int64_t)gridDim.x * WAVES_PER_BLOCK * 4;
    float acc_pos = 0.f, acc_neg = 0.f, acc_rec = 0.f, acc_prec = 0.f;
    int64_t filled = 0;  // OWNER: records in this wave's region so far (wave-uniform)
    const int64_t gw = (int64_t)blockIdx.x * WAVES_PER_BLOCK + wv;
    int64_t o_end = a.batch, step = n_slots, base0 = gw * 4;
    if constexpr (OWNER) {  // this wave's slice of the node-ordered occurrences
        base0 = gw * a.occ_per_wave;
        o_end = base0 + a.occ_per_wave < a.batch ? base0 + a.occ_per_wave : a.batch;
        step = 4;
    }
    int32_t pend_c = -1;  // OWNER: node whose centre gradient is being summed (wave-uniform)
    float pend[F4];
#pragma unroll
    for (int f = 0; f < F4; ++f) pend[f] = 0.f;

    for (int64_t base = base0; base < o_end; base += step) {
        const int64_t jb = base + q;
        // (OWNER with occ NULL: the centres in walk order — the rows-major step's centre pass)
        const int64_t b0 =
            OWNER ? (jb < o_end ? (a.occ ? static_cast<int64_t>(a.occ[jb]) : jb) : 0) : jb;
        // an order entry outside the batch (an order never built for these walks) reads no walk
        const bool bad_b = OWNER && jb < o_end && (b0 < 0 || b0 >= a.batch);
        if (bad_b && gl == 0) dw::status_or(a.status, DW_S_BAD_INDEX);
        const bool active = jb < o_end && !bad_b;
        const int64_t b = bad_b ? 0 : b0;
        const int32_t *walk = nullptr;
        int64_t i = 0, cid = -1;
        if (active) {
            if (FROM_WALKS) {
                const int64_t per = a.L - 2 * a.R;
                const int64_t w = b / per;
                i = a.R + (b - w * per);
                walk = a.walks + w * a.L;
                cid = walk[i];
            } else {
                cid = a.inputs[b];
            }
        }
        const bool ok_c = active && cid >= 0 && cid < a.V;
        if (active && !ok_c && gl == 0) dw::status_or(a.status, DW_S_BAD_INDEX);
        // the group's row ids (-1 = invalid row: zero coefficient)
        int n_own = T;  // rows in the group's list (OWNER: the owned ones, compacted)
        if constexpr (OWNER) {
            // staged in LDS by slot t first (in s_coef, free until the coefficients): contexts
            // from the walk, negatives two per Philox call (noise_pair) — the 16 lanes draw the
            // C*K/2 calls, so a centre costs ceil(C*K/32) Philox per lane, not ceil(T/16). Every
            // rank draws every centre's negatives and keeps ~1/W of them: at W = 8 the draws are
            // a visible share of pass 1.
            int32_t *stage = reinterpret_cast<int32_t *>(&s_coef[wv][q][0]);
            for (int t = gl; t < T; t += 16) stage[t] = -1;
            if (ok_c) {
                const int n_neg = a.C * a.K;
                auto put = [&](int n, int64_t r) {   // negative n -> slot t
                    const int jn = n / a.K;
                    const int t = jn * rows_per_ctx + 1 + (n - jn * a.K);
                    if (r >= 0 && r < a.V)
                        stage[t] = static_cast<int32_t>(r);
                    else
                        dw::status_or(a.status, DW_S_BAD_INDEX);
                };
                for (int j = gl; j < a.C; j += 16) {   // contexts
                    const int64_t r = row_id<FROM_WALKS>(a, b, walk, i, j * rows_per_ctx);
                    if (r >= 0 && r < a.V)
                        stage[j * rows_per_ctx] = static_cast<int32_t>(r);
                    else
                        dw::status_or(a.status, DW_S_BAD_INDEX);
                }
                if (a.noise) {   // replayed negatives
                    for (int n = gl; n < n_neg; n += 16) put(n, a.noise[b * n_neg + n]);
                } else {
                    const uint64_t Vu = static_cast<uint64_t>(a.V);
#pragma unroll 2
                    for (int m = gl; 2 * m < n_neg; m += 16) {
                        const dw::U4 r = noise_pair(a, b, m);
                        put(2 * m, static_cast<int64_t>(dw::bounded64(r.x, r.y, Vu)));
                        if (2 * m + 1 < n_neg)
                            put(2 * m + 1, static_cast<int64_t>(dw::bounded64(r.z, r.w, Vu)));
                    }
                }
            }
            dw::wave_lds_sync();
            n_own = 0;
#pragma unroll
            for (int k = 0; k < G16_TMAX / 16; ++k) {
                const int t = gl + 16 * k;
                const int32_t id = t < T ? stage[t] : -1;
                // owner o % W, local row o / W (shift and mask for the usual W = 2, 4, 8)
                const int32_t lrow = a.own_shift >= 0 ? (id >> a.own_shift) : id / a.n_owners;
                const int32_t orow = id - lrow * a.n_owners;
                // one owner keeps every slot of an active centre, a bad id as a zero record:
                // the per-wave regions then tile [0, batch * T) densely (no compaction)
                const bool own = (id >= 0 && orow == a.owner) ||
                                 (a.n_owners == 1 && active && t < T);
                const uint32_t grp =
                    static_cast<uint32_t>(__ballot(own) >> (16 * q)) & 0xFFFFu;
                if (own) {
                    const int pos = n_own + __popc(grp & ((1u << gl) - 1u));
                    s_id[wv][q][pos] = lrow;
                    s_t[wv][q][pos] = static_cast<uint8_t>(t);
                }
                n_own += __popc(grp);
            }
        } else {
            // one Philox per lane and row (two Philox draws overlap); one device, memory-bound
#pragma unroll 2
            for (int k = 0; k < G16_TMAX / 16; ++k) {
                const int t = gl + 16 * k;
                int32_t id = -1;
                if (t < T && ok_c) {
                    const int64_t r = row_id<FROM_WALKS>(a, b, walk, i, t);
                    if (r >= 0 && r < a.V)
                        id = static_cast<int32_t>(r);
                    else
                        dw::status_or(a.status, DW_S_BAD_INDEX);
                }
                if (t < T) {
                    s_id[wv][q][t] = id;
                    s_coef[wv][q][t] = 0.f;
                }
            }
        }
        // rows the chunk loop runs over: wave-uniform (the longest of the four groups' lists)
        int n_loop = T;
        if constexpr (OWNER) {
            const int c0 = __builtin_amdgcn_readlane(n_own, 0);
            const int c1 = __builtin_amdgcn_readlane(n_own, 16);
            const int c2 = __builtin_amdgcn_readlane(n_own, 32);
            const int c3 = __builtin_amdgcn_readlane(n_own, 48);
            n_loop = max(max(c0, c1), max(c2, c3));
        }
        float4 c4[F4], g4[F4];
        int64_t gx[EXACT ? 4 * F4 : 1];
        const float *crow = a.w_in + (ok_c ? cid : 0) * D + 4 * gl;
#pragma unroll
        for (int f = 0; f < F4; ++f) {
            c4[f] = ok_c ? *reinterpret_cast<const float4 *>(crow + 64 * f)
                         : make_float4(0.f, 0.f, 0.f, 0.f);
            g4[f] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int k = 0; k < (EXACT ? 4 * F4 : 1); ++k) gx[k] = 0;
        dw::wave_lds_sync();
        auto load_chunk = [&](float4(&o4)[CHR][F4], int32_t(&rid)[CHR], int t0) {
#pragma unroll
            for (int u = 0; u < CHR; ++u) {
                const int t = t0 + u;
                rid[u] = (t < n_own) ? s_id[wv][q][t] : -1;
                // (COEFIN: the table row holds p^{s-1}, k_out_rows left it pending)
                const int64_t at = rid[u] < 0 ? 0 : static_cast<int64_t>(rid[u]);
                const float *row = a.w_out + at * D + 4 * gl;
#pragma unroll
                for (int f = 0; f < F4; ++f)
                    o4[u][f] = rid[u] >= 0 ? *reinterpret_cast<const float4 *>(row + 64 * f)
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        };
        auto compute_chunk = [&](const float4(&o4)[CHR][F4], const int32_t(&rid)[CHR],
                                 int t0) {
            float dot[CHR];
            if constexpr (!COEFIN) {
#pragma unroll
                for (int u = 0; u < CHR; ++u) {
                    float p = 0.f;
#pragma unroll
                    for (int f = 0; f < F4; ++f) {
                        p = fmaf(c4[f].x, o4[u][f].x, p);
                        p = fmaf(c4[f].y, o4[u][f].y, p);
                        p = fmaf(c4[f].z, o4[u][f].z, p);
                        p = fmaf(c4[f].w, o4[u][f].w, p);
                    }
                    dot[u] = row_sum16(p);
                }
            }
            // lane gl < CHR owns row t0 + gl of its group
            float x = 0.f;
            int32_t xid = -1;
#pragma unroll
            for (int u = 0; u < CHR; ++u)
                if (gl == u) {
                    if constexpr (!COEFIN) x = dot[u];
                    xid = rid[u];
                }
            float coef = 0.f;
            const int t = t0 + gl;
            if (gl < CHR && t < n_own && xid >= 0) {
                const int slot = OWNER ? static_cast<int>(s_t[wv][q][t]) : t;
                if constexpr (COEFIN) {
                    coef = reinterpret_cast<const float *>(a.rec_val)[b * T + slot];
                } else {
                    coef = row_coef(x, (slot % rows_per_ctx) == 0, a.scale, acc_pos, acc_neg,
                                    acc_rec, acc_prec);
                    s_coef[wv][q][t] = coef;
                }
            }
#pragma unroll
            for (int u = 0; u < CHR; ++u) {
                const float cu = __shfl(coef, (q << 4) | u, WAVE);
                if constexpr (EXACT) {
                    const double fs = a.fx_in.fs;
#pragma unroll
                    for (int f = 0; f < F4; ++f) {
                        const float t0 = cu * o4[u][f].x, t1 = cu * o4[u][f].y;
                        const float t2 = cu * o4[u][f].z, t3 = cu * o4[u][f].w;
                        gx[4 * f + 0] += dw::fixed_bits(t0, fs);
                        gx[4 * f + 1] += dw::fixed_bits(t1, fs);
                        gx[4 * f + 2] += dw::fixed_bits(t2, fs);
                        gx[4 * f + 3] += dw::fixed_bits(t3, fs);
                        tmax = dw::fixed_track(dw::fixed_track(tmax, t0), t1);
                        tmax = dw::fixed_track(dw::fixed_track(tmax, t2), t3);
                    }
                    continue;
                }
#pragma unroll
                for (int f = 0; f < F4; ++f) {
                    g4[f].x = fmaf(cu, o4[u][f].x, g4[f].x);
                    g4[f].y = fmaf(cu, o4[u][f].y, g4[f].y);
                    g4[f].z = fmaf(cu, o4[u][f].z, g4[f].z);
                    g4[f].w = fmaf(cu, o4[u][f].w, g4[f].w);
                }
            }
        };
        // (a software-pipelined variant — next chunk in flight — and 2- / 8-row chunks measured
        // the same on MI355X: the kernel is HBM-bound once the loss atomics were removed)
        for (int t0 = 0; t0 < n_loop; t0 += CHR) {
            float4 o4[CHR][F4];
            int32_t rid[CHR];
            load_chunk(o4, rid, t0);
            compute_chunk(o4, rid, t0);
        }
        if constexpr (EXACT) {   // every chunk added CHR terms per element
            const int64_t nt = static_cast<int64_t>((n_loop + CHR - 1) / CHR) * CHR;
#pragma unroll
            for (int k = 0; k < 4 * F4; ++k) gx[k] = dw::fixed_finish(gx[k], nt);
        }
        if constexpr (!EXACT) {
#pragma unroll
            for (int f = 0; f < F4; ++f) s_g[wv][q][gl + 16 * f] = g4[f];
        }
        dw::wave_lds_sync();
        if constexpr (COEFIN) {
            // (no records: k_out_rows wrote them)
        } else if constexpr (OWNER) {  // the wave's owned records, appended to its region
            const int c0 = __builtin_amdgcn_readlane(n_own, 0);
            const int c1 = __builtin_amdgcn_readlane(n_own, 16);
            const int c2 = __builtin_amdgcn_readlane(n_own, 32);
            const int c3 = __builtin_amdgcn_readlane(n_own, 48);
            const int64_t at = ((int64_t)blockIdx.x * WAVES_PER_BLOCK + wv) * a.region + filled +
                               (q == 0 ? 0 : q == 1 ? c0 : q == 2 ? c0 + c1 : c0 + c1 + c2);
#pragma unroll
            for (int k = 0; k < G16_TMAX / 16; ++k) {
                const int tt = gl + 16 * k;
                if (tt < n_own) {
                    const int32_t id = s_id[wv][q][tt];   // < 0: a bad id (one owner only)
                    if (a.place_off) {   // placed: k_out_claim counted only the valid rows
                        if (id >= 0) {
                            const uint32_t pos = a.place_off[id] +
                                                 a.place_rank[b * T + s_t[wv][q][tt]];
                            a.rec_key[pos] = static_cast<uint32_t>(id);
                            a.rec_val[pos] = pack_record(s_coef[wv][q][tt], ok_c ? cid : 0);
                        }
                    } else {
                        a.rec_key[at + tt] = static_cast<uint32_t>(id < 0 ? 0 : id);
                        a.rec_val[at + tt] = pack_record(id < 0 ? 0.f : s_coef[wv][q][tt],
                                                         ok_c ? cid : 0);
                    }
                }
            }
            filled += c0 + c1 + c2 + c3;
        } else if (active) {  // records: lane gl writes rows gl, gl+16, ... of its centre
#pragma unroll
            for (int k = 0; k < G16_TMAX / 16; ++k) {
                const int tt = gl + 16 * k;
                if (tt < T) {
                    const int32_t id = s_id[wv][q][tt];
                    a.rec_key[b * T + tt] = static_cast<uint32_t>(id < 0 ? 0 : id);
                    a.rec_val[b * T + tt] = pack_record(s_coef[wv][q][tt], ok_c ? cid : 0);
                }
            }
        }
        if constexpr (EXACT) {
            // the four centres one after the other through the wave's LDS row: each centre's
            // sums leave as F4 coalesced 64-lane int64 atomics (512 contiguous bytes each) where
            // the group's own layout (elements 4 gl + 64 f + k) gave 4 F4 atomics per lane at a
            // 32-B stride over four centres — a quarter of the cache-line requests
            const int32_t cq_self = (ok_c && n_own > 0) ? static_cast<int32_t>(cid) : -1;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                const int32_t cq = __builtin_amdgcn_readlane(cq_self, qq * 16);
                if (cq < 0) continue;
                if (q == qq) {
#pragma unroll
                    for (int f = 0; f < F4; ++f)
#pragma unroll
                        for (int k = 0; k < 4; ++k) s_gx[wv][64 * f + 4 * gl + k] = gx[4 * f + k];
                }
                dw::wave_lds_sync();
                int64_t *dst = a.fx_in.acc + static_cast<int64_t>(cq) * D + lane;
#pragma unroll
                for (int f = 0; f < F4; ++f) dw::fixed_add(dst + 64 * f, s_gx[wv][lane + 64 * f]);
                dw::wave_lds_sync();
            }
            dw::wave_lds_sync();
            continue;
        }
        // centre gradients: per centre, 64 lanes x dword = 256 contiguous bytes per atomic
        const float *sg_flat = reinterpret_cast<const float *>(&s_g[wv][0][0]);
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
            const int32_t cq = __builtin_amdgcn_readlane(
                ok_c && n_own > 0 ? static_cast<int32_t>(cid) : -1, qq * 16);
            if constexpr (OWNER) {  // sum runs of one node, one atomic row per run
                if (cq < 0) continue;
                if (cq != pend_c) {
                    if (pend_c >= 0) {
                        float *dst = a.g_in + static_cast<int64_t>(pend_c) * D + lane;
#pragma unroll
                        for (int f = 0; f < F4; ++f) atomicAdd(dst + 64 * f, pend[f]);
                    }
                    pend_c = cq;
#pragma unroll
                    for (int f = 0; f < F4; ++f) pend[f] = 0.f;
                }
                // element 64f + lane sits in float4 slot (lane >> 2) + 16f, component lane & 3
#pragma unroll
                for (int f = 0; f < F4; ++f)
                    pend[f] += sg_flat[qq * 16 * F4 * 4 + ((lane >> 2) + 16 * f) * 4 + (lane & 3)];
                continue;
            }
            if (cq >= 0) {
                float *dst = a.g_in + static_cast<int64_t>(cq) * D;
                // s_g[qq] holds float4 slot j = gl + 16f -> elements 4gl + 64f .. +3
#pragma unroll
                for (int e0 = 0; e0 < D; e0 += WAVE) {
                    const int e = e0 + lane;
                    const int f = e >> 6, g = (e & 63) >> 2, comp = e & 3;
                    atomicAdd(dst + e, sg_flat[qq * 16 * F4 * 4 + (g + 16 * f) * 4 + comp]);
                }
            }
        }
        dw::wave_lds_sync();
    }
    if constexpr (EXACT) {
        range = range || dw::fixed_range(tmax, a.fx_in.fs);
        if (__ballot(range) && lane == 0) dw::status_or(a.status, DW_S_FIXED_RANGE);
    }
    if constexpr (OWNER) {
        if (!EXACT && pend_c >= 0) {
            float *dst = a.g_in + static_cast<int64_t>(pend_c) * D + lane;
#pragma unroll
            for (int f = 0; f < F4; ++f) atomicAdd(dst + 64 * f, pend[f]);
        }
        if (!COEFIN && lane == 0) a.rec_counts[gw] = static_cast<uint32_t>(filled);
        if (!COEFIN && a.count_out && blockIdx.x == 0 && threadIdx.x == 0)
            *a.count_out = static_cast<uint32_t>(a.batch * T);
    }
    if (a.loss_acc) flush_loss(a.loss_acc, acc_pos, acc_neg, acc_rec, acc_prec);
}

// Pass 2: records sorted by output row -> g_out[row] += sum coef * w_in[centre].
// Each wave owns a fixed chunk of gch sorted records (GCH = 512; smaller for small batches),
// balanced whatever the row lengths (hub rows hold thousands). A row wholly inside the chunk is summed in registers and added
// with a plain read-modify-write (the chunk is its only writer); the first / last row of a
// chunk may continue in the neighbouring chunk and is added with float atomics.
// Output-table Adam fused in (ADAM, one device: dw_sgns_walks_phase2_adam): a row wholly
// inside the chunk has its complete gradient in registers, so it is updated right there
// (torch Adam, dw::adam_elem, the same code as dw_adam_dense) and flagged; g_out is never
// touched for it. Boundary rows still accumulate into g_out and are updated, with the rows no
// record touched (g = 0), by k_adam_rest.
// Lazy form (last != nullptr; dw_sgns_owner_pass2_lazy): rows no record touched are not
// updated at all; a row's deferred g = 0 steps (last[row] + 1 .. step - 1, scalars from `hist`)
// are replayed right before its update, through the same adam_elem — bit-identical to the dense
// update (k_rows_adam's rule). Boundary rows then go through k_lazy_boundary, not k_adam_rest.
struct OutAdam {
    float *p, *m, *v;
    uint8_t *flags;
    dw::AdamScalars s;
    int32_t *last = nullptr;
    const float *hist = nullptr;
    int32_t step = 0;
    const dw_step_scalars *dyn = nullptr;   // bound step block: the scalars come from it
    int32_t step_delta = 0;                 //   lazy form: step = dyn->step + step_delta
    bool p_current = false;   // lazy form: the catch-up brought p (not m, v, last) to step - 1
    bool betas_const = false; //   and every step had the same betas: m, v replay with step's
    uint32_t *counts = nullptr;   // placed records: the rows' counts, cleared as they step
    // the rows-major step (dw_sgns_owner_out_rows): rows end PENDING — m, v at `step`, p at
    // step - 1 (the centre pass then reads p^{s-1} from the table itself), pend[row] = 1; a
    // pending row is settled (dw::settle_pending) before its next replay
    uint8_t *pend = nullptr;
};

// One row's lazy Adam step (one wave, VPL elements per lane): replay the missed steps, apply
// `step` (oa.step, or the bound block's) with g (registers), record the step.
template <int VPL, bool MASKED>
__device__ __forceinline__ void lazy_row_step(const OutAdam &oa, int32_t step, uint32_t row,
                                              int32_t d, int lane, const float (&g)[VPL]) {
    // (row is wave-uniform; lanes past d carry zeros through a uniform replay loop)
    const int32_t from = __builtin_amdgcn_readfirstlane(oa.last[row]);
    const bool pd = oa.pend && __builtin_amdgcn_readfirstlane(oa.pend[row]) != 0;
    const int64_t o = static_cast<int64_t>(row) * d + lane;
    float pp[VPL], mm[VPL], vv[VPL], gg[VPL];
#pragma unroll
    for (int m = 0; m < VPL; ++m) {
        const bool live = !MASKED || lane + WAVE * m < d;
        const int64_t i = o + WAVE * m;
        pp[m] = live ? oa.p[i] : 0.f;
        mm[m] = live ? oa.m[i] : 0.f;
        vv[m] = live ? oa.v[i] : 0.f;
        gg[m] = g[m];
    }
    if (oa.p_current) {
        // p is at step - 1 already (the p-only catch-up): m and v replay their g = 0 steps — the
        // same two IEEE operations adam_elem_g0 applies to them, one multiply-add each (the
        // host enables this only while every step has weight_decay 0: then m, v never read p);
        // with constant betas the scalars are this step's (no history load per step)
        if (oa.betas_const) {
            const float *h = oa.hist + 8 * static_cast<int64_t>(step);
            const float w1 = h[0], b2 = h[1];
            for (int32_t t = from + 1; t < step; ++t) {
#pragma unroll
                for (int m = 0; m < VPL; ++m) {
#pragma clang fp contract(off)
                    mm[m] = fmaf(w1, -mm[m], mm[m]);
                    vv[m] = vv[m] * b2;
                }
            }
        } else {
            for (int32_t t = from + 1; t < step; ++t) {
                const float *h = oa.hist + 8 * static_cast<int64_t>(t);
                const float w1 = h[0], b2 = h[1];
#pragma unroll
                for (int m = 0; m < VPL; ++m) {
#pragma clang fp contract(off)
                    mm[m] = fmaf(w1, -mm[m], mm[m]);
                    vv[m] = vv[m] * b2;
                }
            }
        }
    } else {
        const int32_t box_from = dw::hist_box_from(oa.hist);
        if (pd) dw::settle_pending(pp, mm, vv, oa.hist, from, box_from);
        dw::replay_g0(pp, mm, vv, oa.hist, from, step - 1, box_from);
    }
    const dw::AdamScalars h = dw::hist_at(oa.hist, step);
#pragma unroll
    for (int m = 0; m < VPL; ++m) {
        if (MASKED && lane + WAVE * m >= d) continue;
        if (oa.pend)   // the rows-major step's boundary rows: leave the parameter half pending
            dw::adam_mv(pp[m], gg[m], mm[m], vv[m], h);
        else
            dw::adam_elem(pp[m], gg[m], mm[m], vv[m], h);
        const int64_t i = o + WAVE * m;
        oa.p[i] = pp[m];
        oa.m[i] = mm[m];
        oa.v[i] = vv[m];
    }
    if (lane == 0) {
        oa.last[row] = step;
        if (oa.counts) oa.counts[row] = 0u;   // placed records: the count back to zero
        if (oa.pend && !pd) oa.pend[row] = 1;   // (already 1 where it was pending)
    }
}

// range (row pieces, dw_sgns_walks_phase2_piece): only records [range[0], range[1]) — the
// records of whole rows, so a piece's rows never continue in another piece's chunks.
// EXACT: each term coef * w_in enters the row's int64 sum as a fixed-point integer (fo); a row
// inside the chunk converts its exact sum back to float for the update, a straddling row adds
// its integer part into fo.acc (k_fixed_boundary converts it once every chunk has).
template <int VPL, bool MASKED, bool ADAM, bool EXACT = false>
__global__ void __launch_bounds__(WAVES_PER_BLOCK *WAVE)
    k_rec_gather(const uint32_t *__restrict__ keys, const uint64_t *__restrict__ vals,
                 int64_t n_rec, const float *__restrict__ w_in, float *__restrict__ g_out,
                 int32_t d, OutAdam oa, const int64_t *__restrict__ range, int32_t gch,
                 dw::Fixed fo, int32_t *status) {
    bool fx_range = false;
    uint32_t fx_tmax = 0u;   // EXACT: the largest |term|'s bits (the range test, at the end)
    const int lane = threadIdx.x & (WAVE - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
    const int64_t lo = range ? range[0] : 0;
    const int64_t hi = range ? range[1] : n_rec;
    const int64_t n_chunks = (hi - lo + gch - 1) / gch;
    const dw::AdamScalars sc = ADAM ? dw::step_adam(oa.dyn, oa.s) : oa.s;
    const int32_t lstep = dw::eff_step(oa.dyn, oa.step_delta, oa.step);   // lazy form's step
    const int64_t n_waves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
    bool live[VPL];
#pragma unroll
    for (int m = 0; m < VPL; ++m) live[m] = !MASKED || (lane + WAVE * m < d);

    for (int64_t ch = (int64_t)blockIdx.x * WAVES_PER_BLOCK + wv; ch < n_chunks; ch += n_waves) {
        const int64_t e0 = lo + ch * gch;
        const int64_t e1 = (e0 + gch < hi) ? e0 + gch : hi;
        const uint32_t before = e0 > lo ? keys[e0 - 1] : 0xFFFFFFFFu;
        const uint32_t after = e1 < hi ? keys[e1] : 0xFFFFFFFFu;
        // lanes past the chunk's end repeat its LAST key: a partial final group must not switch
        // `cur` back to an earlier row (that flushed the row a second time, with g = 0 — an extra
        // Adam step in the fused form)
        const uint32_t last = keys[e1 - 1];
        uint32_t cur = keys[e0];
        float g[VPL];
        int64_t gx[VPL];
#pragma unroll
        for (int m = 0; m < VPL; ++m) {
            g[m] = 0.f;
            gx[m] = 0;
        }

        int64_t nt = 0;   // EXACT: the terms added to gx since the row began
        auto flush = [&](uint32_t row) {
            float *dst = g_out + static_cast<int64_t>(row) * d + lane;
            if constexpr (EXACT) {
#pragma unroll
                for (int m = 0; m < VPL; ++m) gx[m] = dw::fixed_finish(gx[m], nt);
                if (row == before || row == after) {   // the integer part of a straddling row
                    int64_t *acc = fo.acc + static_cast<int64_t>(row) * d + lane;
#pragma unroll
                    for (int m = 0; m < VPL; ++m)
                        if (live[m]) dw::fixed_add(acc + WAVE * m, gx[m]);
                    return;
                }
#pragma unroll
                for (int m = 0; m < VPL; ++m) g[m] = dw::from_fixed(gx[m], fo.fi);
            }
            if (row != before && row != after) {
                if (ADAM && oa.last) {
                    lazy_row_step<VPL, MASKED>(oa, lstep, row, d, lane, g);
                } else if (ADAM) {
                    const int64_t o = static_cast<int64_t>(row) * d + lane;
#pragma unroll
                    for (int m = 0; m < VPL; ++m) {
                        if (!live[m]) continue;
                        const int64_t i = o + WAVE * m;
                        float pp = oa.p[i], gg = g[m], mm = oa.m[i], vv = oa.v[i];
                        dw::adam_elem(pp, gg, mm, vv, sc);
                        oa.p[i] = pp;
                        oa.m[i] = mm;
                        oa.v[i] = vv;
                    }
                    if (lane == 0) oa.flags[row] = 1;
                } else {
#pragma unroll
                    for (int m = 0; m < VPL; ++m)
                        if (live[m]) dst[WAVE * m] += g[m];
                }
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
                k[u] = in ? keys[e + u] : last;
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
                    nt = 0;
#pragma unroll
                    for (int m = 0; m < VPL; ++m) {
                        g[m] = 0.f;
                        gx[m] = 0;
                    }
                }
                ++nt;
#pragma unroll
                for (int m = 0; m < VPL; ++m) {
                    if constexpr (EXACT) {
                        const float t = coef[u] * x[u][m];
                        gx[m] += dw::fixed_bits(t, fo.fs);
                        fx_tmax = dw::fixed_track(fx_tmax, t);
                    } else {
                        g[m] += coef[u] * x[u][m];
                    }
                }
            }
        }
        flush(cur);
    }
    if constexpr (EXACT) {
        fx_range = fx_range || dw::fixed_range(fx_tmax, fo.fs);
        if (__ballot(fx_range) && lane == 0) dw::status_or(status, DW_S_FIXED_RANGE);
    }
}

// Deterministic mode, after k_rec_gather: the rows that straddle chunks hold their sums in the
// int64 accumulator; each such row converts once (the first and last rows of every chunk are
// visited, the per-element exchange hands each value to exactly one of the visitors, which
// adds it to g_out; the others add nothing), before k_adam_rest / k_lazy_boundary read g_out.
__global__ void __launch_bounds__(WAVES_PER_BLOCK *WAVE)
    k_fixed_boundary(const uint32_t *__restrict__ keys, int64_t n_rec, int32_t gch,
                     const int64_t *__restrict__ range, dw::Fixed fo, float *__restrict__ g_out,
                     int32_t d) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t lo = range ? range[0] : 0;
    const int64_t hi = range ? range[1] : n_rec;
    const int64_t n_chunks = (hi - lo + gch - 1) / gch;
    const int64_t n_waves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
    for (int64_t ch = (int64_t)blockIdx.x * WAVES_PER_BLOCK + threadIdx.x / WAVE; ch < n_chunks;
         ch += n_waves) {
        const int64_t e0 = lo + ch * gch;
        const int64_t e1 = (e0 + gch < hi) ? e0 + gch : hi;
        const uint32_t first = keys[e0], last = keys[e1 - 1];
        const bool a = e0 > lo && keys[e0 - 1] == first;
        const bool b = e1 < hi && keys[e1] == last;
        for (int k = 0; k < 2; ++k) {
            if (!(k == 0 ? a : b)) continue;
            const int64_t o = static_cast<int64_t>(k == 0 ? first : last) * d;
            for (int e = lane; e < d; e += WAVE) {
                const unsigned long long v =
                    atomicExch(reinterpret_cast<unsigned long long *>(fo.acc + o + e), 0ull);
                if (v) atomicAdd(g_out + o + e, dw::from_fixed(static_cast<int64_t>(v), fo.fi));
            }
        }
    }
}

// Deterministic mode, after pass 1: every centre's row of the int64 accumulator converted into
// g_in (the same exchange rule as k_fixed_boundary: one visitor per element adds the value).
template <bool FROM_WALKS>
__global__ void __launch_bounds__(WAVES_PER_BLOCK *WAVE) k_fixed_centres(SgnsArgs a) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t n_waves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
    for (int64_t b = (int64_t)blockIdx.x * WAVES_PER_BLOCK + threadIdx.x / WAVE; b < a.batch;
         b += n_waves) {
        int64_t cid;
        if (FROM_WALKS) {
            const int64_t per = a.L - 2 * a.R;
            const int64_t w = b / per;
            cid = a.walks[w * a.L + a.R + (b - w * per)];
        } else {
            cid = a.inputs[b];
        }
        if (cid < 0 || cid >= a.V) continue;
        const int64_t o = cid * a.d;
        for (int e = lane; e < a.d; e += WAVE) {
            const unsigned long long v =
                atomicExch(reinterpret_cast<unsigned long long *>(a.fx_in.acc + o + e), 0ull);
            if (v) atomicAdd(a.g_in + o + e, dw::from_fixed(static_cast<int64_t>(v), a.fx_in.fi));
        }
    }
}

// Dense conversion (dw_fixed_to_float): g = (accumulate ? g : 0) + fl(acc), acc = 0.
__global__ void k_fixed_dense(int64_t *__restrict__ acc, float *__restrict__ g, int64_t n,
                              double fi, int32_t accumulate) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t v = acc[i];
        if (v) acc[i] = 0;
        const float f = dw::from_fixed(v, fi);
        if (accumulate) {
            if (v) g[i] += f;
        } else {
            g[i] = f;
        }
    }
}

int end_bit_for(int64_t V) {
    int bits = 1;
    while (bits < 32 && (static_cast<uint64_t>(V - 1) >> bits) != 0) ++bits;
    return bits;
}

constexpr int MAX_PIECES = 1024;  // row pieces of dw_sgns_walks_phase2_piece
constexpr int MAX_OWNER_WAVES = 1 << 16;  // pass-1 waves of the owner form (grid_cap(8) * 4)

struct Workspace {
    uint32_t *k0, *k1;
    uint64_t *v0, *v1;
    int64_t *bounds;  // [MAX_PIECES + 1] record bounds of the row pieces
    uint32_t *count;  // records of the owner form (dw_sgns_owner_pass1), after compaction
    uint32_t *wave_counts;   // [MAX_OWNER_WAVES] records per pass-1 wave region (owner form)
    int64_t *wave_offsets;   // [MAX_OWNER_WAVES] their exclusive prefix sums
    void *cub;
    size_t cub_bytes;
    size_t total;
};

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Records sort: onesweep with 11-bit digits on 1024 x 16 tiles — 2 passes for C3's 21-bit row
// ids (the gfx950 default, 8-bit digits on 1024 x 8, needs 3): 0.79 ms vs 1.09 ms for 34.4M
// records on MI355X (scripts/microbench/sort_bench.hip).
// Merge-sort limit 0: rocprim's default sends up to 1M items through its merge sort, which at
// the reference's batch shape (64 walks: 269K records) ran as 20 launches and 120 us.
using RecordSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 16>,
                                        rocprim::kernel_config<1024, 16>, 11,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;
// Smaller sorts (under SMALL_SORT_MAX items): 16K-item tiles leave most of the chip idle (17
// blocks for 269K records, ~30 us per pass), so 2K-item tiles with 8-bit digits; merge sort up
// to 128K items (the C2 shape).
using SmallSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 8>,
                                        rocprim::kernel_config<256, 8>, 8,
                                        rocprim::block_radix_rank_algorithm::match>,
    128 * 1024>;
constexpr uint32_t SMALL_SORT_MAX = 4u << 20;
// Small sorts of more than 16 key bits (C3's 64-walk batch: 269K records on 20-bit rows): 11-bit
// digits on 4K-item tiles — two passes and two lookback resets instead of SmallSortConfig's
// three 8-bit passes: 0.499 vs 0.509 ms per step, twice each (profiles/r03_sort_small11_ab.txt);
// 62 us alone on the chip against 65 for SmallSortConfig and 126 for 11-bit digits on 2K-item
// tiles (scripts/microbench/small_sort_bench.hip). At 1,024 walks (4.3M records) the 4K tiles
// measured slower than RecordSortConfig (1.82 vs 1.73 ms per step), hence SMALL_SORT_MAX.
using Small11SortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 4>,
                                        rocprim::kernel_config<1024, 4>, 11,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;

// Stable LSD sort of (key, value) pairs on bits [0, end_bit), the config chosen by size. With
// tmp == nullptr: *bytes = the largest of the configs' needs for n (so any n' <= n fits).
template <class K, class Vt>
hipError_t sort_pairs(void *tmp, size_t &bytes, rocprim::double_buffer<K> &kb,
                      rocprim::double_buffer<Vt> &vb, uint32_t n, int end_bit, hipStream_t st) {
    if (tmp == nullptr) {
        size_t a = 0, b = 0, c = 0;
        hipError_t e = rocprim::radix_sort_pairs<RecordSortConfig>(nullptr, a, kb, vb, n, 0,
                                                                   end_bit, st);
        if (e == hipSuccess)
            e = rocprim::radix_sort_pairs<SmallSortConfig>(nullptr, b, kb, vb, n, 0, end_bit, st);
        if (e == hipSuccess)
            e = rocprim::radix_sort_pairs<Small11SortConfig>(nullptr, c, kb, vb, n, 0, end_bit,
                                                             st);
        bytes = a > b ? a : b;
        bytes = bytes > c ? bytes : c;
        return e;
    }
    if (n < SMALL_SORT_MAX && end_bit > 16)
        return rocprim::radix_sort_pairs<Small11SortConfig>(tmp, bytes, kb, vb, n, 0, end_bit, st);
    if (n < SMALL_SORT_MAX)
        return rocprim::radix_sort_pairs<SmallSortConfig>(tmp, bytes, kb, vb, n, 0, end_bit, st);
    return rocprim::radix_sort_pairs<RecordSortConfig>(tmp, bytes, kb, vb, n, 0, end_bit, st);
}

int plan_workspace(int64_t n_rec, int64_t V, void *base, Workspace *ws, hipStream_t st) {
    size_t cub_bytes = 0;
    rocprim::double_buffer<uint32_t> kb(nullptr, nullptr);
    rocprim::double_buffer<uint64_t> vb(nullptr, nullptr);
    hipError_t e = sort_pairs(nullptr, cub_bytes, kb, vb, static_cast<uint32_t>(n_rec),
                              end_bit_for(V), st);
    if (e != hipSuccess) {
        dw::set_error("dw_sgns: sort size query failed: %s", hipGetErrorString(e));
        return DW_E_HIP;
    }
    const size_t kbytes = align256((size_t)n_rec * 4), vbytes = align256((size_t)n_rec * 8);
    char *p = static_cast<char *>(base);
    ws->k0 = reinterpret_cast<uint32_t *>(p);
    ws->k1 = reinterpret_cast<uint32_t *>(p + kbytes);
    ws->v0 = reinterpret_cast<uint64_t *>(p + 2 * kbytes);
    ws->v1 = reinterpret_cast<uint64_t *>(p + 2 * kbytes + vbytes);
    const size_t wbytes = align256(sizeof(uint32_t) * MAX_OWNER_WAVES) +
                          align256(sizeof(int64_t) * MAX_OWNER_WAVES);
    const size_t bbytes = align256(sizeof(int64_t) * (MAX_PIECES + 1)) + 256 + wbytes;
    char *q = p + 2 * kbytes + 2 * vbytes;
    ws->bounds = reinterpret_cast<int64_t *>(q);
    q += align256(sizeof(int64_t) * (MAX_PIECES + 1));
    ws->count = reinterpret_cast<uint32_t *>(q);
    q += 256;
    ws->wave_counts = reinterpret_cast<uint32_t *>(q);
    q += align256(sizeof(uint32_t) * MAX_OWNER_WAVES);
    ws->wave_offsets = reinterpret_cast<int64_t *>(q);
    ws->cub = p + 2 * kbytes + 2 * vbytes + bbytes;
    ws->cub_bytes = cub_bytes;
    ws->total = 2 * kbytes + 2 * vbytes + bbytes + align256(cub_bytes);
    return DW_OK;
}

// Grid cap for the grid-stride SGNS kernels: `per_cu` blocks per compute unit (a couple of
// resident rounds), so per-block epilogues (loss atomics) stay in the thousands.
int64_t grid_cap(int per_cu) {
    static int n_cu[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 65536;
    if (n_cu[dev] == 0) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            v <= 0)
            v = 256;
        n_cu[dev] = v;
    }
    return (int64_t)n_cu[dev] * per_cu;
}

// ---- deterministic mode: gradient buffers with an int64 fixed-point accumulator -------------
struct ExactEntry {
    int64_t *acc;
    int64_t n;
    int32_t frac, flags;
};
std::mutex g_exact_mu;
std::unordered_map<const float *, ExactEntry> g_exact;

// The accumulator registered for gradient buffer g (dw_exact_register) as a launch's Fixed,
// {NULL} when g has none; `need` elements must fit.
int exact_of(const float *g, int64_t need, dw::Fixed *fx, int32_t *flags, const char *who) {
    *fx = dw::Fixed{};
    if (flags) *flags = 0;
    if (!g) return DW_OK;
    std::lock_guard<std::mutex> lk(g_exact_mu);
    const auto it = g_exact.find(g);
    if (it == g_exact.end()) return DW_OK;
    DW_REQUIRE(it->second.n >= need, "%s: the registered accumulator holds %lld elements, the "
               "launch needs %lld", who, (long long)it->second.n, (long long)need);
    *fx = dw::Fixed{it->second.acc, ldexp(1.0, it->second.frac), ldexp(1.0, -it->second.frac)};
    if (flags) *flags = it->second.flags;
    return DW_OK;
}

}  // namespace

// (dw_common.h) the registry's entry for a gradient buffer, for the dense Adam's fused conversion
int dw::exact_lookup(const float *g, dw::Fixed *fx, int64_t *n, int32_t *flags) {
    *fx = dw::Fixed{};
    *n = 0;
    *flags = 0;
    if (!g) return 0;
    std::lock_guard<std::mutex> lk(g_exact_mu);
    const auto it = g_exact.find(g);
    if (it == g_exact.end()) return 0;
    *fx = dw::Fixed{it->second.acc, ldexp(1.0, it->second.frac), ldexp(1.0, -it->second.frac)};
    *n = it->second.n;
    *flags = it->second.flags;
    return 1;
}

namespace {

template <bool FROM_WALKS, bool RECORDS>
int launch_pass1(const SgnsArgs &a, hipStream_t st) {
    int64_t blocks = (a.batch + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
    if (blocks > grid_cap(8)) blocks = grid_cap(8);
    if (blocks < 1) blocks = 1;
    const dim3 g((unsigned)blocks), bl(WAVES_PER_BLOCK * WAVE);
    const bool exact = a.fx_in.acc != nullptr;
    DW_REQUIRE(!exact || RECORDS, "dw_sgns: the deterministic mode needs the records (sorted) "
               "output-table path");
    DW_REQUIRE(!exact || FROM_WALKS || a.n_in == 1,
               "dw_sgns: the deterministic mode does not cover pooled (CBOW) inputs");
#define DW_SGNS_CASE(VPL)                                                                    \
    if (a.d <= 64 * VPL) {                                                                    \
        const bool full = a.d == 64 * VPL;                                                    \
        if (exact && RECORDS && full)                                                         \
            hipLaunchKernelGGL((k_sgns<VPL, false, FROM_WALKS, RECORDS, CHUNK, RECORDS>), g,  \
                               bl, 0, st, a);                                                 \
        else if (exact && RECORDS)                                                            \
            hipLaunchKernelGGL((k_sgns<VPL, true, FROM_WALKS, RECORDS, CHUNK, RECORDS>), g,   \
                               bl, 0, st, a);                                                 \
        else if (full)                                                                        \
            hipLaunchKernelGGL((k_sgns<VPL, false, FROM_WALKS, RECORDS, CHUNK>), g, bl, 0, st, \
                               a);                                                            \
        else                                                                                  \
            hipLaunchKernelGGL((k_sgns<VPL, true, FROM_WALKS, RECORDS, CHUNK>), g, bl, 0, st, \
                               a);                                                            \
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

// 16-lane-group pass 1 when d is a multiple of 64 (<= 512) and 2R(1+K) <= 64; otherwise
// DW_E_UNSUPPORTED (the caller falls back to the 64-lane k_sgns).
template <bool FROM_WALKS, bool OWNER = false, bool COEFIN = false>
int launch_pass1_g16(const SgnsArgs &a, hipStream_t st) {
    const int64_t T = (int64_t)a.C * (1 + a.K);
    if (a.d % 64 != 0 || a.d > 512 || T > G16_TMAX) return DW_E_UNSUPPORTED;
    int64_t blocks = (a.batch + 4 * WAVES_PER_BLOCK - 1) / (4 * WAVES_PER_BLOCK);
    if (blocks > grid_cap(8)) blocks = grid_cap(8);
    if (blocks < 1) blocks = 1;
    const dim3 g((unsigned)blocks), bl(WAVES_PER_BLOCK * WAVE);
    if constexpr (COEFIN) {
        // (eight and sixteen rows per chunk measured 45 and 59 us against 42 at C3's 64-walk
        // batch: the pass-1 chunking stays)
        switch ((a.d / 64) * 2 + (a.fx_in.acc ? 1 : 0)) {
            case 2: hipLaunchKernelGGL((k_sgns_g16<1, FROM_WALKS, 8, true, false, true>), g, bl, 0, st, a); break;
            case 3: hipLaunchKernelGGL((k_sgns_g16<1, FROM_WALKS, 8, true, true, true>), g, bl, 0, st, a); break;
            case 4: hipLaunchKernelGGL((k_sgns_g16<2, FROM_WALKS, 4, true, false, true>), g, bl, 0, st, a); break;
            case 5: hipLaunchKernelGGL((k_sgns_g16<2, FROM_WALKS, 4, true, true, true>), g, bl, 0, st, a); break;
            case 8: hipLaunchKernelGGL((k_sgns_g16<4, FROM_WALKS, 2, true, false, true>), g, bl, 0, st, a); break;
            case 9: hipLaunchKernelGGL((k_sgns_g16<4, FROM_WALKS, 2, true, true, true>), g, bl, 0, st, a); break;
            case 16: hipLaunchKernelGGL((k_sgns_g16<8, FROM_WALKS, 1, true, false, true>), g, bl, 0, st, a); break;
            case 17: hipLaunchKernelGGL((k_sgns_g16<8, FROM_WALKS, 1, true, true, true>), g, bl, 0, st, a); break;
            default:
                dw::set_error("dw_sgns: the coefficient-input pass 1 needs d in {64, 128, 256, 512}, got %d", a.d);
                return DW_E_UNSUPPORTED;
        }
        DW_LAUNCH_CHECK("dw_sgns/g16_coefin");
        return DW_OK;
    }
    if (a.fx_in.acc) {   // deterministic mode
        switch (a.d / 64) {
            case 1: hipLaunchKernelGGL((k_sgns_g16<1, FROM_WALKS, 8, OWNER, true>), g, bl, 0, st, a); break;
            case 2: hipLaunchKernelGGL((k_sgns_g16<2, FROM_WALKS, 4, OWNER, true>), g, bl, 0, st, a); break;
            case 4: hipLaunchKernelGGL((k_sgns_g16<4, FROM_WALKS, 2, OWNER, true>), g, bl, 0, st, a); break;
            case 8: hipLaunchKernelGGL((k_sgns_g16<8, FROM_WALKS, 1, OWNER, true>), g, bl, 0, st, a); break;
            default: return DW_E_UNSUPPORTED;   // the caller falls back to k_sgns
        }
        DW_LAUNCH_CHECK("dw_sgns/g16");
        return DW_OK;
    }
    switch (a.d / 64) {  // rows per chunk: CHR * F4 float4 registers per lane
        case 1: hipLaunchKernelGGL((k_sgns_g16<1, FROM_WALKS, 8, OWNER>), g, bl, 0, st, a); break;
        case 2: hipLaunchKernelGGL((k_sgns_g16<2, FROM_WALKS, 4, OWNER>), g, bl, 0, st, a); break;
        case 4: hipLaunchKernelGGL((k_sgns_g16<4, FROM_WALKS, 2, OWNER>), g, bl, 0, st, a); break;
        case 8: hipLaunchKernelGGL((k_sgns_g16<8, FROM_WALKS, 1, OWNER>), g, bl, 0, st, a); break;
        default: return DW_E_UNSUPPORTED;   // the caller falls back to k_sgns
    }
    DW_LAUNCH_CHECK("dw_sgns/g16");
    return DW_OK;
}

// Rows the fused gather did not update: boundary rows (g in g_out) and rows no record touched
// (g_out = 0) — Adam with g_out, which is left zeroed. Each wave reads the flags of 64 rows in
// one load, ballots the unflagged ones and updates only those (lane-coalesced rows), so the
// common case at C3 — almost every row already updated — costs one byte per row. g is
// re-zeroed only where its bits are not +0 (boundary rows, and any -0 a caller left), so the
// skipped store leaves the same bits.
template <int VPL, bool MASKED>
__global__ void __launch_bounds__(256)
    k_adam_rest(int64_t n_rows, int32_t d, uint8_t *__restrict__ flags,
                float *__restrict__ g, OutAdam oa) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t n_waves = (int64_t)gridDim.x * (blockDim.x / WAVE);
    const dw::AdamScalars sc = dw::step_adam(oa.dyn, oa.s);
    for (int64_t base = (blockIdx.x * (int64_t)(blockDim.x / WAVE) + threadIdx.x / WAVE) * WAVE;
         base < n_rows; base += n_waves * WAVE) {
        const int64_t r = base + lane;
        const bool in = r < n_rows;
        const uint8_t f = in ? flags[r] : 1;
        if (in && f != 0) flags[r] = 0;     // the flags are left zero for the next step
        unsigned long long todo = __ballot(in && f == 0);
        // two rows per trip (wave-uniform): both rows' loads are issued before either's stores
        while (todo) {
            const int l0 = __ffsll(static_cast<long long>(todo)) - 1;
            todo &= todo - 1ull;
            const bool two = todo != 0ull;
            const int l1 = two ? __ffsll(static_cast<long long>(todo)) - 1 : l0;
            if (two) todo &= todo - 1ull;
            const int64_t o0 = (base + l0) * d + lane, o1 = (base + l1) * d + lane;
            float pp[2][VPL], gg[2][VPL], mm[2][VPL], vv[2][VPL];
#pragma unroll
            for (int m = 0; m < VPL; ++m) {
                if (MASKED && lane + WAVE * m >= d) continue;
                const int64_t i0 = o0 + WAVE * m, i1 = o1 + WAVE * m;
                pp[0][m] = oa.p[i0]; gg[0][m] = g[i0]; mm[0][m] = oa.m[i0]; vv[0][m] = oa.v[i0];
                pp[1][m] = oa.p[i1]; gg[1][m] = g[i1]; mm[1][m] = oa.m[i1]; vv[1][m] = oa.v[i1];
            }
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (k == 1 && !two) break;
                const int64_t o = k ? o1 : o0;
#pragma unroll
                for (int m = 0; m < VPL; ++m) {
                    if (MASKED && lane + WAVE * m >= d) continue;
                    const int64_t i = o + WAVE * m;
                    dw::adam_elem(pp[k][m], gg[k][m], mm[k][m], vv[k][m], sc);
                    oa.p[i] = pp[k][m];
                    oa.m[i] = mm[k][m];
                    oa.v[i] = vv[k][m];
                    // untouched rows' g is already +0: no write (-0 is cleared too)
                    if (__float_as_uint(gg[k][m]) != 0u) g[i] = 0.f;
                }
            }
        }
    }
}

// Lazy form, after k_rec_gather: the rows that straddle chunks (their gradient summed by
// atomics into g_out). Chunk c's last row is updated here by the chunk where the row begins —
// each straddling row exactly once — with g from g_out, which is re-zeroed.
template <int VPL, bool MASKED>
__global__ void __launch_bounds__(WAVES_PER_BLOCK *WAVE)
    k_lazy_boundary(const uint32_t *__restrict__ keys, int64_t n_rec, int32_t gch,
                    float *__restrict__ g_out, int32_t d, OutAdam oa,
                    const int64_t *__restrict__ range) {
    const int lane = threadIdx.x & (WAVE - 1);
    if (range) n_rec = range[1];   // (range[0] == 0: the padded owner sort, launch_owner_pass2)
    const int64_t n_chunks = (n_rec + gch - 1) / gch;
    const int64_t n_waves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
    for (int64_t ch = (int64_t)blockIdx.x * WAVES_PER_BLOCK + threadIdx.x / WAVE; ch < n_chunks;
         ch += n_waves) {
        const int64_t e0 = ch * gch;
        const int64_t e1 = (e0 + gch < n_rec) ? e0 + gch : n_rec;
        const uint32_t row = keys[e1 - 1];
        if (e1 >= n_rec || keys[e1] != row) continue;               // does not continue
        if (keys[e0] == row && e0 > 0 && keys[e0 - 1] == row) continue;   // began earlier
        float g[VPL];
        const int64_t o = static_cast<int64_t>(row) * d + lane;
#pragma unroll
        for (int m = 0; m < VPL; ++m) {
            g[m] = 0.f;
            if (MASKED && lane + WAVE * m >= d) continue;
            g[m] = g_out[o + WAVE * m];
            g_out[o + WAVE * m] = 0.f;
        }
        lazy_row_step<VPL, MASKED>(oa, dw::eff_step(oa.dyn, oa.step_delta, oa.step), row, d,
                                   lane, g);
    }
}

template <int VPL>
void launch_boundary(hipStream_t st, const uint32_t *keys, int64_t n_rec, int32_t gch,
                     float *g_out, int32_t d, const OutAdam &oa, const int64_t *range) {
    int64_t blocks = ((n_rec + gch - 1) / gch + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
    if (blocks < 1) blocks = 1;
    if (blocks > 65536) blocks = 65536;
    if (d == 64 * VPL)
        hipLaunchKernelGGL((k_lazy_boundary<VPL, false>), dim3((unsigned)blocks),
                           dim3(WAVES_PER_BLOCK * WAVE), 0, st, keys, n_rec, gch, g_out, d, oa,
                           range);
    else
        hipLaunchKernelGGL((k_lazy_boundary<VPL, true>), dim3((unsigned)blocks),
                           dim3(WAVES_PER_BLOCK * WAVE), 0, st, keys, n_rec, gch, g_out, d, oa,
                           range);
}

// ---- the rows-major lazy out step (dw_sgns_owner_out_rows) -----------------------------------
// The 64-walk batch's out rows are ~224K distinct rows of 1M, each read and written as p, m, v
// (3 x 512 B): the catch-up -> pass 1 -> lazy gather sequence moved each across HBM twice and
// read p a third time. Here one kernel does a row's whole out-side step where its p / m / v sit
// in registers: replay its deferred g = 0 steps (dw::replay_g0, to p^{s-1}), the logit of each
// of its records against the record's centre row (pass 1's 16-lane layout and FMA order, the
// row staged in LDS: the same bits), the coefficient (row_coef, the loss sums), the gradient
// sum over its records in placed order (the gather's order) and the Adam step. For the centre
// pass (dw_sgns_owner_pass1 with order_ready & 4, k_sgns_g16's COEFIN form) it leaves, by slot,
// each record's coefficient in coef_slot, and each row PENDING: m and v at step s, p at s - 1 in
// the table (oa.pend[row] = 1), where the centre pass reads it; the parameter half of step s is
// applied (dw::settle_pending) when the row is next replayed or flushed — the same operations
// as adam_elem's, so the same bits, without a per-slot copy of p^{s-1} (138 MB at C3/64).
// A block takes a range of 4 gch <= 256 placed records: its waves read them (one packed 8-B
// record per lane: centre node, slot and context flag, k_place_slots) into LDS with the rows' starts,
// then take the range's rows one at a time from a block counter (an LDS atomic) — a row's time is
// set by its deferred steps, ~4 on average but geometric, so four waves sharing ~150 rows finish
// together where each wave's own fixed chunk left the slowest waves running alone — and ranges
// small enough that there are about twice as many blocks as resident slots, which the hardware
// hands out as blocks finish. Per row: four records' centre rows in flight (one per 16-lane group
// for the logits). No row is split between ranges (whole rows, below).
// (Four rows per wave, one per 16-lane group, measured 350-370 us against the three kernels'
// ~280 us at C3's 64-walk batch: each group waited for the longest replay of the four, and the
// 138-VGPR kernel ran three waves per SIMD.)
// Each row's first-round centre rows (independent of the replay) are issued together with the
// row, and the next row's p / m / v / last / pend are issued before this row's replay (after its
// centre rows, so waiting for those never waits for the prefetch: loads return in order), so one
// round trip is left exposed per row. Seven waves per SIMD (OUT_ROWS_WAVES, 72 VGPRs, a few
// spills outside the row loop): 0.2635-0.2641 ms per step against 0.2676-0.268 at six and
// 0.279-0.280 at eight (profiles/r06_pipe_order_ab.txt).
// EXACT (the deterministic mode, g_out registered): each term coef * w_in enters the row's sum
// as a fixed-point integer (dw::to_fixed, the records gather's rule), so the sum is the same
// whatever order the claim's atomics ranked the records in.
// Whole rows (round 6): a range steps the rows that START in it, whole — the records of its last
// row that continue past the range end (up to off[row + 1], the placement's segment end) are
// read from the placed arrays 64 at a time into the wave's registers — and skips the records of a
// row begun in an earlier range. No row is split, so no g_out atomics, no k_lazy_boundary /
// k_fixed_boundary launch between this kernel and the centre pass (one range finishing a hub row
// alone: the hubs have the low ids, so their ranges start first). (Stepping a straddling row by
// the range that finishes it last — a device fence and a part counter per row — measured 0.41
// against 0.295 ms: an agent-scope release on MI355X writes back the XCD's L2.)
constexpr int OUT_ROWS_WAVES = 7;
template <int F4, bool EXACT = false>
__global__ void __launch_bounds__(WAVES_PER_BLOCK *WAVE, F4 <= 2 ? OUT_ROWS_WAVES : 2)
    k_out_rows(SgnsArgs a, const uint32_t *__restrict__ keys, const uint64_t *__restrict__ vals,
               const int64_t *__restrict__ range, int32_t gch, OutAdam oa,
               float *__restrict__ coef_slot, dw::Fixed fo, const uint32_t *__restrict__ off) {
    constexpr int D = 64 * F4;
    constexpr int BR = WAVES_PER_BLOCK * WAVE;   // records per block range, at most
    bool fx_range = false;
    uint32_t fx_tmax = 0u;   // EXACT: the largest |term|'s bits (the range test, at the end)
    constexpr int RU = 4;   // records per round (one per 16-lane group)
    // the block range's records (slot, centre node, context flag) and its rows' starts
    __shared__ uint32_t s_key[BR], s_slot[BR];   // (slot | context flag << 31)
    __shared__ int32_t s_cid[BR];
    __shared__ uint16_t s_rs[BR + 1];
    __shared__ int32_t s_wrows[WAVES_PER_BLOCK];
    __shared__ int32_t s_next;   // the next row to take
    __shared__ float4 s_p[WAVES_PER_BLOCK][D / 4];        // the row's p^{s-1}
    __shared__ float4 s_c[WAVES_PER_BLOCK][RU][D / 4];    // the round's centre rows
    __shared__ uint32_t s_ovs[WAVES_PER_BLOCK][WAVE];     // a continuing row's records, 64 at a
    __shared__ int32_t s_ovc[WAVES_PER_BLOCK][WAVE];      // time (slot | context << 31, centre)
    const int lane = threadIdx.x & (WAVE - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
    const int q = lane >> 4, gl = lane & 15;
    const uint64_t lt = (1ull << lane) - 1ull;
    const int64_t n_rec = range[1];
    const int32_t br_len = WAVES_PER_BLOCK * gch;   // (gch <= 64)
    const int64_t n_ranges = (n_rec + br_len - 1) / br_len;
    const int32_t step = dw::eff_step(oa.dyn, oa.step_delta, oa.step);
    const dw::AdamScalars hs = dw::hist_at(oa.hist, step);
    const int32_t box_from = dw::hist_box_from(oa.hist);
    const int T = a.C * (1 + a.K), rpc = 1 + a.K;
    const int64_t per = a.L - 2 * a.R;
    float *sp = reinterpret_cast<float *>(&s_p[wv][0]);
    float acc_pos = 0.f, acc_neg = 0.f, acc_rec = 0.f, acc_prec = 0.f;

    for (int64_t br = blockIdx.x; br < n_ranges; br += gridDim.x) {
        const int64_t r0 = br * br_len;
        const int n_blk = static_cast<int>(n_rec - r0 < br_len ? n_rec - r0 : br_len);
        // the record past the range: its row continues the range's last row or not
        const uint32_t after = r0 + n_blk < n_rec ? keys[r0 + n_blk] : 0xFFFFFFFFu;
        {   // wave wv reads records [64 wv, 64 wv + 64) of the range: one per lane, all at once
            const int i = WAVE * wv + lane;
            const bool in = i < n_blk;
            const uint32_t key = in ? keys[r0 + i] : 0xFFFFFFFFu;
            // (record 0 starts a row unless the row began in the range before: not ours)
            const uint32_t prev = lane > 0 ? 0u
                                  : i == 0 ? (r0 > 0 ? keys[r0 - 1] : 0xFFFFFFFFu)
                                           : (in ? keys[r0 + i - 1] : 0u);
            // (k_place_slots: centre << 32 | slot | context flag << 31)
            const uint64_t rec = in ? vals[r0 + i] : 0xFFFFFFFF00000000ull;
            const uint32_t up = __shfl_up(key, 1, WAVE);
            const bool is_start = in && key != (lane > 0 ? up : prev);
            const uint64_t starts = __ballot(is_start);
            s_key[i] = key;
            s_slot[i] = static_cast<uint32_t>(rec);
            s_cid[i] = static_cast<int32_t>(rec >> 32);
            if (lane == 0) s_wrows[wv] = __popcll(starts);
            __syncthreads();
            int base = 0, nr = 0;
#pragma unroll
            for (int x = 0; x < WAVES_PER_BLOCK; ++x) {
                base += x < wv ? s_wrows[x] : 0;
                nr += s_wrows[x];
            }
            if (is_start) s_rs[base + __popcll(starts & lt)] = static_cast<uint16_t>(i);
            if (threadIdx.x == 0) {
                s_rs[nr] = static_cast<uint16_t>(n_blk);
                s_next = 0;
            }
            __syncthreads();
        }
        const int nrows = s_wrows[0] + s_wrows[1] + s_wrows[2] + s_wrows[3];
        // rows one at a time from the block's counter: a row's time is set by its deferred steps,
        // so the four waves share the range's rows instead of each running a fixed quarter
        auto take = [&]() {
            int k = 0;
            if (lane == 0) k = atomicAdd(&s_next, 1);
            return __builtin_amdgcn_readfirstlane(k);
        };
        // the next row's state, loaded one row ahead
        float np[F4], nm[F4], nv[F4];
        int32_t nlast = 0;
        uint32_t npend = 0;
        auto prefetch = [&](int k) {
            const uint32_t r = s_key[s_rs[k]];
            const int64_t o = static_cast<int64_t>(r) * D + lane;
            nlast = oa.last[r];
            npend = oa.pend[r];
#pragma unroll
            for (int f = 0; f < F4; ++f) {
                np[f] = oa.p[o + 64 * f];
                nm[f] = oa.m[o + 64 * f];
                nv[f] = oa.v[o + 64 * f];
            }
        };
        int k = take();
        if (k < nrows) prefetch(k);
        while (k < nrows) {
            const int rs = s_rs[k], re = s_rs[k + 1];   // (wave-uniform)
            const uint32_t row = s_key[rs];
            const int64_t ro = static_cast<int64_t>(row) * D + lane;
            // the range's last row continuing past it: all its records from the placed arrays
            const bool glob = re == n_blk && after == row;
            const int cnt = glob ? static_cast<int>(off[row + 1] - static_cast<uint32_t>(r0 + rs))
                                 : re - rs;
            auto window = [&](int j) {   // glob: records [j, j + 64) of the row into the LDS
                const uint64_t rec = j + lane < cnt ? vals[r0 + rs + j + lane]
                                                    : 0xFFFFFFFF00000000ull;
                s_ovs[wv][lane] = static_cast<uint32_t>(rec);
                s_ovc[wv][lane] = static_cast<int32_t>(rec >> 32);
                dw::wave_lds_sync();
            };
            if (glob) window(0);
            // the row's records in the LDS: the range's staging, or the wave's window (64 at a time)
            const uint32_t *Ls = glob ? &s_ovs[wv][0] : &s_slot[rs];
            const int32_t *Lc = glob ? &s_ovc[wv][0] : &s_cid[rs];
            const int msk = glob ? WAVE - 1 : 0x7FFFFFFF;
            float p[F4], m[F4], v[F4], g[F4];
            int64_t gx[EXACT ? F4 : 1];
#pragma unroll
            for (int f = 0; f < F4; ++f) {
                p[f] = np[f];
                m[f] = nm[f];
                v[f] = nv[f];
                g[f] = 0.f;
            }
#pragma unroll
            for (int f = 0; f < (EXACT ? F4 : 1); ++f) gx[f] = 0;
            const int32_t from = __builtin_amdgcn_readfirstlane(nlast);
            const bool pd = __builtin_amdgcn_readfirstlane(npend) != 0;
            // this row's prefetched loads (issued a row ago) are complete before the next loads
            // go out, so that waiting for those never waits for these and the compiler does not
            // hold them back behind this row's (vector loads return in order)
            __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) (gfx9 encoding; expcnt, lgkmcnt free)
            // round 0's centre rows (group q: record q of the row; lane gl: elements
            // [4gl + 64f, +4)), then the next row's loads — both in flight during the replay
            float4 c4[F4];
            {
                const int32_t cid = q < cnt ? Lc[q] : -1;
                const bool ok = cid >= 0 && cid < a.V;
                const float *crow = a.w_in + static_cast<int64_t>(ok ? cid : 0) * D + 4 * gl;
#pragma unroll
                for (int f = 0; f < F4; ++f)
                    c4[f] = ok ? *reinterpret_cast<const float4 *>(crow + 64 * f)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
            }
            const int kn = take();
            prefetch(kn < nrows ? kn : k);   // (unconditional: no register copies)
            if (pd) dw::settle_pending(p, m, v, oa.hist, from, box_from);   // the previous step's p half
            dw::replay_g0(p, m, v, oa.hist, from, step - 1, box_from);   // -> p^{s-1}
#pragma unroll
            for (int f = 0; f < F4; ++f) sp[lane + 64 * f] = p[f];
            dw::wave_lds_sync();
            for (int j0 = 0; j0 < cnt; j0 += RU) {
                // group q: record j0 + q's logit in pass 1's layout and its coefficient
                const bool in = j0 + q < cnt;
                if (glob && j0 > 0 && (j0 & (WAVE - 1)) == 0) window(j0);   // (wave-uniform)
                const int l = in ? (j0 & msk) + q : 0;
                const uint32_t spx = Ls[l];
                const uint32_t slot = spx & 0x7FFFFFFFu;
                const bool pos = (spx >> 31) != 0u;
                const int32_t cid = in ? Lc[l] : -1;
                const bool ok = in && cid >= 0 && cid < a.V;
                if (j0 > 0) {   // later rounds (rows of more than RU records)
                    const float *crow = a.w_in + static_cast<int64_t>(ok ? cid : 0) * D + 4 * gl;
#pragma unroll
                    for (int f = 0; f < F4; ++f)
                        c4[f] = ok ? *reinterpret_cast<const float4 *>(crow + 64 * f)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
                }
                float pr = 0.f;   // pass 1's order: x, y, z, w of each float4, then the DPP sum
#pragma unroll
                for (int f = 0; f < F4; ++f) {
                    const float4 of = s_p[wv][gl + 16 * f];
                    pr = fmaf(c4[f].x, of.x, pr);
                    pr = fmaf(c4[f].y, of.y, pr);
                    pr = fmaf(c4[f].z, of.z, pr);
                    pr = fmaf(c4[f].w, of.w, pr);
                    s_c[wv][q][gl + 16 * f] = c4[f];
                }
                const float x = row_sum16(pr);
                float coef = 0.f;
                if (ok && gl == 0)
                    coef = row_coef(x, pos, a.scale, acc_pos, acc_neg, acc_rec, acc_prec);
                if (in && gl == 0) coef_slot[slot] = coef;
                dw::wave_lds_sync();
                // the gradient over the round's records in placed order (lane-strided elements,
                // the gather's accumulation)
#pragma unroll
                for (int u = 0; u < RU; ++u) {
                    if (j0 + u >= cnt) break;
                    const float cu = __shfl(coef, u << 4, WAVE);
                    const float *cr = reinterpret_cast<const float *>(&s_c[wv][u][0]);
                    if constexpr (EXACT) {
#pragma unroll
                        for (int f = 0; f < F4; ++f) {
                            const float t = cu * cr[lane + 64 * f];
                            gx[f] += dw::fixed_bits(t, fo.fs);
                            fx_tmax = dw::fixed_track(fx_tmax, t);
                        }
                    } else {
#pragma unroll
                        for (int f = 0; f < F4; ++f) g[f] += cu * cr[lane + 64 * f];
                    }
                }
                dw::wave_lds_sync();   // s_c is rewritten next round
            }
            if constexpr (EXACT) {
#pragma unroll
                for (int f = 0; f < F4; ++f) {
                    gx[f] = dw::fixed_finish(gx[f], cnt);   // cnt terms
                    g[f] = dw::from_fixed(gx[f], fo.fi);
                }
            }
            {
                // the moments of step s; p stays p^{s-1} for the centre pass, which reads it from
                // the table (no per-slot copies), and the parameter half waits (pend[row])
#pragma unroll
                for (int f = 0; f < F4; ++f) {
                    dw::adam_mv(p[f], g[f], m[f], v[f], hs);
                    oa.p[ro + 64 * f] = p[f];
                    oa.m[ro + 64 * f] = m[f];
                    oa.v[ro + 64 * f] = v[f];
                }
                if (lane == 0) {
                    oa.last[row] = step;
                    if (!pd) oa.pend[row] = 1;   // (already 1 where the row was pending)
                    if (oa.counts) oa.counts[row] = 0u;
                }
            }
            k = kn;
        }
        __syncthreads();   // the range's LDS is rewritten by the next one
    }
    if constexpr (EXACT) {
        fx_range = fx_range || dw::fixed_range(fx_tmax, fo.fs);
        if (__ballot(fx_range) && lane == 0) dw::status_or(a.status, DW_S_FIXED_RANGE);
    }
    if (a.loss_acc) flush_loss(a.loss_acc, acc_pos, acc_neg, acc_rec, acc_prec);
}

template <int VPL, bool EXACT>
void launch_gather_fx(dim3 g, dim3 bl, hipStream_t st, const uint32_t *keys,
                      const uint64_t *vals, int64_t n_rec, const float *w_in, float *g_out,
                      int32_t d, const OutAdam *oa, const int64_t *range, int32_t gch,
                      const dw::Fixed &fo, int32_t *status) {
    const bool full = d == 64 * VPL;
    if (oa) {
        if (full)
            hipLaunchKernelGGL((k_rec_gather<VPL, false, true, EXACT>), g, bl, 0, st, keys, vals,
                               n_rec, w_in, g_out, d, *oa, range, gch, fo, status);
        else
            hipLaunchKernelGGL((k_rec_gather<VPL, true, true, EXACT>), g, bl, 0, st, keys, vals,
                               n_rec, w_in, g_out, d, *oa, range, gch, fo, status);
    } else {
        if (full)
            hipLaunchKernelGGL((k_rec_gather<VPL, false, false, EXACT>), g, bl, 0, st, keys,
                               vals, n_rec, w_in, g_out, d, OutAdam{}, range, gch, fo, status);
        else
            hipLaunchKernelGGL((k_rec_gather<VPL, true, false, EXACT>), g, bl, 0, st, keys, vals,
                               n_rec, w_in, g_out, d, OutAdam{}, range, gch, fo, status);
    }
}

template <int VPL>
void launch_gather(dim3 g, dim3 bl, hipStream_t st, const uint32_t *keys, const uint64_t *vals,
                   int64_t n_rec, const float *w_in, float *g_out, int32_t d,
                   const OutAdam *oa, const int64_t *range, int32_t gch, const dw::Fixed &fo,
                   int32_t *status) {
    if (fo.acc)
        launch_gather_fx<VPL, true>(g, bl, st, keys, vals, n_rec, w_in, g_out, d, oa, range, gch,
                                    fo, status);
    else
        launch_gather_fx<VPL, false>(g, bl, st, keys, vals, n_rec, w_in, g_out, d, oa, range,
                                     gch, fo, status);
}

template <int VPL>
void launch_rest(hipStream_t st, int64_t V, int32_t d, float *g_out, const OutAdam &oa) {
    int64_t rb = (V + 255) / 256;   // 4 waves x 64 rows per block
    if (rb > grid_cap(8)) rb = grid_cap(8);
    if (rb < 1) rb = 1;
    if (d == 64 * VPL)
        hipLaunchKernelGGL((k_adam_rest<VPL, false>), dim3((unsigned)rb), dim3(256), 0, st, V, d,
                           oa.flags, g_out, oa);
    else
        hipLaunchKernelGGL((k_adam_rest<VPL, true>), dim3((unsigned)rb), dim3(256), 0, st, V, d,
                           oa.flags, g_out, oa);
}

// oa != NULL: the fused output-table Adam (rows 0..V of the out table) — gather, then the
// rest-of-rows update, which also clears the row flags.
// range != NULL: one row piece (records [range[0], range[1]), read on the device); the grid is
// sized for `share` of the records (grid-stride beyond).
int launch_pass2(const uint32_t *keys, const uint64_t *vals, int64_t n_rec, const float *w_in,
                 float *g_out, int32_t d, const OutAdam *oa, int64_t V, hipStream_t st,
                 const int64_t *range = nullptr, double share = 1.0, int32_t *status = nullptr) {
    dw::Fixed fo;   // deterministic mode: g_out's accumulator
    {
        const int rc = exact_of(g_out, V * d, &fo, nullptr, "dw_sgns pass 2");
        if (rc != DW_OK) return rc;
    }
    // chunk size: GCH for large batches (balanced, few boundary rows); halved down to 32 while
    // the chunks would not give every SIMD of the chip a few waves — a 9K-record batch (C2 shape)
    // in 512-record chunks ran as 18 waves, 240 us of latency-bound gathers
    // (scripts/experiments/gch_sweep.sh measured the sizes)
    int32_t gch = GCH;
    {
        const int64_t want = grid_cap(16);   // 4 waves per SIMD
        while (gch > 32 && (n_rec + gch - 1) / gch < want) gch >>= 1;
    }
    const int64_t n_chunks = (n_rec + gch - 1) / gch;
    int64_t blocks = (int64_t)((double)(n_chunks + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK * share);
    if (blocks < 1) blocks = 1;
    if (blocks > 65536) blocks = 65536;
    const dim3 g((unsigned)blocks), bl(WAVES_PER_BLOCK * WAVE);
    if (d <= 64) launch_gather<1>(g, bl, st, keys, vals, n_rec, w_in, g_out, d, oa, range, gch, fo, status);
    else if (d <= 128) launch_gather<2>(g, bl, st, keys, vals, n_rec, w_in, g_out, d, oa, range, gch, fo, status);
    else if (d <= 256) launch_gather<4>(g, bl, st, keys, vals, n_rec, w_in, g_out, d, oa, range, gch, fo, status);
    else if (d <= 512) launch_gather<8>(g, bl, st, keys, vals, n_rec, w_in, g_out, d, oa, range, gch, fo, status);
    else return DW_E_UNSUPPORTED;
    DW_LAUNCH_CHECK("dw_sgns/gather");
    if (fo.acc && n_rec > 0) {   // the straddling rows' exact sums into g_out
        hipLaunchKernelGGL(k_fixed_boundary, g, bl, 0, st, keys, n_rec, gch, range, fo, g_out, d);
        DW_LAUNCH_CHECK("dw_sgns/fixed_boundary");
    }
    if (oa && oa->last) {   // lazy: only the straddling rows remain; untouched rows wait
        if (n_rec > 0) {
            if (d <= 64) launch_boundary<1>(st, keys, n_rec, gch, g_out, d, *oa, range);
            else if (d <= 128) launch_boundary<2>(st, keys, n_rec, gch, g_out, d, *oa, range);
            else if (d <= 256) launch_boundary<4>(st, keys, n_rec, gch, g_out, d, *oa, range);
            else launch_boundary<8>(st, keys, n_rec, gch, g_out, d, *oa, range);
            DW_LAUNCH_CHECK("dw_sgns/lazy_boundary");
        }
    } else if (oa) {
        if (d <= 64) launch_rest<1>(st, V, d, g_out, *oa);
        else if (d <= 128) launch_rest<2>(st, V, d, g_out, *oa);
        else if (d <= 256) launch_rest<4>(st, V, d, g_out, *oa);
        else launch_rest<8>(st, V, d, g_out, *oa);
        DW_LAUNCH_CHECK("dw_sgns/adam_rest");   // (k_adam_rest also clears the flags)
    }
    return DW_OK;
}

// Per-phase HIP-event timing of dw_sgns_* calls (bench / profiling; off by default). Each
// recorded call holds 4 events: start | pass 1 | sort | pass 2 (sort and pass 2 are empty
// in atomic mode). Host-side state, not thread-safe: one profiling caller per process.
struct PhaseTimer {
    static constexpr size_t MAX_CALLS = 4096;
    bool on = false;
    size_t calls = 0;
    std::vector<hipEvent_t> ev;
    bool active() const { return on && calls < MAX_CALLS; }
    void mark(int slot, hipStream_t st) {
        if (!active()) return;
        const size_t i = 4 * calls + slot;
        while (ev.size() <= i) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) {
                on = false;
                return;
            }
            ev.push_back(e);
        }
        (void)hipEventRecord(ev[i], st);
        if (slot == 3) ++calls;
    }
};
PhaseTimer g_timer;

// phase 0: the whole call. phase 1: pass 1 only (centre-table gradients, loss sums, records).
// phase 2: the records sort + pass 2 (output-table gradients) of a preceding phase-1 call with
// the same arguments and workspace. Atomic mode (no workspace) completes in phase 1; its
// phase 2 is empty. The split lets a caller start the centre-table gradient exchange while
// the output-table phase runs (ShardedTables.exchange_in).
template <bool FROM_WALKS>
int launch_sgns_impl(SgnsArgs a, void *workspace, size_t workspace_bytes, int phase,
                     hipStream_t st, const OutAdam *oa);

// phase: 0 = both passes, 1 = pass 1, 2 = the output-table phase
template <bool FROM_WALKS>
int launch_sgns(SgnsArgs a, void *workspace, size_t workspace_bytes, int phase, hipStream_t st,
                const OutAdam *oa = nullptr) {
    if (phase != 2) g_timer.mark(0, st);
    const int rc = launch_sgns_impl<FROM_WALKS>(a, workspace, workspace_bytes, phase, st, oa);
    if (rc != DW_OK) {
        if (g_timer.active()) g_timer.on = false;  // a failed call leaves its slots unusable
        return rc;
    }
    if (phase != 1) g_timer.mark(3, st);
    return DW_OK;
}

template <bool FROM_WALKS>
int launch_sgns_impl(SgnsArgs a, void *workspace, size_t workspace_bytes, int phase,
                     hipStream_t st, const OutAdam *oa) {
    const bool do1 = phase != 2, do2 = phase != 1;
    if (a.batch == 0 && do2 && oa) {  // no records: every out row gets Adam with g = g_out
        if (do1) g_timer.mark(1, st);
        g_timer.mark(2, st);
        return launch_pass2(nullptr, nullptr, 0, a.w_in, a.g_out, a.d, oa, a.V, st);
    }
    if (a.batch == 0 || workspace == nullptr) {
        if (do1 && a.batch > 0) {
            dw::Fixed f0;
            int rc0 = exact_of(a.g_in, 0, &f0, nullptr, "dw_sgns");
            if (rc0 == DW_OK) rc0 = exact_of(a.g_out, 0, &f0, nullptr, "dw_sgns");
            if (rc0 != DW_OK) return rc0;
            DW_REQUIRE(!f0.acc, "dw_sgns: the deterministic mode needs the records (sorted) "
                       "output-table path (a workspace)");
            const int rc = launch_pass1<FROM_WALKS, false>(a, st);
            if (rc != DW_OK) return rc;
        }
        if (do1) g_timer.mark(1, st);
        if (do2) g_timer.mark(2, st);
        return DW_OK;
    }
    const int64_t T = (int64_t)a.C * (1 + a.K);
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
    if (do1) {
        a.rec_key = ws.k0;
        a.rec_val = ws.v0;
        int32_t fl = 0;
        rc = exact_of(a.g_in, a.V * a.d, &a.fx_in, &fl, "dw_sgns pass 1");
        if (rc != DW_OK) return rc;
        rc = launch_pass1_g16<FROM_WALKS>(a, st);
        if (rc == DW_E_UNSUPPORTED) rc = launch_pass1<FROM_WALKS, true>(a, st);
        if (rc != DW_OK) return rc;
        if (a.fx_in.acc && !(fl & (DW_EXACT_DEFER | DW_EXACT_ADAM))) {   // the centres' exact
            int64_t cb = (a.batch + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
            if (cb > grid_cap(8)) cb = grid_cap(8);
            hipLaunchKernelGGL(k_fixed_centres<FROM_WALKS>, dim3((unsigned)cb),
                               dim3(WAVES_PER_BLOCK * WAVE), 0, st, a);
            DW_LAUNCH_CHECK("dw_sgns/fixed_centres");
        }
        g_timer.mark(1, st);
    }
    if (!do2) return DW_OK;
    rocprim::double_buffer<uint32_t> kb(ws.k0, ws.k1);
    rocprim::double_buffer<uint64_t> vb(ws.v0, ws.v1);
    size_t cub_bytes = ws.cub_bytes;
    hipError_t e = sort_pairs(ws.cub, cub_bytes, kb, vb, static_cast<uint32_t>(n_rec),
                              end_bit_for(a.V), st);
    if (e != hipSuccess) {
        dw::set_error("dw_sgns: records sort failed: %s", hipGetErrorString(e));
        return DW_E_HIP;
    }
    g_timer.mark(2, st);
    return launch_pass2(kb.current(), vb.current(), n_rec, a.w_in, a.g_out, a.d, oa, a.V, st,
                        nullptr, 1.0, a.status);
}

// ---- output-table phase in row pieces (N > 1: exchange a piece while the next one runs) -------
// bounds[p] = first record whose row >= p * piece_rows (lower bound in the sorted keys).
__global__ void k_piece_bounds(const uint32_t *__restrict__ keys, int64_t n_rec, int32_t n_pieces,
                               int64_t piece_rows, int64_t *__restrict__ bounds) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p > n_pieces) return;
    if (p == n_pieces) {
        bounds[p] = n_rec;
        return;
    }
    const uint64_t target = static_cast<uint64_t>(p) * static_cast<uint64_t>(piece_rows);
    int64_t lo = 0, hi = n_rec;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (static_cast<uint64_t>(keys[mid]) < target) lo = mid + 1;
        else hi = mid;
    }
    bounds[p] = lo;
}

// Which buffer of the workspace holds the sorted records after the piece == -1 call (rocprim's
// double buffer tells the host only): recorded per workspace for the piece calls that follow.
std::mutex g_sorted_mu;
std::unordered_map<const void *, bool> g_sorted_in_k1;

int launch_pieces(SgnsArgs a, void *workspace, size_t workspace_bytes, int piece, int n_pieces,
                  int64_t piece_rows, hipStream_t st) {
    DW_REQUIRE(workspace != nullptr, "dw_sgns_walks_phase2_piece: needs the records workspace");
    DW_REQUIRE(n_pieces >= 1 && n_pieces <= MAX_PIECES && piece >= -1 && piece < n_pieces,
               "dw_sgns_walks_phase2_piece: piece %d of %d (at most %d pieces)", piece, n_pieces,
               MAX_PIECES);
    DW_REQUIRE(piece_rows >= 1 && piece_rows * (int64_t)n_pieces >= a.V,
               "dw_sgns_walks_phase2_piece: %d pieces of %lld rows do not cover %lld rows",
               n_pieces, (long long)piece_rows, (long long)a.V);
    const int64_t T = (int64_t)a.C * (1 + a.K);
    DW_REQUIRE(T <= TMAX && a.V <= 0x7FFFFFFF, "dw_sgns_walks_phase2_piece: records mode limits");
    const int64_t n_rec = a.batch * T;
    DW_REQUIRE(n_rec < 0x7FFFFFFF, "dw_sgns_walks_phase2_piece: too many records");
    Workspace ws;
    int rc = plan_workspace(n_rec > 0 ? n_rec : 1, a.V, workspace, &ws, st);
    if (rc != DW_OK) return rc;
    DW_REQUIRE(workspace_bytes >= ws.total, "dw_sgns: workspace too small (%zu < %zu)",
               workspace_bytes, ws.total);
    if (piece == -1) {
        bool in_k1 = false;
        if (n_rec > 0) {
            rocprim::double_buffer<uint32_t> kb(ws.k0, ws.k1);
            rocprim::double_buffer<uint64_t> vb(ws.v0, ws.v1);
            size_t cub_bytes = ws.cub_bytes;
            hipError_t e = sort_pairs(ws.cub, cub_bytes, kb, vb, static_cast<uint32_t>(n_rec),
                                      end_bit_for(a.V), st);
            if (e != hipSuccess) {
                dw::set_error("dw_sgns: records sort failed: %s", hipGetErrorString(e));
                return DW_E_HIP;
            }
            in_k1 = kb.current() == ws.k1;
        }
        {
            std::lock_guard<std::mutex> lk(g_sorted_mu);
            g_sorted_in_k1[workspace] = in_k1;
        }
        hipLaunchKernelGGL(k_piece_bounds, dim3((n_pieces + 256) / 256), dim3(256), 0, st,
                           in_k1 ? ws.k1 : ws.k0, n_rec, n_pieces, piece_rows, ws.bounds);
        DW_LAUNCH_CHECK("dw_sgns/piece_bounds");
        g_timer.mark(2, st);
        return DW_OK;
    }
    bool in_k1;
    {
        std::lock_guard<std::mutex> lk(g_sorted_mu);
        auto it = g_sorted_in_k1.find(workspace);
        DW_REQUIRE(it != g_sorted_in_k1.end(),
                   "dw_sgns_walks_phase2_piece: piece %d before the sort call (piece -1)", piece);
        in_k1 = it->second;
    }
    if (n_rec > 0) {
        rc = launch_pass2(in_k1 ? ws.k1 : ws.k0, in_k1 ? ws.v1 : ws.v0, n_rec, a.w_in, a.g_out,
                          a.d, nullptr, a.V, st, ws.bounds + piece, 2.0 / n_pieces);
        if (rc != DW_OK) return rc;
    }
    if (piece == n_pieces - 1) g_timer.mark(3, st);
    return DW_OK;
}

// ---- owner-computes form (N > 1: the out table sharded by row owner, no out-table exchange) ---
// Every rank forms ALL the global batch's windows but keeps only the output slots whose row it
// owns (o % n_owners == owner). Pass 1 writes their records (local row o / n_owners) into one
// region per wave and adds the centre-table gradient of those slots into the full g_in
// (reduce-scattered by the caller); k_wave_scan + k_rec_compact pack the regions in wave order
// (so the records, and pass 2's per-row sums, come out in the same order every run). Pass 2
// sorts them by local row and gathers, with the slice's Adam fused in or not. The regions are
// sized for every slot of a wave's iterations, so they can never overflow.
struct OwnerLayout {
    int64_t blocks, n_waves, region, total;
};

OwnerLayout owner_layout(int64_t n_centres, int64_t T) {
    OwnerLayout l;
    l.blocks = (n_centres + 4 * WAVES_PER_BLOCK - 1) / (4 * WAVES_PER_BLOCK);  // = launch_pass1_g16
    if (l.blocks > grid_cap(8)) l.blocks = grid_cap(8);
    if (l.blocks < 1) l.blocks = 1;
    l.n_waves = l.blocks * WAVES_PER_BLOCK;
    const int64_t per_sweep = l.n_waves * 4;  // centres per grid-stride iteration
    const int64_t iters = (n_centres + per_sweep - 1) / per_sweep;
    l.region = iters * 4 * T;
    l.total = l.n_waves * l.region;
    return l;
}

// exclusive prefix sums of the per-wave record counts (one block; n <= MAX_OWNER_WAVES); the
// total goes to *count
__global__ void __launch_bounds__(1024)
    k_wave_scan(const uint32_t *__restrict__ counts, int64_t n, int64_t *__restrict__ offsets,
                uint32_t *__restrict__ count) {
    __shared__ int64_t part[1024];
    const int t = threadIdx.x;
    const int64_t per = (n + 1023) / 1024;
    const int64_t lo = t * per, hi = lo + per < n ? lo + per : n;
    int64_t sum = 0;
    for (int64_t i = lo; i < hi; ++i) sum += counts[i];
    part[t] = sum;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan of the partials
        const int64_t v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int64_t run = part[t] - sum;  // exclusive prefix of this thread's first count
    for (int64_t i = lo; i < hi; ++i) {
        offsets[i] = run;
        run += counts[i];
    }
    if (t == 1023) *count = static_cast<uint32_t>(part[1023]);
}

// wave g's region [g * region, g * region + counts[g]) of (k_src, v_src) -> offsets[g] of (k_dst,
// v_dst); one block per region (grid-stride beyond the grid)
__global__ void __launch_bounds__(256)
    k_rec_compact(const uint32_t *__restrict__ counts, const int64_t *__restrict__ offsets,
                  int64_t n_waves, int64_t region, const uint32_t *__restrict__ k_src,
                  const uint64_t *__restrict__ v_src, uint32_t *__restrict__ k_dst,
                  uint64_t *__restrict__ v_dst) {
    for (int64_t g = blockIdx.x; g < n_waves; g += gridDim.x) {
        const int64_t n = counts[g], src = g * region, dst = offsets[g];
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
            k_dst[dst + i] = k_src[src + i];
            v_dst[dst + i] = v_src[src + i];
        }
    }
}

// Pass 2 without the count readback (n_records NULL): the compacted records [0, *count) are
// followed by sentinel keys up to the bound n_centres * T (all ones: with the sort's end bit they
// rank after every row, and the stable sort keeps them behind equal low bits), and range =
// {0, *count} limits the gather. With one owner every slot is kept and nothing is padded.
__global__ void __launch_bounds__(256)
    k_rec_pad(const uint32_t *__restrict__ count, int64_t bound, uint32_t *__restrict__ keys,
              uint64_t *__restrict__ vals, int64_t *__restrict__ range) {
    const int64_t n = *count;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        range[0] = 0;
        range[1] = n < bound ? n : bound;
    }
    for (int64_t i = n + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < bound;
         i += (int64_t)gridDim.x * blockDim.x) {
        keys[i] = 0xFFFFFFFFu;
        vals[i] = 0ull;
    }
}

// occurrence b (centre position of the walks) keyed by its node, for the node-order sort
__global__ void __launch_bounds__(256)
    k_occ_keys(const int32_t *__restrict__ walks, int64_t n_centres, int32_t L, int32_t R,
               uint32_t *__restrict__ keys, uint32_t *__restrict__ vals) {
    const int64_t per = L - 2 * R;
    for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < n_centres;
         b += (int64_t)gridDim.x * blockDim.x) {
        const int64_t w = b / per;
        keys[b] = static_cast<uint32_t>(walks[w * L + R + (b - w * per)]);
        vals[b] = static_cast<uint32_t>(b);
    }
}

// Small batches (<= OCC_SMALL_MAX centres, e.g. the reference's 64-walk batch: 4,480): the
// occurrence keys, their stable sort by node and the distinct nodes in ONE block — where the
// device-wide sort + unique took ~11 launches (merge sort, copies, lookback scans).
constexpr int OCC_SMALL_THREADS = 1024, OCC_SMALL_IPT = 8;
constexpr int64_t OCC_SMALL_MAX = (int64_t)OCC_SMALL_THREADS * OCC_SMALL_IPT;

__global__ void __launch_bounds__(OCC_SMALL_THREADS)
    k_occ_small(const int32_t *__restrict__ walks, int64_t n_centres, int32_t L, int32_t R,
                int32_t end_bit, uint32_t *__restrict__ keys_out, uint32_t *__restrict__ vals_out,
                uint32_t *__restrict__ touched, int64_t *__restrict__ n_touched) {
    using Sort = rocprim::block_radix_sort<uint32_t, OCC_SMALL_THREADS, OCC_SMALL_IPT, uint32_t>;
    using Scan = rocprim::block_scan<uint32_t, OCC_SMALL_THREADS>;
    __shared__ typename Sort::storage_type s_sort;
    __shared__ typename Scan::storage_type s_scan;
    __shared__ uint32_t s_last[OCC_SMALL_THREADS];
    const int t = threadIdx.x;
    const int64_t per = L - 2 * R;
    uint32_t k[OCC_SMALL_IPT], v[OCC_SMALL_IPT];
#pragma unroll
    for (int i = 0; i < OCC_SMALL_IPT; ++i) {   // blocked: thread t holds items t*IPT + i
        const int64_t b = (int64_t)t * OCC_SMALL_IPT + i;
        if (b < n_centres) {
            const int64_t w = b / per;
            k[i] = static_cast<uint32_t>(walks[w * L + R + (b - w * per)]);
            v[i] = static_cast<uint32_t>(b);
        } else {   // padding sorts last (stable: it follows every real item)
            k[i] = 0xFFFFFFFFu;
            v[i] = 0xFFFFFFFFu;
        }
    }
    Sort().sort(k, v, s_sort, 0, end_bit);   // stable: walk order within a node
#pragma unroll
    for (int i = 0; i < OCC_SMALL_IPT; ++i) {
        const int64_t b = (int64_t)t * OCC_SMALL_IPT + i;
        if (b < n_centres) {
            keys_out[b] = k[i];
            vals_out[b] = v[i];
        }
    }
    if (!touched) return;   // (block-uniform)
    s_last[t] = k[OCC_SMALL_IPT - 1];
    __syncthreads();
    uint32_t prev = t > 0 ? s_last[t - 1] : 0u;
    bool f[OCC_SMALL_IPT];
    uint32_t cnt = 0;
#pragma unroll
    for (int i = 0; i < OCC_SMALL_IPT; ++i) {
        const int64_t b = (int64_t)t * OCC_SMALL_IPT + i;
        f[i] = b < n_centres && (b == 0 || k[i] != prev);
        prev = k[i];
        cnt += f[i] ? 1u : 0u;
    }
    uint32_t off = 0, total = 0;
    Scan().exclusive_scan(cnt, off, 0u, total, s_scan);
#pragma unroll
    for (int i = 0; i < OCC_SMALL_IPT; ++i)
        if (f[i]) touched[off++] = k[i];
    if (t == 0) *n_touched = static_cast<int64_t>(total);
}

// the owner form's tail of the workspace (after the records part): the occurrence sort
struct OccSpace {
    uint32_t *k0, *k1, *v0, *v1;
    void *tmp;
    size_t tmp_bytes, total;
};

int plan_occ(int64_t n_centres, int64_t V, void *base, OccSpace *o, hipStream_t st) {
    size_t tmp = 0, utmp = 0;
    rocprim::double_buffer<uint32_t> kb(nullptr, nullptr), vb(nullptr, nullptr);
    if (sort_pairs(nullptr, tmp, kb, vb, static_cast<uint32_t>(n_centres), end_bit_for(V),
                   st) != hipSuccess ||
        rocprim::unique(nullptr, utmp, static_cast<const uint32_t *>(nullptr),
                        static_cast<uint32_t *>(nullptr), static_cast<int64_t *>(nullptr),
                        static_cast<size_t>(n_centres), rocprim::equal_to<uint32_t>(),
                        st) != hipSuccess) {
        dw::set_error("dw_sgns_owner: occurrence sort / unique size query failed");
        return DW_E_HIP;
    }
    if (utmp > tmp) tmp = utmp;
    const size_t a = align256((size_t)n_centres * 4);
    char *p = static_cast<char *>(base);
    o->k0 = reinterpret_cast<uint32_t *>(p);
    o->k1 = reinterpret_cast<uint32_t *>(p + a);
    o->v0 = reinterpret_cast<uint32_t *>(p + 2 * a);
    o->v1 = reinterpret_cast<uint32_t *>(p + 3 * a);
    o->tmp = p + 4 * a;
    o->tmp_bytes = tmp;
    o->total = 4 * a + align256(tmp);
    return DW_OK;
}

// the records' placement (k_out_claim's ranks, one owner or many): rank[slot], off[row] (the
// exclusive scan of the per-row counts, with one zero past the rows: off[local_rows] = their
// total) and the scan's temporary storage; between the records part and OccSpace
constexpr int PLACE_TILE = 4096;   // placement-scan counts per block (16 per thread; k_place_scan)

struct PlaceSpace {
    uint32_t *rank, *off;
    void *tmp;
    size_t tmp_bytes, total;
};

int plan_place(int64_t n_slots, int64_t local_rows, void *base, PlaceSpace *pl, hipStream_t st) {
    (void)st;
    const size_t tmp = static_cast<size_t>((local_rows + PLACE_TILE - 1) / PLACE_TILE) * 4;
    const size_t a = align256((size_t)(n_slots > 0 ? n_slots : 1) * 4);
    const size_t b = align256((size_t)(local_rows + 1) * 4);
    char *p = static_cast<char *>(base);
    pl->rank = reinterpret_cast<uint32_t *>(p);
    pl->off = reinterpret_cast<uint32_t *>(p + a);
    pl->tmp = p + a + b;
    pl->tmp_bytes = tmp;
    pl->total = a + b + align256(tmp);
    return DW_OK;
}

int owner_workspace(int64_t n_centres, int64_t T, int64_t local_rows, void *workspace,
                    size_t workspace_bytes, Workspace *ws, OwnerLayout *lay, hipStream_t st,
                    const char *what, int64_t V = 0, OccSpace *occ = nullptr,
                    PlaceSpace *place = nullptr) {
    *lay = owner_layout(n_centres, T);
    DW_REQUIRE(lay->total < 0x7FFFFFFF, "%s: too many records (%lld)", what,
               (long long)lay->total);
    DW_REQUIRE(lay->n_waves <= MAX_OWNER_WAVES, "%s: %lld pass-1 waves > %d", what,
               (long long)lay->n_waves, MAX_OWNER_WAVES);
    DW_REQUIRE(workspace != nullptr, "%s: needs the records workspace", what);
    int rc = plan_workspace(lay->total, local_rows, workspace, ws, st);
    if (rc != DW_OK) return rc;
    PlaceSpace pl;
    rc = plan_place(n_centres * T, local_rows, static_cast<char *>(workspace) + ws->total, &pl, st);
    if (rc != DW_OK) return rc;
    if (place) *place = pl;
    size_t need = ws->total + pl.total;
    if (occ) {
        rc = plan_occ(n_centres > 0 ? n_centres : 1, V, static_cast<char *>(workspace) + need, occ,
                      st);
        if (rc != DW_OK) return rc;
        need += occ->total;
    }
    DW_REQUIRE(workspace_bytes >= need, "%s: workspace too small (%zu < %zu)", what,
               workspace_bytes, need);
    return DW_OK;
}

// The global batch's centres in node order into occ.v0 (their nodes in occ.k0); touched != NULL:
// also the distinct nodes, sorted, and their count (device int64).
int owner_order(const SgnsArgs &a, const OccSpace &occ, uint32_t *touched, int64_t *n_touched,
                hipStream_t st) {
    if (a.batch <= OCC_SMALL_MAX) {
        hipLaunchKernelGGL(k_occ_small, dim3(1), dim3(OCC_SMALL_THREADS), 0, st, a.walks,
                           a.batch, a.L, a.R, end_bit_for(a.V), occ.k0, occ.v0, touched,
                           n_touched);
        DW_LAUNCH_CHECK("dw_sgns_owner/occ_small");
        return DW_OK;
    }
    int64_t ob = (a.batch + 255) / 256;
    if (ob > grid_cap(8)) ob = grid_cap(8);
    hipLaunchKernelGGL(k_occ_keys, dim3((unsigned)ob), dim3(256), 0, st, a.walks, a.batch, a.L,
                       a.R, occ.k0, occ.v0);
    DW_LAUNCH_CHECK("dw_sgns_owner/occ_keys");
    rocprim::double_buffer<uint32_t> kb(occ.k0, occ.k1), vb(occ.v0, occ.v1);
    size_t tb = occ.tmp_bytes;
    if (sort_pairs(occ.tmp, tb, kb, vb, static_cast<uint32_t>(a.batch), end_bit_for(a.V),
                   st) != hipSuccess) {
        dw::set_error("dw_sgns_owner: occurrence sort failed");
        return DW_E_HIP;
    }
    if (kb.current() != occ.k0) {  // keep the order where pass 1 and the unique step read it
        const size_t nb = static_cast<size_t>(a.batch) * sizeof(uint32_t);
        if (hipMemcpyAsync(occ.k0, kb.current(), nb, hipMemcpyDeviceToDevice, st) != hipSuccess ||
            hipMemcpyAsync(occ.v0, vb.current(), nb, hipMemcpyDeviceToDevice, st) != hipSuccess) {
            dw::set_error("dw_sgns_owner: occurrence copy failed");
            return DW_E_HIP;
        }
    }
    if (touched) {
        size_t ub = occ.tmp_bytes;
        if (rocprim::unique(occ.tmp, ub, static_cast<const uint32_t *>(occ.k0), touched, n_touched,
                            static_cast<size_t>(a.batch), rocprim::equal_to<uint32_t>(),
                            st) != hipSuccess) {
            dw::set_error("dw_sgns_owner: distinct centres failed");
            return DW_E_HIP;
        }
    }
    return DW_OK;
}

int launch_owner_prepare(SgnsArgs a, int64_t local_rows, uint32_t *touched, int64_t *n_touched,
                         void *workspace, size_t workspace_bytes, hipStream_t st) {
    const int64_t T = (int64_t)a.C * (1 + a.K);
    Workspace ws;
    OwnerLayout lay;
    OccSpace occ;
    int rc = owner_workspace(a.batch, T, local_rows, workspace, workspace_bytes, &ws, &lay, st,
                             "dw_sgns_owner_prepare", a.V, &occ);
    if (rc != DW_OK) return rc;
    if (a.batch == 0) {
        if (n_touched && hipMemsetAsync(n_touched, 0, sizeof(int64_t), st) != hipSuccess) {
            dw::set_error("dw_sgns_owner_prepare: count reset failed");
            return DW_E_HIP;
        }
        return DW_OK;
    }
    return owner_order(a, occ, touched, n_touched, st);
}

int launch_owner_pass1(SgnsArgs a, int64_t local_rows, int32_t order_ready, void *workspace,
                       size_t workspace_bytes, hipStream_t st) {
    const int64_t T = (int64_t)a.C * (1 + a.K);
    DW_REQUIRE(a.n_owners >= 1 && a.owner >= 0 && a.owner < a.n_owners,
               "dw_sgns_owner_pass1: owner %d of %d", a.owner, a.n_owners);
    DW_REQUIRE(local_rows * a.n_owners >= a.V, "dw_sgns_owner_pass1: %lld local rows x %d owners "
               "do not cover %lld rows", (long long)local_rows, a.n_owners, (long long)a.V);
    DW_REQUIRE(a.V <= 0x7FFFFFFF, "dw_sgns_owner_pass1: vocab_size must be < 2^31");
    DW_REQUIRE((a.d == 64 || a.d == 128 || a.d == 256 || a.d == 512) && T <= G16_TMAX,
               "dw_sgns_owner_pass1: needs d in {64, 128, 256, 512} (got %d) and 2R(1+K) <= %d",
               a.d, G16_TMAX);
    Workspace ws;
    OwnerLayout lay;
    OccSpace occ;
    PlaceSpace pl;
    int rc = owner_workspace(a.batch, T, local_rows, workspace, workspace_bytes, &ws, &lay, st,
                             "dw_sgns_owner_pass1", a.V, &occ, &pl);
    if (rc != DW_OK) return rc;
    g_timer.mark(0, st);
    // n_owners > 1: per-wave regions in (k0, v0), compacted into (k1, v1); one owner keeps
    // every slot, so the regions tile (k1, v1) densely and pass 1 writes there directly;
    // placed (order_ready & 2, after dw_sgns_owner_out_catch_up with flags & 1): each record
    // straight to its row's segment of (k1, v1)
    const bool placed = (order_ready & 2) != 0;
    // coefficients in (order_ready & 4, after dw_sgns_owner_out_rows): the centre gradient only
    const bool coefin = (order_ready & 4) != 0;
    DW_REQUIRE(!coefin || placed, "dw_sgns_owner_pass1: the coefficients come with the placed "
               "records (order_ready & 2)");
    DW_REQUIRE(!(order_ready & 8) || coefin, "dw_sgns_owner_pass1: walk order (order_ready & 8) "
               "is the coefficients-in form's (order_ready & 4)");
    const bool dense = a.n_owners == 1 || placed;
    if (placed) {
        a.place_rank = pl.rank;
        a.place_off = pl.off;
    }
    a.rec_key = dense ? ws.k1 : ws.k0;
    a.rec_val = dense ? ws.v1 : ws.v0;
    if (coefin) a.rec_val = ws.v0;   // k_out_rows' coefficients by slot (float) there
    a.count_out = dense ? ws.count : nullptr;
    a.rec_counts = ws.wave_counts;
    a.region = lay.region;
    a.occ_per_wave = lay.region / T;
    if (a.batch > 0) {
        if (order_ready & 8) {     // walk order (one rank, coefficients in: no node order needed)
            a.occ = nullptr;
        } else {
            if (!(order_ready & 1)) {  // the centres in node order (stable: walk order in a node)
                rc = owner_order(a, occ, nullptr, nullptr, st);
                if (rc != DW_OK) return rc;
            }
            a.occ = occ.v0;
        }
        int32_t fl = 0;
        rc = exact_of(a.g_in, a.V * a.d, &a.fx_in, &fl, "dw_sgns_owner_pass1");
        if (rc != DW_OK) return rc;
        rc = coefin ? launch_pass1_g16<true, true, true>(a, st)
                    : launch_pass1_g16<true, true>(a, st);
        if (rc != DW_OK) return rc;
        if (a.fx_in.acc && !(fl & (DW_EXACT_DEFER | DW_EXACT_ADAM))) {   // one rank: the centres' exact sums
            int64_t cb = (a.batch + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
            if (cb > grid_cap(8)) cb = grid_cap(8);
            hipLaunchKernelGGL(k_fixed_centres<true>, dim3((unsigned)cb),
                               dim3(WAVES_PER_BLOCK * WAVE), 0, st, a);
            DW_LAUNCH_CHECK("dw_sgns_owner_pass1/fixed_centres");
        }
        if (!dense) {
            hipLaunchKernelGGL(k_wave_scan, dim3(1), dim3(1024), 0, st, ws.wave_counts,
                               lay.n_waves, ws.wave_offsets, ws.count);
            DW_LAUNCH_CHECK("dw_sgns_owner_pass1/scan");
            int64_t cb = lay.n_waves < 65536 ? lay.n_waves : 65536;
            hipLaunchKernelGGL(k_rec_compact, dim3((unsigned)cb), dim3(256), 0, st,
                               ws.wave_counts, ws.wave_offsets, lay.n_waves, lay.region, ws.k0,
                               ws.v0, ws.k1, ws.v1);
            DW_LAUNCH_CHECK("dw_sgns_owner_pass1/compact");
        }
    } else if (hipMemsetAsync(ws.count, 0, sizeof(uint32_t), st) != hipSuccess) {
        dw::set_error("dw_sgns_owner_pass1: counter reset failed");
        return DW_E_HIP;
    }
    g_timer.mark(1, st);
    return DW_OK;
}

int launch_owner_pass2(int64_t n_centres, int64_t T, int64_t local_rows, int32_t d,
                       const float *w_in, float *g_out, const OutAdam *oa, void *workspace,
                       size_t workspace_bytes, int64_t *n_records, hipStream_t st,
                       bool placed = false) {
    Workspace ws;
    OwnerLayout lay;
    int rc = owner_workspace(n_centres, T, local_rows, workspace, workspace_bytes, &ws, &lay, st,
                             "dw_sgns_owner_pass2");
    if (rc != DW_OK) return rc;
    const int64_t bound = n_centres * T;
    const int64_t *range = nullptr;
    int64_t n_rec = bound;
    if (placed) {
        // pass 1 wrote every record into its row's segment of (k1, v1): no sort; the range
        // [0, count) was written by the catch-up (k_place_scan); the grid is sized for the bound
        DW_REQUIRE(!n_records, "dw_sgns_owner_pass2: placed records need n_records NULL");
        g_timer.mark(2, st);
        if (bound > 0 || oa) {
            rc = launch_pass2(ws.k1, ws.v1, bound, w_in, g_out, d, oa, local_rows, st,
                              bound > 0 ? ws.bounds : nullptr);
            if (rc != DW_OK) return rc;
        }
        g_timer.mark(3, st);
        return DW_OK;
    }
    if (n_records) {
        // the record count decides the sort's size on the host: one stream synchronisation
        uint32_t n = 0;
        if (hipMemcpyAsync(&n, ws.count, sizeof(n), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            dw::set_error("dw_sgns_owner_pass2: reading the record count failed");
            return DW_E_HIP;
        }
        n_rec = static_cast<int64_t>(n) < bound ? n : bound;
        *n_records = n_rec;
    } else if (bound > 0) {
        // no readback: sort the bound with the tail padded, gather [0, count) (k_rec_pad)
        int64_t pb = (bound + 255) / 256;
        if (pb > grid_cap(4)) pb = grid_cap(4);
        hipLaunchKernelGGL(k_rec_pad, dim3((unsigned)pb), dim3(256), 0, st, ws.count, bound,
                           ws.k1, ws.v1, ws.bounds);
        DW_LAUNCH_CHECK("dw_sgns_owner_pass2/pad");
        range = ws.bounds;
    }
    const uint32_t *keys = ws.k1;  // compacted by pass 1
    const uint64_t *vals = ws.v1;
    if (n_rec > 0) {
        rocprim::double_buffer<uint32_t> kb(ws.k1, ws.k0);
        rocprim::double_buffer<uint64_t> vb(ws.v1, ws.v0);
        size_t cub_bytes = ws.cub_bytes;
        hipError_t e = sort_pairs(ws.cub, cub_bytes, kb, vb, static_cast<uint32_t>(n_rec),
                                  end_bit_for(local_rows), st);
        if (e != hipSuccess) {
            dw::set_error("dw_sgns_owner_pass2: records sort failed: %s", hipGetErrorString(e));
            return DW_E_HIP;
        }
        keys = kb.current();
        vals = vb.current();
    }
    g_timer.mark(2, st);
    if (n_rec > 0 || oa) {
        rc = launch_pass2(keys, vals, n_rec, w_in, g_out, d, oa, local_rows, st, range);
        if (rc != DW_OK) return rc;
    }
    g_timer.mark(3, st);
    return DW_OK;
}

// ---- SkipGram.forward logits and its backward (autograd path of the reference API) ----------
// logits[b, n] = <mean_p w_in[inputs[b, p]], w_out[outputs[b, n]]> (SkipGram: P = 1; CBOW:
// P = the context width). One wave per row b.
__global__ void __launch_bounds__(256)
    k_logits(const int64_t *__restrict__ inputs, int32_t P, const int64_t *__restrict__ outputs,
             int64_t B, int32_t N, int64_t V, int32_t d, const float *__restrict__ w_in,
             const float *__restrict__ w_out, int32_t proba, float *__restrict__ logits,
             int32_t *status) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t n_waves = (int64_t)gridDim.x * (blockDim.x / WAVE);
    for (int64_t b = blockIdx.x * (int64_t)(blockDim.x / WAVE) + threadIdx.x / WAVE; b < B;
         b += n_waves) {
        const bool in_ok = inputs_ok(inputs, b, P, V);
        for (int n = 0; n < N; ++n) {
            const int64_t o = outputs[b * N + n];
            float s = 0.f;
            const bool ok = in_ok && o >= 0 && o < V;
            if (ok)
                for (int e = lane; e < d; e += WAVE)
                    s += pooled(inputs, b, P, w_in, d, e) * w_out[o * d + e];
            s = dw::wave_sum(s);
            if (lane == 0) {
                if (!ok) dw::status_or(status, DW_S_BAD_INDEX);
                logits[b * N + n] = proba ? sigmoidf(s) : s;
            }
        }
    }
}

__global__ void __launch_bounds__(256)
    k_logits_bwd(const int64_t *__restrict__ inputs, int32_t P,
                 const int64_t *__restrict__ outputs, int64_t B, int32_t N, int64_t V, int32_t d,
                 const float *__restrict__ w_in, const float *__restrict__ w_out,
                 const float *__restrict__ dl, float *__restrict__ g_in,
                 float *__restrict__ g_out, int32_t *status) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t n_waves = (int64_t)gridDim.x * (blockDim.x / WAVE);
    for (int64_t b = blockIdx.x * (int64_t)(blockDim.x / WAVE) + threadIdx.x / WAVE; b < B;
         b += n_waves) {
        if (!inputs_ok(inputs, b, P, V)) {
            if (lane == 0) dw::status_or(status, DW_S_BAD_INDEX);
            continue;
        }
        for (int e0 = 0; e0 < d; e0 += WAVE) {
            const int e = e0 + lane;
            float gh = 0.f;
            const float he = e < d ? pooled(inputs, b, P, w_in, d, e) : 0.f;
            for (int n = 0; n < N; ++n) {
                const int64_t o = outputs[b * N + n];
                if (o < 0 || o >= V) continue;
                const float g = dl[b * N + n];
                if (e < d) {
                    gh += g * w_out[o * d + e];
                    atomicAdd(g_out + o * d + e, g * he);
                }
            }
            if (e < d) {  // mean backward: every pooled input row receives gh / P
                const float gi = P == 1 ? gh : gh / static_cast<float>(P);
                for (int p = 0; p < P; ++p) atomicAdd(g_in + inputs[b * P + p] * d + e, gi);
            }
        }
    }
}

// ---- max_norm renormalisation (nn.Embedding(max_norm=...), torch embedding_renorm_) ----------
// The referenced ids are sorted (duplicates adjacent) so each distinct row is renormalised once:
// norm = ||row||_2 (float); if norm > max_norm: row *= float(max_norm / (norm + 1e-7)) with the
// ratio in double, as the reference's CPU kernel computes it.
__global__ void __launch_bounds__(256)
    k_renorm_keys(const int64_t *__restrict__ ids, int64_t n, int64_t V,
                  uint32_t *__restrict__ keys, int32_t *status) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t id = ids[i];
    const bool ok = id >= 0 && id < V;
    if (!ok) dw::status_or(status, DW_S_BAD_INDEX);
    keys[i] = static_cast<uint32_t>(ok ? id : V);  // V = "skip"
}

__global__ void __launch_bounds__(256)
    k_renorm_rows(const uint32_t *__restrict__ keys, int64_t n, int64_t V, float *__restrict__ w,
                  int32_t d, double max_norm) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t n_waves = (int64_t)gridDim.x * (blockDim.x / WAVE);
    for (int64_t i = blockIdx.x * (int64_t)(blockDim.x / WAVE) + threadIdx.x / WAVE; i < n;
         i += n_waves) {
        const uint32_t k = keys[i];
        if (k >= V || (i > 0 && keys[i - 1] == k)) continue;
        float *row = w + static_cast<int64_t>(k) * d;
        float ss = 0.f;
        for (int e = lane; e < d; e += WAVE) ss += row[e] * row[e];
        const float norm = sqrtf(dw::wave_sum(ss));
        if (static_cast<double>(norm) > max_norm) {
            const float scale = static_cast<float>(max_norm / (static_cast<double>(norm) + 1e-7));
            for (int e = lane; e < d; e += WAVE) row[e] *= scale;
        }
    }
}

// Device negatives exactly as the fused kernels draw them (noise_id): ids[(b*C + j)*K + k].
__global__ void __launch_bounds__(256)
    k_noise_fill(int64_t batch, int32_t C, int32_t K, int64_t V, uint32_t k0, uint32_t k1,
                 uint64_t noise_offset, int64_t *__restrict__ out) {
    const int64_t n = batch * C * K;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t b = i / (static_cast<int64_t>(C) * K);
        const int slot = static_cast<int>(i - b * C * K);  // j*K + k
        const uint64_t g = noise_offset + static_cast<uint64_t>(b);
        const dw::U4 r = dw::philox<DW_NOISE_ROUNDS>(   // the pair of slot (noise_pair)
            dw::U4{static_cast<uint32_t>(g), static_cast<uint32_t>(g >> 32),
                   static_cast<uint32_t>(slot >> 1), TAG_SGNS},
            k0, k1);
        const uint64_t Vu = static_cast<uint64_t>(V);
        out[i] = static_cast<int64_t>((slot & 1) ? dw::bounded64(r.z, r.w, Vu)
                                                 : dw::bounded64(r.x, r.y, Vu));
    }
}

using RenormSortConfig = RecordSortConfig;

SgnsArgs base_args(int64_t V, int32_t dim, int32_t K, const float *w_in, const float *w_out,
                   float *g_in, float *g_out, const int64_t *noise, uint64_t seed,
                   uint64_t noise_offset, float grad_scale, double *loss_acc, int32_t *status) {
    SgnsArgs a{};
    a.n_in = 1;
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
    a.dyn = dw::bound_step_scalars();
    return a;
}

// Lazy out slice (dw_sgns_owner_out_catch_up), before pass 1: every owned output row a slot of
// this batch references must be brought current to step - 1 (its deferred g = 0 steps replayed
// through adam_elem with hist's scalars), so pass 1 reads the rows the dense update would hold.
// This kernel lists them once each: one wave per centre, lane t = slot t (T <= 64); a row is
// claimed by exactly one lane in the launch — atomicMax(claim[row], step) returning < step — and
// listed when its last claim is older than step - 1 (a row the previous step claimed held a
// record there, so its lazy gather already brought it to step - 1); the wave's listed rows are
// appended to `list` with one counter atomic per block. dw_adam_rows then replays the listed
// rows, all in parallel.
// Placement (count != NULL): every slot also adds 1 to its row's count (zero between steps: the
// lazy gather clears the counts of the rows it steps); the value it got back is its rank among
// the step's slots of that row, kept per slot (rank[b * T + t]). An exclusive scan of the counts
// then gives every row a segment of the records array, and pass 1 writes each record at
// off[row] + rank: the records come out grouped by row with no sort (the 64-walk batch: 269K
// records, whose radix sort was ~10 launches and ~85 us of the step). The order of a row's
// records is the order the atomics resolved — as nondeterministic as the float atomics of rows
// that straddle two gather chunks. (The two atomics of a slot are independent: one round trip.)
// CLAIM_TRIPS centres per wave, their row ids and atomics issued together (independent chains
// in flight), and ONE list atomic per block for all of them: a same-address atomic per block
// serialises (1,120 blocks of one trip each were ~36 us at C3's 64-walk batch).
// !CLAIM (the rows-major step, dw_sgns_owner_out_rows): the ranks alone — k_out_rows replays
// every row right before its step, so no row is listed or caught up here.
// dw_sgns_owner_touch_claim: the batch's distinct centre nodes (the in rows a step touches),
// unsorted — one rank needs no common order of them. claim[node] = step by atomicMax; the
// first claimer of a node appends it, one list atomic per wave. (k_occ_small's one-block sort +
// unique gave the sorted list in 30-40 us at C3's 64-walk batch, on the step's critical path
// before the in-table catch-up; this takes a few microseconds.)
__global__ void __launch_bounds__(256)
    k_touch_claim(const int32_t *__restrict__ walks, int64_t n_centres, int32_t L, int32_t R,
                  int64_t V, int32_t *__restrict__ claim, int32_t step_arg,
                  const dw_step_scalars *__restrict__ dyn, int32_t delta,
                  uint32_t *__restrict__ touched, unsigned long long *__restrict__ n_touched,
                  uint32_t *__restrict__ fresh, unsigned long long *__restrict__ n_fresh) {
    const int32_t step = dw::eff_step(dyn, delta, step_arg);
    const int lane = threadIdx.x & (WAVE - 1);
    const uint64_t lt = (1ull << lane) - 1ull;
    const int64_t per = L - 2 * R;
    for (int64_t base = ((int64_t)blockIdx.x * 4 + threadIdx.x / WAVE) * WAVE; base < n_centres;
         base += (int64_t)gridDim.x * 4 * WAVE) {
        const int64_t b = base + lane;
        bool mine = false, cold = false;
        int32_t node = 0;
        if (b < n_centres) {
            const int64_t w = b / per;
            node = walks[w * L + R + (b - w * per)];
            // (an out-of-range id is reported by the SGNS pass)
            if (node >= 0 && node < V) {
                const int32_t old = atomicMax(claim + node, step);
                mine = old < step;
                cold = mine && old < step - 1;   // not a centre of step - 1
            }
        }
        const uint64_t mask = __ballot(mine);
        if (mask == 0) continue;
        unsigned long long at = 0;
        if (lane == 0) at = atomicAdd(n_touched, static_cast<unsigned long long>(__popcll(mask)));
        at = (static_cast<unsigned long long>(__builtin_amdgcn_readfirstlane(
                  static_cast<uint32_t>(at >> 32))) << 32) |
             __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(at));
        if (mine) touched[at + __popcll(mask & lt)] = static_cast<uint32_t>(node);
        if (!fresh) continue;
        const uint64_t cmask = __ballot(cold);
        if (cmask == 0) continue;
        unsigned long long ct = 0;
        if (lane == 0) ct = atomicAdd(n_fresh, static_cast<unsigned long long>(__popcll(cmask)));
        ct = (static_cast<unsigned long long>(__builtin_amdgcn_readfirstlane(
                  static_cast<uint32_t>(ct >> 32))) << 32) |
             __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(ct));
        if (cold) fresh[ct + __popcll(cmask & lt)] = static_cast<uint32_t>(node);
    }
}

constexpr int CLAIM_TRIPS = 4;
// (the ranks alone: one centre per wave, four times the waves — the atomics are the chain)
template <bool CLAIM, int TRIPS = CLAIM ? CLAIM_TRIPS : 1>
__global__ void __launch_bounds__(WAVES_PER_BLOCK *WAVE)
    k_out_claim(SgnsArgs a, int32_t *__restrict__ claim, int32_t step_arg, int32_t delta,
                uint32_t *__restrict__ list, unsigned long long *__restrict__ n_list,
                uint32_t *__restrict__ count, uint32_t *__restrict__ rank,
                uint32_t *__restrict__ rowid) {
    const int32_t step = dw::eff_step(a.dyn, delta, step_arg);   // graph replay: from the block
    __shared__ uint32_t s_rows[WAVES_PER_BLOCK][TRIPS * WAVE];
    __shared__ uint32_t s_cnt[WAVES_PER_BLOCK];
    __shared__ unsigned long long s_base;
    const int lane = threadIdx.x & (WAVE - 1);
    const int wv = threadIdx.x / WAVE;
    const int T = a.C * (1 + a.K);
    const int64_t per = a.L - 2 * a.R;
    const int64_t tile = (int64_t)WAVES_PER_BLOCK * TRIPS;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int64_t b0 = (int64_t)blockIdx.x * tile; b0 < a.batch; b0 += (int64_t)gridDim.x * tile) {
        int64_t o[TRIPS];   // each trip's row (-1: none)
#pragma unroll
        for (int k = 0; k < TRIPS; ++k) {
            const int64_t b = b0 + k * WAVES_PER_BLOCK + wv;
            o[k] = -1;
            if (b < a.batch && lane < T) {
                const int64_t w = b / per, i = a.R + b % per;
                const int64_t r = row_id<true>(a, b, a.walks + w * a.L, i, lane);
                if (r < 0 || r >= a.V)
                    dw::status_or(a.status, DW_S_BAD_INDEX);
                else if (r % a.n_owners == a.owner)
                    o[k] = r / a.n_owners;
            }
        }
        bool mine[TRIPS];
#pragma unroll
        for (int k = 0; k < TRIPS; ++k) {
            mine[k] = false;
            if (o[k] >= 0) {
                const int64_t b = b0 + k * WAVES_PER_BLOCK + wv;
                if (CLAIM) mine[k] = atomicMax(claim + o[k], step) < step - 1;
                if (count) rank[b * T + lane] = atomicAdd(count + o[k], 1u);
            }
            if (!CLAIM) {   // every slot's local row (~0: none) for k_place_slots
                const int64_t b = b0 + k * WAVES_PER_BLOCK + wv;
                if (b < a.batch && lane < T)
                    rowid[b * T + lane] = o[k] >= 0 ? static_cast<uint32_t>(o[k]) : 0xFFFFFFFFu;
            }
        }
        if constexpr (!CLAIM) continue;
        uint32_t n_mine = 0;   // wave-uniform
#pragma unroll
        for (int k = 0; k < TRIPS; ++k) {
            const uint64_t mask = __ballot(mine[k]);
            if (mine[k]) s_rows[wv][n_mine + __popcll(mask & lt)] = static_cast<uint32_t>(o[k]);
            n_mine += __popcll(mask);
        }
        if (lane == 0) s_cnt[wv] = n_mine;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t tot = 0;
            for (int k = 0; k < WAVES_PER_BLOCK; ++k) tot += s_cnt[k];
            s_base = tot ? atomicAdd(n_list, static_cast<unsigned long long>(tot)) : 0ull;
        }
        __syncthreads();
        unsigned long long base = s_base;
        for (int k = 0; k < wv; ++k) base += s_cnt[k];
        for (uint32_t e = lane; e < n_mine; e += WAVE) list[base + e] = s_rows[wv][e];
        __syncthreads();   // s_rows / s_cnt / s_base are rewritten next tile
    }
}

// The rows-major step, after the placement scan: slot s = b T + t (k_out_claim gave it its
// local row rowid[s] and its rank among that row's slots) goes to off[row] + rank[s] —
// keys[pos] = the row, vals[pos] = (the slot's centre node << 32) | s | (t is a context, not a
// negative) << 31: k_out_rows reads a record in one load, with no walk lookup behind it.
__global__ void __launch_bounds__(256)
    k_place_slots(int64_t n_slots, const uint32_t *__restrict__ rowid,
                  const uint32_t *__restrict__ rank, const uint32_t *__restrict__ off,
                  uint32_t *__restrict__ keys, uint64_t *__restrict__ vals,
                  const int32_t *__restrict__ walks, int32_t L, int32_t R, int32_t T,
                  int32_t rpc) {
    const uint32_t per = static_cast<uint32_t>(L - 2 * R);
    for (int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x; s < n_slots;
         s += (int64_t)gridDim.x * 256) {
        const uint32_t o = rowid[s];
        if (o == 0xFFFFFFFFu) continue;   // a bad id or another owner's row
        const uint32_t pos = off[o] + rank[s];
        const uint32_t su = static_cast<uint32_t>(s);
        const uint32_t b = su / static_cast<uint32_t>(T);
        const uint32_t w = b / per;
        const int32_t cid = walks[static_cast<int64_t>(w) * L + R + (b - w * per)];
        const uint32_t ctx = ((su - b * static_cast<uint32_t>(T)) % static_cast<uint32_t>(rpc)) == 0u
                                 ? 0x80000000u : 0u;
        keys[pos] = o;
        vals[pos] = (static_cast<uint64_t>(static_cast<uint32_t>(cid)) << 32) | su | ctx;
    }
}

// The placement offsets in two short launches instead of a lookback scan (a 1M-row slice's
// counts are 4 MB: the scan's cost is its latency, ~25 us as rocprim's decoupled lookback at
// C3's 64-walk batch). k_place_sums: each 256-thread block sums its PLACE_TILE counts;
// k_place_scan: each block adds the sums of the blocks before it (at most a few hundred, read
// from L2) and scans its tile; the last block also writes the gather's range {0, total}.

__global__ void __launch_bounds__(256)
    k_place_sums(const uint32_t *__restrict__ counts, int64_t n, uint32_t *__restrict__ sums) {
    __shared__ uint32_t s_w[4];
    const int64_t a = (int64_t)blockIdx.x * PLACE_TILE;
    uint32_t t = 0;
    for (int k = 0; k < PLACE_TILE / 256; ++k) {
        const int64_t i = a + k * 256 + threadIdx.x;
        t += i < n ? counts[i] : 0u;
    }
    for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) sums[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

// The counts are cleared here once read (coalesced, the tile's own lines) — the step's kernels
// then leave them alone, where each stepped row's reset was a scattered 4-B write.
__global__ void __launch_bounds__(256)
    k_place_scan(uint32_t *__restrict__ counts, int64_t n, const uint32_t *__restrict__ sums,
                 uint32_t *__restrict__ off, int64_t *__restrict__ range) {
    __shared__ uint32_t s_w[4];
    __shared__ uint32_t s_base;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // this block's base: the sums of the blocks before it
    uint32_t b = 0;
    for (int64_t j = threadIdx.x; j < blockIdx.x; j += 256) b += sums[j];
    for (int o = 32; o > 0; o >>= 1) b += __shfl_xor(b, o, 64);
    if (lane == 0) s_w[wv] = b;
    __syncthreads();
    if (threadIdx.x == 0) s_base = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
    // thread k holds counts [a + 16k, a + 16k + 16): its sum, the block's exclusive scan of them
    const int64_t a = (int64_t)blockIdx.x * PLACE_TILE + 16 * threadIdx.x;
    uint32_t c[16], t = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        c[k] = a + k < n ? counts[a + k] : 0u;
        t += c[k];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (c[k] != 0u) counts[a + k] = 0u;
    uint32_t x = t;   // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    __syncthreads();
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    uint32_t pre = s_base;
    for (int w = 0; w < wv; ++w) pre += s_w[w];
    uint32_t run = pre + x - t;   // exclusive prefix of this thread's first count
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        if (a + k < n) off[a + k] = run;
        run += c[k];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 255) {   // off[n]: the total
        off[n] = run;
        range[0] = 0;
        range[1] = static_cast<int64_t>(run);
    }
}

}  // namespace

extern "C" {

int dw_sgns_owner_out_catch_up(const int32_t *walks, int64_t n_walks, int32_t walk_length,
                               int32_t context_radius, int32_t neg_samples, int64_t vocab_size,
                               int32_t dim, int32_t owner, int32_t n_owners, int64_t local_rows,
                               const int64_t *noise, uint64_t seed, uint64_t noise_offset,
                               float *w_out_local, float *m_out, float *v_out,
                               int32_t *last_step, int32_t *claim, uint32_t *counts,
                               uint32_t *rows_buf, int64_t *n_rows, const float *hist,
                               int32_t step, int32_t flags, int32_t *status, void *workspace,
                               size_t workspace_bytes, void *stream) {
    DW_REQUIRE(context_radius >= 1 && walk_length >= 2 * context_radius + 1 && n_walks >= 0 &&
                   dim >= 1 && vocab_size >= 1 && neg_samples >= 0 && n_owners >= 1 &&
                   owner >= 0 && owner < n_owners && step >= 1,
               "dw_sgns_owner_out_catch_up: bad sizes");
    DW_REQUIRE(2 * (int64_t)context_radius * (1 + neg_samples) <= WAVE,
               "dw_sgns_owner_out_catch_up: 2R(1+K) must be <= 64");
    DW_REQUIRE(local_rows * n_owners >= vocab_size,
               "dw_sgns_owner_out_catch_up: the owners' rows do not cover the vocabulary");
    if (n_walks == 0) return DW_OK;
    DW_REQUIRE(walks && w_out_local && m_out && v_out && last_step && claim && rows_buf &&
                   n_rows && hist && status,
               "dw_sgns_owner_out_catch_up: null pointer");
    DW_REQUIRE((flags & ~7) == 0, "dw_sgns_owner_out_catch_up: flags must be a set of 1 | 2 | 4");
    const bool place = (flags & 1) != 0, p_only = (flags & 2) != 0;
    const bool rows_major = (flags & 4) != 0;   // dw_sgns_owner_out_rows replays the rows itself
    DW_REQUIRE(!place || counts, "dw_sgns_owner_out_catch_up: placing needs the row counts");
    DW_REQUIRE(!rows_major || place, "dw_sgns_owner_out_catch_up: the rows-major step places "
               "the records (flags & 1)");
    hipStream_t st = dw::as_stream(stream);
    const dw_step_scalars *dyn = nullptr;
    int32_t delta = 0;
    int rc = dw::bound_step_rel(step, &dyn, &delta, "dw_sgns_owner_out_catch_up");
    if (rc != DW_OK) return rc;
    SgnsArgs a = base_args(vocab_size, dim, neg_samples, nullptr, w_out_local, nullptr, nullptr,
                           noise, seed, noise_offset, 0.f, nullptr, status);
    a.walks = walks;
    a.L = walk_length;
    a.R = context_radius;
    a.batch = n_walks * (walk_length - 2 * context_radius);
    a.C = 2 * context_radius;
    a.owner = owner;
    a.n_owners = n_owners;
    if (!(flags & 4) && hipMemsetAsync(n_rows, 0, sizeof(int64_t), st) != hipSuccess) {
        dw::set_error("dw_sgns_owner_out_catch_up: counter reset failed");
        return DW_E_HIP;
    }
    const int64_t T = (int64_t)a.C * (1 + a.K);
    Workspace ws;
    OwnerLayout lay;
    PlaceSpace pl{};
    if (place) {
        rc = owner_workspace(a.batch, T, local_rows, workspace, workspace_bytes, &ws, &lay, st,
                             "dw_sgns_owner_out_catch_up", vocab_size, nullptr, &pl);
        if (rc != DW_OK) return rc;
    }
    const int64_t ctile = (int64_t)WAVES_PER_BLOCK * (rows_major ? 1 : CLAIM_TRIPS);
    int64_t blocks = (a.batch + ctile - 1) / ctile;
    if (blocks > grid_cap(8)) blocks = grid_cap(8);
    if (blocks < 1) blocks = 1;
    // (rows-major: every slot's row into the records' spare key buffer, k0)
    if (rows_major)
        hipLaunchKernelGGL(k_out_claim<false>, dim3((unsigned)blocks),
                           dim3(WAVES_PER_BLOCK * WAVE), 0, st, a, claim, step, delta, rows_buf,
                           reinterpret_cast<unsigned long long *>(n_rows), counts, pl.rank,
                           ws.k0);
    else
        hipLaunchKernelGGL(k_out_claim<true>, dim3((unsigned)blocks),
                           dim3(WAVES_PER_BLOCK * WAVE), 0, st, a, claim, step, delta, rows_buf,
                           reinterpret_cast<unsigned long long *>(n_rows),
                           place ? counts : nullptr, place ? pl.rank : nullptr, nullptr);
    DW_LAUNCH_CHECK("dw_sgns_owner_out_catch_up/claim");
    if (place) {   // every row's segment of the records: the scan of the counts (+ the total)
        const int64_t nb = (local_rows + PLACE_TILE - 1) / PLACE_TILE;
        DW_REQUIRE(pl.tmp_bytes >= (size_t)nb * 4, "dw_sgns_owner_out_catch_up: scan scratch");
        uint32_t *sums = static_cast<uint32_t *>(pl.tmp);
        hipLaunchKernelGGL(k_place_sums, dim3((unsigned)nb), dim3(256), 0, st, counts, local_rows,
                           sums);
        hipLaunchKernelGGL(k_place_scan, dim3((unsigned)nb), dim3(256), 0, st, counts, local_rows,
                           sums, pl.off, ws.bounds);
        DW_LAUNCH_CHECK("dw_sgns_owner_out_catch_up/place");
    }
    if (rows_major) {   // the slots into their rows' segments; no catch-up
        int64_t pb = (a.batch * T + 255) / 256;
        if (pb > grid_cap(8)) pb = grid_cap(8);
        if (pb < 1) pb = 1;
        hipLaunchKernelGGL(k_place_slots, dim3((unsigned)pb), dim3(256), 0, st, a.batch * T,
                           ws.k0, pl.rank, pl.off, ws.k1, ws.v1, walks, walk_length,
                           context_radius, static_cast<int32_t>(T), 1 + neg_samples);
        DW_LAUNCH_CHECK("dw_sgns_owner_out_catch_up/place_slots");
        return DW_OK;
    }
    // the listed rows (at most min(local_rows, B' * T)) replay their steps up to step - 1 (p_only:
    // only p is written back; the lazy gather replays m and v itself, cheaply, before the step)
    const int64_t n_max = std::min<int64_t>(local_rows, a.batch * T);
    return dw::adam_rows_launch(w_out_local, m_out, v_out, last_step, nullptr, local_rows, dim,
                                rows_buf,
                                n_rows, n_max, nullptr, hist, step - 1, p_only, st);
}

int dw_exact_register(const float *grad, int64_t *acc, int64_t n_elems, int32_t frac,
                      int32_t flags) {
    DW_REQUIRE(grad && acc && n_elems >= 0, "dw_exact_register: bad arguments");
    DW_REQUIRE(frac >= 0 && frac <= 62, "dw_exact_register: frac %d outside [0, 62]", frac);
    DW_REQUIRE((flags & ~(DW_EXACT_DEFER | DW_EXACT_ADAM)) == 0,
               "dw_exact_register: unknown flags %d", flags);
    std::lock_guard<std::mutex> lk(g_exact_mu);
    g_exact[grad] = ExactEntry{acc, n_elems, frac, flags};
    return DW_OK;
}

int dw_exact_unregister(const float *grad) {
    std::lock_guard<std::mutex> lk(g_exact_mu);
    g_exact.erase(grad);
    return DW_OK;
}

int32_t dw_exact_frac_bits(double scale) {
    // terms are |coef| <= scale times table entries: 2^32 of headroom above scale's magnitude
    // for the entries (|w| < 2^19 keeps a term under 2^51) and 2^31 of sum range left in int64
    const double a = fabs(scale);
    if (!(a > 0.0) || !std::isfinite(a)) return 40;
    int f = 32 + static_cast<int>(ceil(-log2(a)));
    return f < 16 ? 16 : (f > 62 ? 62 : f);
}

int dw_fixed_to_float(int64_t *acc, float *grad, int64_t n, int32_t frac, int32_t accumulate,
                      void *stream) {
    DW_REQUIRE(n >= 0 && frac >= 0 && frac <= 62, "dw_fixed_to_float: bad arguments");
    if (n == 0) return DW_OK;
    DW_REQUIRE(acc && grad, "dw_fixed_to_float: null pointer");
    int64_t blocks = (n + 255) / 256;
    if (blocks > grid_cap(8)) blocks = grid_cap(8);
    hipLaunchKernelGGL(k_fixed_dense, dim3((unsigned)blocks), dim3(256), 0, dw::as_stream(stream),
                       acc, grad, n, ldexp(1.0, -frac), accumulate);
    DW_LAUNCH_CHECK("dw_fixed_to_float");
    return DW_OK;
}

int dw_sgns_timing(int32_t enable) {
    g_timer.on = enable != 0;
    if (enable) g_timer.calls = 0;
    return DW_OK;
}

int dw_sgns_phase_ms(double *ms, int64_t *n_calls) {
    DW_REQUIRE(ms && n_calls, "dw_sgns_phase_ms: null pointer");
    ms[0] = ms[1] = ms[2] = 0.0;
    *n_calls = static_cast<int64_t>(g_timer.calls);
    if (g_timer.calls == 0) return DW_OK;
    hipError_t e = hipEventSynchronize(g_timer.ev[4 * g_timer.calls - 1]);
    for (size_t c = 0; c < g_timer.calls && e == hipSuccess; ++c) {
        for (int k = 0; k < 3 && e == hipSuccess; ++k) {
            float t = 0.f;
            e = hipEventElapsedTime(&t, g_timer.ev[4 * c + k], g_timer.ev[4 * c + k + 1]);
            ms[k] += t;
        }
    }
    if (e != hipSuccess) {
        dw::set_error("dw_sgns_phase_ms: %s", hipGetErrorString(e));
        return DW_E_HIP;
    }
    for (int k = 0; k < 3; ++k) ms[k] /= static_cast<double>(g_timer.calls);
    return DW_OK;
}

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

namespace {
int sgns_walks(int phase, const int32_t *walks, int64_t n_walks, int32_t walk_length,
               int32_t context_radius, int32_t neg_samples, int64_t vocab_size, int32_t dim,
               const float *w_in, const float *w_out, float *g_in, float *g_out,
               const int64_t *noise, uint64_t seed, uint64_t noise_offset, float grad_scale,
               double *loss_acc, int32_t *status, void *workspace, size_t workspace_bytes,
               void *stream) {
    DW_REQUIRE(phase >= 0 && phase <= 2, "dw_sgns_walks_phase: phase must be 0, 1 or 2");
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
    return launch_sgns<true>(a, workspace, workspace_bytes, phase, dw::as_stream(stream));
}
}  // namespace

int dw_sgns_walks(const int32_t *walks, int64_t n_walks, int32_t walk_length,
                  int32_t context_radius, int32_t neg_samples, int64_t vocab_size, int32_t dim,
                  const float *w_in, const float *w_out, float *g_in, float *g_out,
                  const int64_t *noise, uint64_t seed, uint64_t noise_offset, float grad_scale,
                  double *loss_acc, int32_t *status, void *workspace, size_t workspace_bytes,
                  void *stream) {
    return sgns_walks(0, walks, n_walks, walk_length, context_radius, neg_samples, vocab_size,
                      dim, w_in, w_out, g_in, g_out, noise, seed, noise_offset, grad_scale,
                      loss_acc, status, workspace, workspace_bytes, stream);
}

int dw_sgns_walks_phase2_adam(const int32_t *walks, int64_t n_walks, int32_t walk_length,
                              int32_t context_radius, int32_t neg_samples, int64_t vocab_size,
                              int32_t dim, const float *w_in, float *w_out, float *g_out,
                              float *m_out, float *v_out, uint8_t *row_flags,
                              float one_minus_beta1, float beta2, float one_minus_beta2,
                              float bias_correction2_sqrt, float neg_step_size, float eps,
                              float weight_decay, int32_t *status, void *workspace,
                              size_t workspace_bytes, void *stream) {
    DW_REQUIRE(workspace && m_out && v_out && row_flags && w_out && g_out,
               "dw_sgns_walks_phase2_adam: needs the records workspace and the Adam state");
    DW_REQUIRE(bias_correction2_sqrt > 0.f, "dw_sgns_walks_phase2_adam: bad Adam scalars");
    DW_REQUIRE(context_radius >= 1 && walk_length >= 2 * context_radius + 1 && n_walks >= 0 &&
                   dim >= 1 && vocab_size >= 1 && neg_samples >= 0,
               "dw_sgns_walks_phase2_adam: bad sizes");
    DW_REQUIRE(walks && w_in && status, "dw_sgns_walks_phase2_adam: null pointer");
    SgnsArgs a = base_args(vocab_size, dim, neg_samples, w_in, w_out, nullptr, g_out, nullptr,
                           0, 0, 1.f, nullptr, status);
    a.walks = walks;
    a.L = walk_length;
    a.R = context_radius;
    a.batch = n_walks * (walk_length - 2 * context_radius);
    a.C = 2 * context_radius;
    OutAdam oa{w_out, m_out, v_out, row_flags,
               dw::AdamScalars{one_minus_beta1, beta2, one_minus_beta2, bias_correction2_sqrt,
                               neg_step_size, eps, weight_decay,
                               bias_correction2_sqrt > 0.f ? 1.0f / bias_correction2_sqrt : 0.f}};
    oa.dyn = dw::bound_step_scalars();
    return launch_sgns<true>(a, workspace, workspace_bytes, 2, dw::as_stream(stream), &oa);
}

int dw_sgns_walks_phase2_piece(int32_t piece, int32_t n_pieces, int64_t piece_rows,
                               const int32_t *walks, int64_t n_walks, int32_t walk_length,
                               int32_t context_radius, int32_t neg_samples, int64_t vocab_size,
                               int32_t dim, const float *w_in, float *g_out, int32_t *status,
                               void *workspace, size_t workspace_bytes, void *stream) {
    DW_REQUIRE(context_radius >= 1 && walk_length >= 2 * context_radius + 1 && n_walks >= 0 &&
                   dim >= 1 && vocab_size >= 1 && neg_samples >= 0,
               "dw_sgns_walks_phase2_piece: bad sizes");
    DW_REQUIRE(walks && w_in && g_out && status, "dw_sgns_walks_phase2_piece: null pointer");
    SgnsArgs a = base_args(vocab_size, dim, neg_samples, w_in, nullptr, nullptr, g_out, nullptr,
                           0, 0, 1.f, nullptr, status);
    a.walks = walks;
    a.L = walk_length;
    a.R = context_radius;
    a.batch = n_walks * (walk_length - 2 * context_radius);
    a.C = 2 * context_radius;
    return launch_pieces(a, workspace, workspace_bytes, piece, n_pieces, piece_rows,
                         dw::as_stream(stream));
}

int dw_sgns_walks_phase(int32_t phase, const int32_t *walks, int64_t n_walks,
                        int32_t walk_length, int32_t context_radius, int32_t neg_samples,
                        int64_t vocab_size, int32_t dim, const float *w_in, const float *w_out,
                        float *g_in, float *g_out, const int64_t *noise, uint64_t seed,
                        uint64_t noise_offset, float grad_scale, double *loss_acc,
                        int32_t *status, void *workspace, size_t workspace_bytes,
                        void *stream) {
    return sgns_walks(phase, walks, n_walks, walk_length, context_radius, neg_samples,
                      vocab_size, dim, w_in, w_out, g_in, g_out, noise, seed, noise_offset,
                      grad_scale, loss_acc, status, workspace, workspace_bytes, stream);
}

int dw_sgns_owner_workspace_bytes(int64_t n_centres, int32_t n_ctx, int32_t neg_samples,
                                  int64_t vocab_size, int64_t local_rows, size_t *bytes) {
    DW_REQUIRE(bytes, "dw_sgns_owner_workspace_bytes: bytes is null");
    DW_REQUIRE(n_centres >= 0 && n_ctx >= 1 && neg_samples >= 0 && local_rows >= 1 &&
                   vocab_size >= 1,
               "dw_sgns_owner_workspace_bytes: bad sizes");
    const OwnerLayout lay = owner_layout(n_centres, (int64_t)n_ctx * (1 + neg_samples));
    DW_REQUIRE(lay.total < 0x7FFFFFFF, "dw_sgns_owner_workspace_bytes: too many records");
    Workspace ws;
    OccSpace occ;
    PlaceSpace pl;
    char dummy;
    int rc = plan_workspace(lay.total > 0 ? lay.total : 1, local_rows, &dummy, &ws, nullptr);
    if (rc != DW_OK) return rc;
    rc = plan_place(n_centres * (int64_t)n_ctx * (1 + neg_samples), local_rows, &dummy, &pl,
                    nullptr);
    if (rc != DW_OK) return rc;
    rc = plan_occ(n_centres > 0 ? n_centres : 1, vocab_size, &dummy, &occ, nullptr);
    if (rc != DW_OK) return rc;
    *bytes = ws.total + pl.total + occ.total;
    return DW_OK;
}

int dw_sgns_owner_prepare(const int32_t *walks, int64_t n_walks, int32_t walk_length,
                          int32_t context_radius, int32_t neg_samples, int64_t vocab_size,
                          int64_t local_rows, uint32_t *touched, int64_t *n_touched,
                          void *workspace, size_t workspace_bytes, void *stream) {
    DW_REQUIRE(context_radius >= 1 && walk_length >= 2 * context_radius + 1 && n_walks >= 0 &&
                   vocab_size >= 1 && local_rows >= 1 && neg_samples >= 0,
               "dw_sgns_owner_prepare: bad sizes");
    DW_REQUIRE((walks || n_walks == 0) && (!touched || n_touched),
               "dw_sgns_owner_prepare: null pointer");
    SgnsArgs a = base_args(vocab_size, 64, neg_samples, nullptr, nullptr, nullptr, nullptr,
                           nullptr, 0, 0, 1.f, nullptr, nullptr);
    a.walks = walks;
    a.L = walk_length;
    a.R = context_radius;
    a.batch = n_walks * (walk_length - 2 * context_radius);
    a.C = 2 * context_radius;
    return launch_owner_prepare(a, local_rows, touched, n_touched, workspace, workspace_bytes,
                                dw::as_stream(stream));
}

int dw_sgns_owner_touch_claim(const int32_t *walks, int64_t n_walks, int32_t walk_length,
                              int32_t context_radius, int64_t vocab_size, int32_t *claim,
                              int32_t step, uint32_t *touched, int64_t *n_touched,
                              uint32_t *fresh, int64_t *n_fresh, int32_t flags, void *stream) {
    DW_REQUIRE(context_radius >= 1 && walk_length >= 2 * context_radius + 1 && n_walks >= 0 &&
                   vocab_size >= 1 && step >= 1,
               "dw_sgns_owner_touch_claim: bad sizes");
    DW_REQUIRE(claim && touched && n_touched && (walks || n_walks == 0) && (!fresh || n_fresh),
               "dw_sgns_owner_touch_claim: null pointer");
    const hipStream_t st = dw::as_stream(stream);
    const dw_step_scalars *dyn = nullptr;
    int32_t delta = 0;
    const int rc = dw::bound_step_rel(step, &dyn, &delta, "dw_sgns_owner_touch_claim");
    if (rc != DW_OK) return rc;
    DW_REQUIRE((flags & ~1) == 0, "dw_sgns_owner_touch_claim: flags must be 0 or 1");
    // flags & 1: the caller zeroed the counters (owner_lazy_steps: one ring of counters per
    // call, cleared by one memset at its head — no memset node per captured step)
    if (!(flags & 1) &&
        (hipMemsetAsync(n_touched, 0, sizeof(int64_t), st) != hipSuccess ||
         (fresh && hipMemsetAsync(n_fresh, 0, sizeof(int64_t), st) != hipSuccess))) {
        dw::set_error("dw_sgns_owner_touch_claim: counter reset failed");
        return DW_E_HIP;
    }
    const int64_t n_centres = n_walks * (walk_length - 2 * context_radius);
    if (n_centres == 0) return DW_OK;
    int64_t blocks = (n_centres + 255) / 256;
    if (blocks > grid_cap(8)) blocks = grid_cap(8);
    hipLaunchKernelGGL(k_touch_claim, dim3((unsigned)blocks), dim3(256), 0, st, walks, n_centres,
                       walk_length, context_radius, vocab_size, claim, step, dyn, delta, touched,
                       reinterpret_cast<unsigned long long *>(n_touched), fresh,
                       reinterpret_cast<unsigned long long *>(n_fresh));
    DW_LAUNCH_CHECK("dw_sgns_owner_touch_claim");
    return DW_OK;
}

int dw_sgns_owner_pass1(const int32_t *walks, int64_t n_walks, int32_t walk_length,
                        int32_t context_radius, int32_t neg_samples, int64_t vocab_size,
                        int32_t dim, int32_t owner, int32_t n_owners, int64_t local_rows,
                        int32_t order_ready, const float *w_in, const float *w_out_local,
                        float *g_in,
                        const int64_t *noise, uint64_t seed, uint64_t noise_offset,
                        float grad_scale, double *loss_acc, int32_t *status, void *workspace,
                        size_t workspace_bytes, void *stream) {
    DW_REQUIRE(context_radius >= 1 && walk_length >= 2 * context_radius + 1 && n_walks >= 0 &&
                   dim >= 1 && vocab_size >= 1 && neg_samples >= 0,
               "dw_sgns_owner_pass1: bad sizes");
    DW_REQUIRE((walks || n_walks == 0) && w_in && w_out_local && g_in && status,
               "dw_sgns_owner_pass1: null pointer");
    SgnsArgs a = base_args(vocab_size, dim, neg_samples, w_in, w_out_local, g_in, nullptr, noise,
                           seed, noise_offset, grad_scale, loss_acc, status);
    a.walks = walks;
    a.L = walk_length;
    a.R = context_radius;
    a.batch = n_walks * (walk_length - 2 * context_radius);
    a.C = 2 * context_radius;
    a.owner = owner;
    a.n_owners = n_owners;
    a.own_shift = -1;
    for (int sh = 0; sh < 31; ++sh)
        if ((1 << sh) == n_owners) a.own_shift = sh;
    return launch_owner_pass1(a, local_rows, order_ready, workspace, workspace_bytes,
                              dw::as_stream(stream));
}

int dw_sgns_owner_pass2(int64_t n_walks, int32_t walk_length, int32_t context_radius,
                        int32_t neg_samples, int64_t local_rows, int32_t dim, const float *w_in,
                        float *w_out_local, float *g_out_local, float *m_out, float *v_out,
                        uint8_t *row_flags, float one_minus_beta1, float beta2,
                        float one_minus_beta2, float bias_correction2_sqrt, float neg_step_size,
                        float eps, float weight_decay, int32_t *status, void *workspace,
                        size_t workspace_bytes, int64_t *n_records, void *stream) {
    DW_REQUIRE(context_radius >= 1 && walk_length >= 2 * context_radius + 1 && n_walks >= 0 &&
                   dim >= 1 && local_rows >= 1 && neg_samples >= 0,
               "dw_sgns_owner_pass2: bad sizes");
    DW_REQUIRE(w_in && g_out_local && status, "dw_sgns_owner_pass2: null pointer");
    const bool adam = m_out != nullptr;
    DW_REQUIRE(!adam || (v_out && row_flags && w_out_local && bias_correction2_sqrt > 0.f),
               "dw_sgns_owner_pass2: the fused Adam needs w_out_local, m, v, flags, scalars");
    OutAdam oa{w_out_local, m_out, v_out, row_flags,
               dw::AdamScalars{one_minus_beta1, beta2, one_minus_beta2, bias_correction2_sqrt,
                               neg_step_size, eps, weight_decay,
                               bias_correction2_sqrt > 0.f ? 1.0f / bias_correction2_sqrt : 0.f}};
    oa.dyn = dw::bound_step_scalars();
    const int64_t T = 2 * (int64_t)context_radius * (1 + neg_samples);
    return launch_owner_pass2(n_walks * (walk_length - 2 * context_radius), T, local_rows, dim,
                              w_in, g_out_local, adam ? &oa : nullptr, workspace,
                              workspace_bytes, n_records, dw::as_stream(stream));
}

int dw_sgns_owner_pass2_lazy(int64_t n_walks, int32_t walk_length, int32_t context_radius,
                             int32_t neg_samples, int64_t local_rows, int32_t dim,
                             const float *w_in, float *w_out_local, float *g_out_local,
                             float *m_out, float *v_out, int32_t *last_step, const float *hist,
                             int32_t step, int32_t flags, uint32_t *counts, int32_t *status,
                             void *workspace, size_t workspace_bytes, int64_t *n_records,
                             void *stream) {
    DW_REQUIRE(context_radius >= 1 && walk_length >= 2 * context_radius + 1 && n_walks >= 0 &&
                   dim >= 1 && local_rows >= 1 && neg_samples >= 0 && step >= 1,
               "dw_sgns_owner_pass2_lazy: bad sizes");
    DW_REQUIRE(w_in && w_out_local && g_out_local && m_out && v_out && last_step && hist &&
                   status,
               "dw_sgns_owner_pass2_lazy: null pointer");
    DW_REQUIRE((flags & ~7) == 0, "dw_sgns_owner_pass2_lazy: flags must be a set of 1 | 2 | 4");
    DW_REQUIRE(!(flags & 1) || counts, "dw_sgns_owner_pass2_lazy: placed records need counts");
    OutAdam oa{w_out_local, m_out, v_out, nullptr, dw::AdamScalars{}, last_step, hist, step};
    oa.p_current = (flags & 2) != 0;
    oa.betas_const = (flags & 4) != 0;
    oa.counts = nullptr;   // (placed records: the catch-up's scan cleared the counts)
    (void)counts;
    const int rc = dw::bound_step_rel(step, &oa.dyn, &oa.step_delta, "dw_sgns_owner_pass2_lazy");
    if (rc != DW_OK) return rc;
    const int64_t T = 2 * (int64_t)context_radius * (1 + neg_samples);
    return launch_owner_pass2(n_walks * (walk_length - 2 * context_radius), T, local_rows, dim,
                              w_in, g_out_local, &oa, workspace, workspace_bytes, n_records,
                              dw::as_stream(stream), (flags & 1) != 0);
}

int dw_sgns_owner_out_rows(const int32_t *walks, int64_t n_walks, int32_t walk_length,
                           int32_t context_radius, int32_t neg_samples, int64_t vocab_size,
                           int32_t dim, int32_t owner, int32_t n_owners, int64_t local_rows,
                           const int64_t *noise, uint64_t seed, uint64_t noise_offset,
                           float grad_scale, const float *w_in, float *w_out_local,
                           float *g_out_local, float *m_out, float *v_out, int32_t *last_step,
                           uint32_t *counts, uint8_t *pending, const float *hist,
                           int32_t step, double *loss_acc, int32_t *status,
                           void *workspace, size_t workspace_bytes, void *stream) {
    DW_REQUIRE(context_radius >= 1 && walk_length >= 2 * context_radius + 1 && n_walks >= 0 &&
                   dim >= 1 && vocab_size >= 1 && neg_samples >= 0 && n_owners >= 1 &&
                   owner >= 0 && owner < n_owners && local_rows >= 1 && step >= 1,
               "dw_sgns_owner_out_rows: bad sizes");
    DW_REQUIRE(dim % 64 == 0 && dim <= 512, "dw_sgns_owner_out_rows: needs dim a multiple of 64 "
               "(<= 512)");
    DW_REQUIRE(2 * (int64_t)context_radius * (1 + neg_samples) <= G16_TMAX,
               "dw_sgns_owner_out_rows: 2R(1+K) must be <= %d", G16_TMAX);
    DW_REQUIRE(local_rows * n_owners >= vocab_size && vocab_size <= 0x7FFFFFFF,
               "dw_sgns_owner_out_rows: the owners' rows do not cover the vocabulary");
    if (n_walks == 0) return DW_OK;
    DW_REQUIRE(walks && w_in && w_out_local && g_out_local && m_out && v_out && last_step &&
                   counts && pending && hist && status,
               "dw_sgns_owner_out_rows: null pointer");
    const int64_t T = 2 * (int64_t)context_radius * (1 + neg_samples);
    const int64_t n_centres = n_walks * (walk_length - 2 * context_radius);
    hipStream_t st = dw::as_stream(stream);
    SgnsArgs a = base_args(vocab_size, dim, neg_samples, w_in, w_out_local, nullptr, g_out_local,
                           noise, seed, noise_offset, grad_scale, loss_acc, status);
    a.walks = walks;
    a.L = walk_length;
    a.R = context_radius;
    a.batch = n_centres;
    a.C = 2 * context_radius;
    a.owner = owner;
    a.n_owners = n_owners;
    int32_t fl = 0;
    dw::Fixed fx;
    int rc = exact_of(g_out_local, local_rows * dim, &fx, &fl, "dw_sgns_owner_out_rows");
    if (rc != DW_OK) return rc;
    Workspace ws;
    OwnerLayout lay;
    PlaceSpace pl;
    rc = owner_workspace(n_centres, T, local_rows, workspace, workspace_bytes, &ws, &lay, st,
                         "dw_sgns_owner_out_rows", vocab_size, nullptr, &pl);
    if (rc != DW_OK) return rc;
    OutAdam oa{w_out_local, m_out, v_out, nullptr, dw::AdamScalars{}, last_step, hist, step};
    (void)counts;   // (cleared by the placement scan)
    oa.pend = pending;    // the stepped rows are left pending (p at step - 1 for the centre pass)
    rc = dw::bound_step_rel(step, &oa.dyn, &oa.step_delta, "dw_sgns_owner_out_rows");
    if (rc != DW_OK) return rc;
    // a block range of 4 gch records (gch <= 64): about two blocks per resident slot
    // (OUT_ROWS_WAVES per SIMD, k_out_rows' bound), so that the hardware hands the second half
    // out as blocks finish — at C3's 64-walk batch (269K records) 88-record ranges, 0.302-0.308
    // ms per step against 0.320-0.321 with one range per slot; 48 / 64 / 88 / 176 / 128 records
    // measured 0.303-0.305 / 0.305-0.306 / 0.302-0.308 / 0.316 / 0.322, 32 0.310
    // (profiles/r05_out_rows_ab.txt) — and no fewer than 16 per wave (small batches: fewer
    // straddling rows)
    const int64_t bound = n_centres * T;
    const int64_t resident = grid_cap(4 * OUT_ROWS_WAVES);
    // (three or four ranges per slot with the next step's preparation beside the kernel: within
    // 0.3%, profiles/r06_pipe_order_ab.txt)
    int32_t gch = static_cast<int32_t>((bound + 2 * resident - 1) / (2 * resident));
    gch = gch < 16 ? 16 : gch > 64 ? 64 : gch;
    int64_t blocks = ((bound + gch - 1) / gch + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) blocks = 1;
    const dim3 g((unsigned)blocks), bl(WAVES_PER_BLOCK * WAVE);
    float *cs = reinterpret_cast<float *>(ws.v0);
#define DW_OUT_ROWS(F, X)                                                                       \
    hipLaunchKernelGGL((k_out_rows<F, X>), g, bl, 0, st, a, ws.k1, ws.v1, ws.bounds, gch, oa,    \
                       cs, fx, pl.off)
    switch ((dim / 64) * 2 + (fx.acc ? 1 : 0)) {
        case 2: DW_OUT_ROWS(1, false); break;
        case 3: DW_OUT_ROWS(1, true); break;
        case 4: DW_OUT_ROWS(2, false); break;
        case 5: DW_OUT_ROWS(2, true); break;
        case 8: DW_OUT_ROWS(4, false); break;
        case 9: DW_OUT_ROWS(4, true); break;
        case 16: DW_OUT_ROWS(8, false); break;
        case 17: DW_OUT_ROWS(8, true); break;
        default:
            dw::set_error("dw_sgns_owner_out_rows: d must be one of 64, 128, 256, 512 (got %d)", dim);
            return DW_E_UNSUPPORTED;
    }
#undef DW_OUT_ROWS
    DW_LAUNCH_CHECK("dw_sgns_owner_out_rows/rows");
    return DW_OK;   // (every row stepped whole by the range it starts in)
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
    return launch_sgns<false>(a, workspace, workspace_bytes, 0, dw::as_stream(stream));
}

int dw_sgns_pooled_pairs(const int64_t *inputs, int32_t n_in, const int64_t *targets,
                         int64_t batch, int32_t n_ctx, int32_t neg_samples, int64_t vocab_size,
                         int32_t dim, const float *w_in, const float *w_out, float *g_in,
                         float *g_out, const int64_t *noise, uint64_t seed,
                         uint64_t noise_offset, float grad_scale, double *loss_acc,
                         int32_t *status, void *stream) {
    DW_REQUIRE(n_in >= 1 && n_ctx >= 1 && neg_samples >= 0 && dim >= 1 && vocab_size >= 1 &&
                   batch >= 0,
               "dw_sgns_pooled_pairs: bad sizes");
    DW_REQUIRE(inputs && targets && w_in && w_out && g_in && g_out && status,
               "dw_sgns_pooled_pairs: null pointer");
    SgnsArgs a = base_args(vocab_size, dim, neg_samples, w_in, w_out, g_in, g_out, noise, seed,
                           noise_offset, grad_scale, loss_acc, status);
    a.inputs = inputs;
    a.n_in = n_in;
    a.targets = targets;
    a.batch = batch;
    a.C = n_ctx;
    return launch_sgns<false>(a, nullptr, 0, 0, dw::as_stream(stream));  // atomic mode
}

int dw_sgns_noise(int64_t batch, int32_t n_ctx, int32_t neg_samples, int64_t vocab_size,
                  uint64_t seed, uint64_t noise_offset, int64_t *noise, void *stream) {
    DW_REQUIRE(batch >= 0 && n_ctx >= 0 && neg_samples >= 0 && vocab_size >= 1,
               "dw_sgns_noise: bad sizes");
    const int64_t n = batch * n_ctx * neg_samples;
    if (n == 0) return DW_OK;
    DW_REQUIRE(noise, "dw_sgns_noise: null pointer");
    int64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_noise_fill, dim3((unsigned)blocks), dim3(256), 0,
                       dw::as_stream(stream), batch, n_ctx, neg_samples, vocab_size,
                       static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32),
                       noise_offset, noise);
    DW_LAUNCH_CHECK("dw_sgns_noise");
    return DW_OK;
}

int dw_embedding_renorm_workspace_bytes(int64_t n_ids, int64_t vocab_size, size_t *bytes) {
    DW_REQUIRE(bytes && n_ids >= 0 && vocab_size >= 1 && vocab_size < 0x7FFFFFFF,
               "dw_embedding_renorm_workspace_bytes: bad arguments");
    size_t tmp = 0;
    rocprim::double_buffer<uint32_t> kb(nullptr, nullptr);
    hipError_t e = rocprim::radix_sort_keys<RenormSortConfig>(
        nullptr, tmp, kb, static_cast<uint32_t>(n_ids > 0 ? n_ids : 1), 0,
        end_bit_for(vocab_size + 1), nullptr);
    if (e != hipSuccess) {
        dw::set_error("dw_embedding_renorm: sort size query failed: %s", hipGetErrorString(e));
        return DW_E_HIP;
    }
    *bytes = 2 * align256(static_cast<size_t>(n_ids) * 4) + align256(tmp);
    return DW_OK;
}

int dw_embedding_renorm(float *weight, int64_t vocab_size, int32_t dim, const int64_t *ids,
                        int64_t n_ids, double max_norm, void *workspace, size_t workspace_bytes,
                        int32_t *status, void *stream) {
    DW_REQUIRE(dim >= 1 && vocab_size >= 1 && vocab_size < 0x7FFFFFFF && n_ids >= 0,
               "dw_embedding_renorm: bad sizes");
    if (n_ids == 0) return DW_OK;
    DW_REQUIRE(weight && ids && workspace && status, "dw_embedding_renorm: null pointer");
    DW_REQUIRE(n_ids < 0x7FFFFFFF, "dw_embedding_renorm: too many ids");
    size_t need = 0;
    int rc = dw_embedding_renorm_workspace_bytes(n_ids, vocab_size, &need);
    if (rc != DW_OK) return rc;
    DW_REQUIRE(workspace_bytes >= need, "dw_embedding_renorm: workspace too small (%zu < %zu)",
               workspace_bytes, need);
    hipStream_t st = dw::as_stream(stream);
    char *p = static_cast<char *>(workspace);
    const size_t kbytes = align256(static_cast<size_t>(n_ids) * 4);
    uint32_t *k0 = reinterpret_cast<uint32_t *>(p), *k1 = reinterpret_cast<uint32_t *>(p + kbytes);
    hipLaunchKernelGGL(k_renorm_keys, dim3((unsigned)((n_ids + 255) / 256)), dim3(256), 0, st,
                       ids, n_ids, vocab_size, k0, status);
    DW_LAUNCH_CHECK("dw_embedding_renorm/keys");
    rocprim::double_buffer<uint32_t> kb(k0, k1);
    size_t tmp = need - 2 * kbytes;
    hipError_t e = rocprim::radix_sort_keys<RenormSortConfig>(
        p + 2 * kbytes, tmp, kb, static_cast<uint32_t>(n_ids), 0, end_bit_for(vocab_size + 1),
        st);
    if (e != hipSuccess) {
        dw::set_error("dw_embedding_renorm: sort failed: %s", hipGetErrorString(e));
        return DW_E_HIP;
    }
    int64_t blocks = (n_ids + 3) / 4;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_renorm_rows, dim3((unsigned)blocks), dim3(256), 0, st, kb.current(),
                       n_ids, vocab_size, weight, dim, max_norm);
    DW_LAUNCH_CHECK("dw_embedding_renorm/rows");
    return DW_OK;
}

int dw_pooled_logits(const int64_t *inputs, int32_t n_in, const int64_t *outputs,
                     int64_t batch, int32_t n_out, int64_t vocab_size, int32_t dim,
                     const float *w_in, const float *w_out, int32_t proba, float *logits,
                     int32_t *status, void *stream) {
    DW_REQUIRE(batch >= 0 && n_out >= 0 && n_in >= 1 && dim >= 1, "dw_pooled_logits: bad sizes");
    if (batch == 0 || n_out == 0) return DW_OK;
    DW_REQUIRE(inputs && outputs && w_in && w_out && logits && status,
               "dw_pooled_logits: null pointer");
    int64_t blocks = (batch + 3) / 4;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_logits, dim3((unsigned)blocks), dim3(256), 0, dw::as_stream(stream),
                       inputs, n_in, outputs, batch, n_out, vocab_size, dim, w_in, w_out, proba,
                       logits, status);
    DW_LAUNCH_CHECK("dw_pooled_logits");
    return DW_OK;
}

int dw_pooled_logits_backward(const int64_t *inputs, int32_t n_in, const int64_t *outputs,
                              int64_t batch, int32_t n_out, int64_t vocab_size, int32_t dim,
                              const float *w_in, const float *w_out, const float *dlogits,
                              float *g_in, float *g_out, int32_t *status, void *stream) {
    DW_REQUIRE(batch >= 0 && n_out >= 0 && n_in >= 1 && dim >= 1,
               "dw_pooled_logits_backward: bad sizes");
    if (batch == 0 || n_out == 0) return DW_OK;
    DW_REQUIRE(inputs && outputs && w_in && w_out && dlogits && g_in && g_out && status,
               "dw_pooled_logits_backward: null pointer");
    int64_t blocks = (batch + 3) / 4;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_logits_bwd, dim3((unsigned)blocks), dim3(256), 0, dw::as_stream(stream),
                       inputs, n_in, outputs, batch, n_out, vocab_size, dim, w_in, w_out, dlogits,
                       g_in, g_out, status);
    DW_LAUNCH_CHECK("dw_pooled_logits_backward");
    return DW_OK;
}

int dw_skipgram_logits(const int64_t *inputs, const int64_t *outputs, int64_t batch,
                       int32_t n_out, int64_t vocab_size, int32_t dim, const float *w_in,
                       const float *w_out, int32_t proba, float *logits, int32_t *status,
                       void *stream) {
    return dw_pooled_logits(inputs, 1, outputs, batch, n_out, vocab_size, dim, w_in, w_out, proba,
                            logits, status, stream);
}

int dw_skipgram_logits_backward(const int64_t *inputs, const int64_t *outputs, int64_t batch,
                                int32_t n_out, int64_t vocab_size, int32_t dim,
                                const float *w_in, const float *w_out, const float *dlogits,
                                float *g_in, float *g_out, int32_t *status, void *stream) {
    return dw_pooled_logits_backward(inputs, 1, outputs, batch, n_out, vocab_size, dim, w_in,
                                     w_out, dlogits, g_in, g_out, status, stream);
}

}  // extern "C"
