// Random-walk generation on gfx950 (hot path A).
//
// Reference: shallow_encoders/graph/random_walk_generator.py
//   DeepWalk.walk   61-72   first-order step: random.choices(neighbors, normalized weights)
//   Node2Vec.walk   94-119  second-order step with the reference's (p, q) rule:
//                           x == prev -> w *= 1/p ; prev in N(x) -> w *= 1/q ; else w
//
// Two families of kernels:
//   * replay: bit-exact with the reference given the uniforms random.random() returns. The
//     weights of one step are computed lane-parallel (one wave per walker, adjacency tests
//     against N(prev) staged sorted in LDS), then ONE lane reproduces CPython's left-to-right
//     fp64 sum / accumulate / bisect_right serially — a parallel scan would round differently.
//     This file is compiled with -ffp-contract=off so no mul+add pair fuses into an FMA.
//   * fast: Philox4x32-10 keyed by (seed, global walk id, step, proposal/round).
//     DeepWalk: one lane per walker. node2vec: 8 lanes per walker, 64 proposals per round
//     evaluated 8 at a time, exact rejection against alpha/alpha_max, lowest accepting
//     proposal wins (ballot); adjacency tests only where the uniform leaves the outcome open.
#include <stdlib.h>

#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include "dw_common.h"

namespace {

constexpr int WAVE = 64;
constexpr uint32_t ALWAYS = 0xFFFFFFFFu;

// ---- adjacency tests ------------------------------------------------------------------------
__device__ __forceinline__ bool contains_global(const int32_t *__restrict__ s, int64_t n,
                                                int32_t key) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int32_t v = s[mid];
        if (v < key)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo < n && s[lo] == key;
}

__device__ __forceinline__ bool contains_lds(const int32_t *s, int n, int32_t key) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s[mid] < key)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo < n && s[lo] == key;
}

// =============================================================================================
// Replay walker
// =============================================================================================
constexpr int REPLAY_WAVES = 2;      // waves per block
constexpr int REPLAY_CH = 2048;      // cached step weights per wave (float64): 16 KiB
constexpr int REPLAY_NCAP = 2048;    // staged N(prev) entries per wave (int32): 8 KiB
// with the exact picks (unweighted): the step-weight cache only serves the rare serial
// fallback, so it shrinks to 4 KiB (= the class masks of 256 rounds), and N(prev) is staged up
// to 1024 entries (longer lists: binary search in HBM): 8 KiB per wave instead of 24, three
// times the walkers per CU (measured at C3, 65,536 walks: 38.5 ms at 12 KiB, 31.0 at 8 KiB;
// 768 or 512 staged entries, or a 2-KiB mask cache, were slower)
#ifndef DW_REPLAY_CH_EXACT
#define DW_REPLAY_CH_EXACT 512
#endif
constexpr int REPLAY_CH_EXACT = DW_REPLAY_CH_EXACT;
#ifndef DW_REPLAY_NCAP_EXACT
#define DW_REPLAY_NCAP_EXACT 1024
#endif
constexpr int REPLAY_NCAP_EXACT = DW_REPLAY_NCAP_EXACT;
// with the per-edge class counts no class masks are kept (k_walk_replay COUNTS): the weight
// cache of the serial fallback shrinks to 64 doubles, 4.6 KiB of LDS per wave
#ifndef DW_REPLAY_CH_CN
#define DW_REPLAY_CH_CN 64
#endif
constexpr int REPLAY_CH_CN = DW_REPLAY_CH_CN;

struct ReplayCtx {
    const int64_t *row_ptr;
    const int32_t *col;
    const int32_t *col_sorted;
    const double *w;
    bool node2vec;
    double inv_p, inv_q;
};

// Weight of candidate e (global CSR index) after the node2vec modification
// (random_walk_generator.py:100-108). `nprev` is N(prev) sorted, in LDS or global memory.
__device__ __forceinline__ double step_weight(const ReplayCtx &c, int64_t e, int32_t prev,
                                              const int32_t *nprev_lds, int nprev_lds_n,
                                              const int32_t *nprev_g, int64_t nprev_g_n) {
    double w = c.w ? c.w[e] : 1.0;
    if (c.node2vec && prev >= 0) {
        const int32_t x = c.col[e];
        if (x == prev) {
            w = w * c.inv_p;
        } else {
            // prev in N(x)  <=>  x in N(prev) on an undirected graph
            const bool adj = nprev_lds ? contains_lds(nprev_lds, nprev_lds_n, x)
                                       : contains_global(nprev_g, nprev_g_n, x);
            if (adj) w = w * c.inv_q;
        }
    }
    return w;
}

// bisect_right(cum, x, 0, hi) over a non-decreasing array (CPython Lib/bisect.py).
__device__ __forceinline__ int64_t bisect_right_lds(const double *cum, double x, int64_t hi) {
    int64_t lo = 0;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (x < cum[mid])
            hi = mid;
        else
            lo = mid + 1;
    }
    return lo;
}

// ---- exact picks without the serial sum (unweighted graphs) ---------------------------------
// On an unweighted graph a step's weights take at most three values (1, 1/p, 1/q), so the exact
// real prefix W_i = a_i/p + b_i + c_i/q (a, b, c: integer counts of each class up to neighbour i)
// and total T are known without CPython's left-to-right sums. CPython's cum[i] (accumulate of
// fl(w / fl-sum(w))) and x = fl(U * cum[n-1]) differ from W_i / T and U by at most
// (4n + 3) * 1.02 * 2^-53 (n roundings in the sum, n in the accumulate, one per division and
// product; every partial sum is <= 1 + n 2^-53). The fp64 evaluation of D_i = W_i - U*T adds
// under 10 * 2^-53 * T. So where |D_i| > M = (4.5 n + 20) 2^-53 T at the two neighbours that
// bracket the crossing, sign(D_i) = sign(cum[i] - x) for every i (W is strictly increasing),
// and bisect_right(cum, x, 0, n-1) = #{i <= n-2 : D_i <= 0} exactly. Where the margin fails
// (probability ~1e-6 per step at a 45K-neighbour hub) the serial replay decides.
__device__ __forceinline__ double exact_margin(int64_t n, double T) {
    return (4.5 * static_cast<double>(n) + 20.0) * 0x1p-53 * T;
}

// All weights equal (DeepWalk unweighted, node2vec's first step): W_i = i + 1, T = n.
// Returns the pick, or -1 where the margin leaves it to the serial replay.
__device__ __forceinline__ int64_t uniform_pick_exact(double U, int64_t n) {
    const double T = static_cast<double>(n);
    const double f = U * T;
    const double M = exact_margin(n, T);
    double k = floor(f);  // #{i : i + 1 <= f}, i + 1 in [1, n-1]
    if (k > T - 1.0) k = T - 1.0;
    if (k >= 1.0 && fabs(k - f) <= M) return -1;                 // D_{k-1} = k - f
    if (k + 1.0 <= T - 1.0 && fabs(k + 1.0 - f) <= M) return -1;  // D_k = k + 1 - f
    return static_cast<int64_t>(k);
}

// The serial replay of one unweighted first-order step in one lane (the margin failed):
// sum = n, nw = 1/n, cum = accumulate(nw), bisect_right(cum, U * cum[n-1], 0, n-1).
__device__ int64_t uniform_pick_serial(double U, int64_t n) {
    const double nw = 1.0 / static_cast<double>(n);
    double total = nw;
    for (int64_t i = 1; i < n; ++i) total = total + nw;
    total = total + 0.0;
    const double x = U * total;
    double cum = nw;
    for (int64_t i = 0; i < n - 1; ++i) {
        if (i > 0) cum = cum + nw;
        if (x < cum) return i;
    }
    return n - 1;
}

// DeepWalk on an unweighted graph: one lane per walker, O(1) per step.
__global__ void __launch_bounds__(256)
    k_walk_replay_uniform(const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
                          int64_t n_rows, const int32_t *__restrict__ starts, int64_t n_walks,
                          int32_t L, const double *__restrict__ uniforms,
                          int32_t *__restrict__ out, int32_t *status, int serial_only) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t wk = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; wk < n_walks;
         wk += stride) {
        int32_t v = starts[wk];
        int32_t *o = out + wk * (int64_t)L;
        o[0] = v;
        const double *u = uniforms + wk * (int64_t)(L - 1);
        int32_t s = 1;
        for (; s < L; ++s) {
            if (v < 0 || (int64_t)v >= n_rows) {
                dw::status_or(status, DW_S_BAD_CSR);
                break;
            }
            const int64_t a = row_ptr[v];
            const int64_t n = row_ptr[v + 1] - a;
            if (n <= 0) {
                dw::status_or(status, DW_S_ISOLATED_NODE);
                break;
            }
            const double U = u[s - 1];
            int64_t pick = serial_only ? -1 : uniform_pick_exact(U, n);
            if (pick < 0) pick = uniform_pick_serial(U, n);
            v = col[a + pick];
            o[s] = v;
        }
        for (; s < L; ++s) o[s] = -1;
    }
}

// The same walks over the edge-inline CSR (dw_edges_inline_build: {x, deg(x), row_ptr[x]} per
// entry): the picked entry carries the next row, so a step is one dependent 16-B load. The
// uniforms arrive walk-major (the reference's stream order: walk w's L-1 draws together), so a
// lane reading its own walk's draw touches a separate line per lane and step; a block instead
// stages RU_T steps of its 256 walks in LDS with coalesced loads (16 lanes read one walk's
// 128-B slice) and each lane then reads its draws from there.
constexpr int RU_T = 16;  // staged steps per tile
__global__ void __launch_bounds__(256)
    k_walk_replay_uniform_inline(const int64_t *__restrict__ row_ptr,
                                 const int4 *__restrict__ edges, int64_t n_rows,
                                 const int32_t *__restrict__ starts, int64_t n_walks, int32_t L,
                                 const double *__restrict__ uniforms, int32_t *__restrict__ out,
                                 int32_t *status, int serial_only) {
    __shared__ double tile[256][RU_T + 1];  // +1: lanes of one wave read different banks
    const int tid = threadIdx.x;
    const int64_t n_chunks = (n_walks + 255) / 256;
    const int64_t UL = L - 1;  // draws per walk
    for (int64_t ch = blockIdx.x; ch < n_chunks; ch += gridDim.x) {
        const int64_t w0 = ch * 256;
        const int n_here = (n_walks - w0 < 256) ? static_cast<int>(n_walks - w0) : 256;
        const int64_t wk = w0 + tid;
        const bool live = tid < n_here;
        int32_t v0 = live ? starts[wk] : 0;
        int32_t *o = out + wk * (int64_t)L;
        bool ok = live && v0 >= 0 && (int64_t)v0 < n_rows;
        if (live && !ok) dw::status_or(status, DW_S_BAD_CSR);
        int64_t a = ok ? row_ptr[v0] : 0;
        int64_t n = ok ? row_ptr[v0 + 1] - a : 0;
        const bool pack = (L & 3) == 0;
        int32_t q0 = v0, q1 = -1, q2 = -1;  // the current 4-step group (pack)
        if (live && !pack) o[0] = v0;
        for (int64_t t0 = 0; t0 < UL; t0 += RU_T) {
            const int tn = (UL - t0 < RU_T) ? static_cast<int>(UL - t0) : RU_T;
            __syncthreads();  // the previous tile is consumed
#pragma unroll 4
            for (int it = 0; it < RU_T; ++it) {
                const int e = it * 256 + tid;
                const int wl = e / RU_T, sl = e % RU_T;
                if (wl < n_here && sl < tn) tile[wl][sl] = uniforms[(w0 + wl) * UL + t0 + sl];
            }
            __syncthreads();
            if (!live) continue;
            for (int j = 0; j < tn; ++j) {
                const int32_t st = static_cast<int32_t>(t0) + 1 + j;  // the step this draw makes
                int32_t node = -1;
                if (ok) {
                    if (n <= 0) {
                        dw::status_or(status, DW_S_ISOLATED_NODE);
                        ok = false;
                    } else {
                        const double U = tile[tid][j];
                        int64_t pick = serial_only ? -1 : uniform_pick_exact(U, n);
                        if (pick < 0) pick = uniform_pick_serial(U, n);
                        const int4 e = edges[a + pick];
                        a = static_cast<int64_t>(static_cast<uint32_t>(e.z)) |
                            (static_cast<int64_t>(e.w) << 32);
                        n = e.y;
                        node = e.x;
                    }
                }
                if (!pack) {
                    o[st] = node;
                } else {
                    switch (st & 3) {  // the walk leaves in 16-B stores of 4 steps
                        case 0: q0 = node; break;
                        case 1: q1 = node; break;
                        case 2: q2 = node; break;
                        default:
                            reinterpret_cast<int4 *>(o)[st >> 2] = int4{q0, q1, q2, node};
                    }
                }
            }
        }
    }
}

// node2vec, unweighted, one wave per walker: the class of every neighbour (x == prev, x in
// N(prev), other) in rounds of 64 as two ballots, the class counts give T, and the round and
// lane where W crosses U*T give the pick. Returns -1 (serial replay) where the margin fails.
// `masks`: this wave's LDS, one u64 per round (the common-neighbour ballot; x == prev happens at
// most once in a simple graph, so its position is kept instead), cap rounds; rounds past cap
// re-classify in the second pass.
__device__ int64_t node2vec_pick_exact(const ReplayCtx &c, int64_t a, int64_t n, int32_t prev,
                                       const int32_t *np_lds, int np_lds_n,
                                       const int32_t *np_g, int64_t np_g_n, double U,
                                       uint64_t *masks, int64_t cap, int lane,
                                       const uint32_t *np_bits = nullptr) {
    const int64_t rounds = (n + WAVE - 1) / WAVE;
    auto classify = [&](int64_t r, uint64_t &mp, uint64_t &mq) {
        const int64_t i = r * WAVE + lane;
        bool is_p = false, is_q = false;
        if (i < n) {
            const int32_t x = c.col[a + i];
            if (x == prev)
                is_p = true;
            else
                is_q = np_bits ? ((np_bits[x >> 5] >> (x & 31)) & 1u) != 0u
                       : np_lds ? contains_lds(np_lds, np_lds_n, x)
                                : contains_global(np_g, np_g_n, x);
        }
        mp = __ballot(is_p);
        mq = __ballot(is_q);
    };
    int64_t A = 0, C = 0;
    int64_t pos_p = -1;   // the position of prev in N(v) (bisected rounds: from the ballots)
    auto tally = [&](int64_t r, bool is_p, bool is_q) {
        const uint64_t mp = __ballot(is_p), mq = __ballot(is_q);
        if (r < rounds) {
            if (r < cap && lane == 0) masks[r] = mq;
            if (mp) pos_p = r * WAVE + (__ffsll((unsigned long long)mp) - 1);
            A += __popcll(mp);
            C += __popcll(mq);
        }
    };
    if (np_bits) {   // prev's neighbour bitmap (a hub): one 4-B load per test, no search
        // rounds per trip: their col and bitmap loads in flight together (a hub-to-hub step
        // classifies up to ~700 rounds: the walk's critical path)
        constexpr int RBB = 16;
        for (int64_t r0 = 0; r0 < rounds; r0 += RBB) {
            int32_t x[RBB];
            uint32_t w[RBB];
#pragma unroll
            for (int j = 0; j < RBB; ++j) {
                const int64_t i = (r0 + j) * WAVE + lane;
                x[j] = i < n ? c.col[a + i] : prev;
            }
#pragma unroll
            for (int j = 0; j < RBB; ++j) w[j] = x[j] != prev ? np_bits[x[j] >> 5] : 0u;
#pragma unroll
            for (int j = 0; j < RBB; ++j) {
                const int64_t r = r0 + j;
                const bool in_row = r * WAVE + lane < n;
                const bool is_p = in_row && x[j] == prev;
                tally(r, is_p, in_row && !is_p && ((w[j] >> (x[j] & 31)) & 1u) != 0u);
            }
        }
    } else {
    // first pass, 4 rounds per trip: the four membership searches are independent, so their
    // dependent load chains overlap (branchless lower_bound over the same sorted N(prev));
    // 32-bit index arithmetic when N(prev) is staged in LDS
#ifndef DW_N2V_RB
#define DW_N2V_RB 4
#endif
    constexpr int RB = DW_N2V_RB;
    if (np_lds) {
        const int nn = np_lds_n;
        for (int64_t r0 = 0; r0 < rounds; r0 += RB) {
            int32_t x[RB];
            int base[RB];
#pragma unroll
            for (int j = 0; j < RB; ++j) {
                const int64_t i = (r0 + j) * WAVE + lane;
                x[j] = i < n ? c.col[a + i] : prev;  // past the row: counted as neither class
                base[j] = 0;
            }
            int len = nn;
            while (len > 1) {
                const int half = len >> 1;
#pragma unroll
                for (int j = 0; j < RB; ++j)
                    base[j] = (np_lds[base[j] + half] < x[j]) ? base[j] + half : base[j];
                len -= half;
            }
#pragma unroll
            for (int j = 0; j < RB; ++j) {
                const int64_t r = r0 + j;
                const bool in_row = r * WAVE + lane < n;
                const bool is_p = in_row && x[j] == prev;
                int lb = base[j];
                if (nn > 0 && np_lds[lb] < x[j]) ++lb;
                tally(r, is_p, in_row && !is_p && lb < nn && np_lds[lb] == x[j]);
            }
        }
    } else {
    const int32_t *ns = np_g;
    const int64_t nn = np_g_n;
    for (int64_t r0 = 0; r0 < rounds; r0 += RB) {
        int32_t x[RB];
        int64_t base[RB];
#pragma unroll
        for (int j = 0; j < RB; ++j) {
            const int64_t i = (r0 + j) * WAVE + lane;
            x[j] = i < n ? c.col[a + i] : prev;  // past the row: counted as neither class
            base[j] = 0;
        }
        int64_t len = nn;
        while (len > 1) {
            const int64_t half = len >> 1;
#pragma unroll
            for (int j = 0; j < RB; ++j)
                base[j] = (ns[base[j] + half] < x[j]) ? base[j] + half : base[j];
            len -= half;
        }
#pragma unroll
        for (int j = 0; j < RB; ++j) {
            const int64_t r = r0 + j;
            const bool in_row = r * WAVE + lane < n;
            const bool is_p = in_row && x[j] == prev;
            int64_t lb = base[j];
            if (nn > 0 && ns[lb] < x[j]) ++lb;
            tally(r, is_p, in_row && !is_p && lb < nn && ns[lb] == x[j]);
        }
    }
    }
    }
    dw::wave_lds_sync();
    const double ip = c.inv_p, iq = c.inv_q;
    auto W = [&](int64_t na, int64_t nb, int64_t nc) {
        return static_cast<double>(na) * ip + static_cast<double>(nb) +
               static_cast<double>(nc) * iq;
    };
    const double T = W(A, n - A - C, C);
    const double UT = U * T;
    const double M = exact_margin(n, T);
    int64_t na = 0, nc = 0;  // counts before round r
    double d_prev = -UT;     // D of the neighbour before the round (W = 0 before neighbour 0)
    for (int64_t r = 0; r < rounds; ++r) {
        uint64_t mp, mq;
        if (r < cap) {
            mq = masks[r];
            mp = (pos_p >= r * WAVE && pos_p < (r + 1) * WAVE) ? (1ull << (pos_p - r * WAVE)) : 0ull;
        } else {
            classify(r, mp, mq);
        }
        const int64_t base = r * WAVE;
        const int64_t in_round = n - base < WAVE ? n - base : WAVE;
        {   // the round's last D from its counts (wave-uniform): no crossing in it -> next round
            const int64_t ea = na + __popcll(mp), ec = nc + __popcll(mq);
            const double d_end = W(ea, (base + in_round) - ea - ec, ec) - UT;
            if (!(d_end > 0.0)) {
                d_prev = d_end;
                na = ea;
                nc = ec;
                continue;
            }
        }
        const uint64_t le = (lane == WAVE - 1) ? ~0ull : ((2ull << lane) - 1);  // lanes <= lane
        const int64_t pa = na + __popcll(mp & le), pc = nc + __popcll(mq & le);
        const int64_t i = base + lane;
        const double d = W(pa, (i + 1) - pa - pc, pc) - UT;  // D_i (lanes past n: unused)
        const uint64_t over = __ballot(lane < in_round && d > 0.0);
        if (over) {
            const int first = __ffsll((unsigned long long)over) - 1;
            int64_t k = base + first;  // first i with D_i > 0
            const double d_k = __shfl(d, first);
            const double d_km1 = first > 0 ? __shfl(d, first - 1) : d_prev;
            if (k > n - 1) k = n - 1;
            if (k >= 1 && fabs(d_km1) <= M) return -1;
            if (k <= n - 2 && fabs(d_k) <= M) return -1;
            return k;
        }
        d_prev = __shfl(d, static_cast<int>(in_round - 1));
        na += __popcll(mp);
        nc += __popcll(mq);
    }
    return -1;  // no D_i > 0: rounding at the top end; the serial replay decides
}

// ---- node2vec replay over the adjacency hash: probe the shorter list --------------------------
// The exact picks need, at a step (t -> v), the class of every neighbour of v: t itself, a
// common neighbour (x in N(t)), or other. node2vec_pick_exact classifies all n = deg(v) of them
// against N(t) (staged sorted in LDS, or searched in HBM). When N(t) is much the shorter list
// (m = deg(t), m * b_factor < n), k_walk_replay maps N(t) into N(v) instead: m + 1 probes of v's
// adjacency hash, each hit read back as the key's position in v's neighbour order (adj_hpos);
// the positions P of the common neighbours and t's own position give every prefix count
// c_i = #{P <= i}, T = A/p + B + C/q from the counts, and a binary search over i of
// D_i = W(a_i, b_i, c_i) - U T (c_i summed over the wave) finds the crossing; the same margin
// rule decides, the serial replay where it cannot. A walk visits hubs in proportion to their
// degree (mean visited degree 1,425 at C3) while the mean of min(deg v, deg t) over its edges is
// 276: a hub reached from a small node costs m probes instead of n classifications. A probe is
// a random 64-B line where a staged search is a few LDS reads, hence the factor (a sweep on one
// MI355X: scripts/experiments/n2v_bfactor_sweep.sh).

struct AdjRow {       // a row's CSR range and adjacency-hash buckets
    int64_t a, n, h;
    uint32_t nb;
};

__device__ __forceinline__ AdjRow adj_row(const int64_t *__restrict__ row_ptr,
                                          const int64_t *__restrict__ adj_off, int32_t v) {
    const int64_t a = row_ptr[v], b = row_ptr[v + 1];
    const int64_t h = adj_off[v], hb = adj_off[v + 1];
    return AdjRow{a, b - a, h, static_cast<uint32_t>((hb - h) >> 4)};
}

// Slot of key x in a row's hash (relative to adj_hash), or -1; one lane, one key.
__device__ __forceinline__ int64_t lane_hash_find(const int32_t *__restrict__ tab,
                                                  const AdjRow &r, int32_t x, uint32_t &probes) {
    uint32_t b = dw::adj_bucket(x, r.nb);
    for (uint32_t k = 0; k < r.nb; ++k) {
        const int64_t s0 = r.h + (int64_t)b * 16;
        const int4 *q = reinterpret_cast<const int4 *>(tab + s0);
        const int4 e0 = q[0], e1 = q[1], e2 = q[2], e3 = q[3];
        ++probes;
        const int32_t sl[16] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w,
                                e2.x, e2.y, e2.z, e2.w, e3.x, e3.y, e3.z, e3.w};
        bool free_slot = false;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (sl[j] == x) return s0 + j;
            free_slot = free_slot || sl[j] < 0;
        }
        if (free_slot) return -1;
        if (++b == r.nb) b = 0;
    }
    return -1;
}

// x in N(row)? (hash, or a scan of a short row's list)
__device__ __forceinline__ bool lane_member(const int32_t *__restrict__ col,
                                            const int32_t *__restrict__ tab, const AdjRow &r,
                                            int32_t x, uint32_t &probes) {
    if (r.nb > 0) return lane_hash_find(tab, r, x, probes) >= 0;
    for (int64_t k = 0; k < r.n; ++k)
        if (col[r.a + k] == x) return true;
    return false;
}

// position of x in N(row) (neighbour order), or -1
__device__ __forceinline__ int64_t lane_position(const int32_t *__restrict__ col,
                                                 const int32_t *__restrict__ tab,
                                                 const int32_t *__restrict__ hpos, const AdjRow &r,
                                                 int32_t x, uint32_t &probes) {
    if (r.nb > 0) {
        const int64_t s = lane_hash_find(tab, r, x, probes);
        return s >= 0 ? static_cast<int64_t>(hpos[s]) : -1;
    }
    for (int64_t k = 0; k < r.n; ++k)
        if (col[r.a + k] == x) return k;
    return -1;
}

__device__ __forceinline__ double n2v_w(int64_t na, int64_t nb, int64_t nc, double ip, double iq) {
    return static_cast<double>(na) * ip + static_cast<double>(nb) + static_cast<double>(nc) * iq;
}

// positions of N(t)'s members in N(v) (m <= the per-wave buffer), then a binary search for
// the crossing.
__device__ int64_t n2v_pick_positions(const int32_t *__restrict__ col,
                                      const int32_t *__restrict__ tab,
                                      const int32_t *__restrict__ hpos, const AdjRow &rv,
                                      const AdjRow &rt, int32_t t, double U, double ip,
                                      double iq, int32_t *pos, int lane, uint32_t &probes,
                                      uint32_t &loads) {
    const int64_t n = rv.n, m = rt.n;
    int64_t C = 0;
    for (int64_t j0 = 0; j0 < m; j0 += WAVE) {
        const int64_t j = j0 + lane;
        int32_t ps = -1;
        if (j < m) {
            const int32_t y = col[rt.a + j];
            ++loads;
            // t in N(t) (a self-loop at t): x == t is the 1/p class (counted by pos_t below),
            // never a common neighbour (random_walk_generator.py:102-104 tests x == prev first)
            if (y != t) ps = static_cast<int32_t>(lane_position(col, tab, hpos, rv, y, probes));
            pos[j] = ps;
        }
        C += __popcll(__ballot(ps >= 0));
    }
    int64_t pos_t = -1;                          // t's own position in N(v)
    if (lane == 0) pos_t = lane_position(col, tab, hpos, rv, t, probes);
    pos_t = __shfl(pos_t, 0);
    dw::wave_lds_sync();
    const int64_t A = pos_t >= 0 ? 1 : 0;
    const double T = n2v_w(A, n - A - C, C, ip, iq);
    const double UT = U * T;
    const double M = exact_margin(n, T);
    auto D = [&](int64_t i) {                    // D_i = W_i - U T, exact counts
        int64_t c = 0;
        for (int64_t j = lane; j < m; j += WAVE) {
            const int32_t ps = pos[j];
            c += (ps >= 0 && ps <= i) ? 1 : 0;
        }
#pragma unroll
        for (int off = WAVE / 2; off > 0; off >>= 1) c += __shfl_xor(c, off, WAVE);
        const int64_t a = (pos_t >= 0 && pos_t <= i) ? 1 : 0;
        return n2v_w(a, (i + 1) - a - c, c, ip, iq) - UT;
    };
    int64_t lo = 0, hi = n - 1;                  // first i in [0, n-1] with D_i > 0
    if (!(D(n - 1) > 0.0)) return -1;            // rounding at the top end: serial replay
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (D(mid) > 0.0)
            hi = mid;
        else
            lo = mid + 1;
    }
    const int64_t k = lo;
    if (k >= 1 && fabs(D(k - 1)) <= M) return -1;
    if (k <= n - 2 && fabs(D(k)) <= M) return -1;
    return k;
}

// ---- node2vec picks with the step's class counts known (dw_edge_common_counts) ----------------
// At a step t -> v over edge e, A = #{x in N(v) : x == t} and C = #{x in N(v) : x != t, x in
// N(t)} are the edge's precomputed counts, so T = W(A, n - A - C, C) is known before any
// neighbour is classified. D_i = W_i - U T is increasing in i, so the crossing round is found by
// classifying rounds from the nearer end only — from the front while a round's last D is <= 0,
// or from the back (prefix counts = totals - suffix counts) while the D before a round is > 0 —
// and stops there: about a quarter of N(v) on average instead of all of it. The D values, T, M
// and the bracketing test are the same expressions on the same integers as node2vec_pick_exact,
// so the pick (or the serial fallback) is the same.

// The classes of RB rounds (r0, r0 + dir, ...; rounds outside [0, rounds) are empty): the
// membership searches of the RB rounds are interleaved so their dependent loads overlap.
template <int RB>
__device__ __forceinline__ void n2v_classify_trip(const int32_t *__restrict__ col, int64_t a,
                                                  int64_t n, int64_t rounds, int32_t prev,
                                                  const int32_t *np_lds, int np_lds_n,
                                                  const int32_t *np_g, int64_t np_g_n,
                                                  const uint32_t *np_bits, int64_t r0, int dir,
                                                  int lane, uint64_t (&mp)[RB],
                                                  uint64_t (&mq)[RB]) {
    int32_t x[RB];
    bool in_row[RB], memb[RB];
#pragma unroll
    for (int j = 0; j < RB; ++j) {
        const int64_t r = r0 + dir * j;
        const int64_t i = r * WAVE + lane;
        in_row[j] = r >= 0 && r < rounds && i < n;
        x[j] = in_row[j] ? col[a + i] : prev;   // outside the row: counted as neither class
    }
    if (np_bits) {
        uint32_t w[RB];
#pragma unroll
        for (int j = 0; j < RB; ++j) w[j] = x[j] != prev ? np_bits[x[j] >> 5] : 0u;
#pragma unroll
        for (int j = 0; j < RB; ++j) memb[j] = ((w[j] >> (x[j] & 31)) & 1u) != 0u;
    } else if (np_lds) {
        const int nn = np_lds_n;
        int base[RB];
#pragma unroll
        for (int j = 0; j < RB; ++j) base[j] = 0;
        int len = nn;
        while (len > 1) {
            const int half = len >> 1;
#pragma unroll
            for (int j = 0; j < RB; ++j)
                base[j] = (np_lds[base[j] + half] < x[j]) ? base[j] + half : base[j];
            len -= half;
        }
#pragma unroll
        for (int j = 0; j < RB; ++j) {
            int lb = base[j];
            if (nn > 0 && np_lds[lb] < x[j]) ++lb;
            memb[j] = lb < nn && np_lds[lb] == x[j];
        }
    } else {
        const int64_t nn = np_g_n;
        int64_t base[RB];
#pragma unroll
        for (int j = 0; j < RB; ++j) base[j] = 0;
        int64_t len = nn;
        while (len > 1) {
            const int64_t half = len >> 1;
#pragma unroll
            for (int j = 0; j < RB; ++j)
                base[j] = (np_g[base[j] + half] < x[j]) ? base[j] + half : base[j];
            len -= half;
        }
#pragma unroll
        for (int j = 0; j < RB; ++j) {
            int64_t lb = base[j];
            if (nn > 0 && np_g[lb] < x[j]) ++lb;
            memb[j] = lb < nn && np_g[lb] == x[j];
        }
    }
#pragma unroll
    for (int j = 0; j < RB; ++j) {
        const bool is_p = in_row[j] && x[j] == prev;
        mp[j] = __ballot(is_p);
        mq[j] = __ballot(in_row[j] && !is_p && memb[j]);
    }
}

#ifndef DW_N2V_CN_RB
#define DW_N2V_CN_RB 4
#endif
#ifndef DW_N2V_CN_RBB
#define DW_N2V_CN_RBB 8
#endif

// Returns the pick, or -1 (serial replay); `scanned` += the rounds classified.
template <int RB>
__device__ int64_t n2v_pick_counted_rb(const ReplayCtx &c, int64_t a, int64_t n, int32_t prev,
                                       const int32_t *np_lds, int np_lds_n, const int32_t *np_g,
                                       int64_t np_g_n, const uint32_t *np_bits, double U,
                                       int64_t A, int64_t C, int lane, uint32_t &scanned) {
    const int64_t rounds = (n + WAVE - 1) / WAVE;
    const double ip = c.inv_p, iq = c.inv_q;
    const double T = n2v_w(A, n - A - C, C, ip, iq);
    const double UT = U * T;
    const double M = exact_margin(n, T);
    if (!(T - UT > 0.0)) return -1;   // D_{n-1} <= 0: rounding at the top end
    // the crossing is in round r: D before it <= 0 < D at its end
    auto resolve = [&](int64_t r, uint64_t mp, uint64_t mq, int64_t na, int64_t nc,
                       double d_before) -> int64_t {
        const int64_t base = r * WAVE;
        const int64_t in_round = n - base < WAVE ? n - base : WAVE;
        const uint64_t le = (lane == WAVE - 1) ? ~0ull : ((2ull << lane) - 1);  // lanes <= lane
        const int64_t pa = na + __popcll(mp & le), pc = nc + __popcll(mq & le);
        const int64_t i = base + lane;
        const double d = n2v_w(pa, (i + 1) - pa - pc, pc, ip, iq) - UT;
        const uint64_t over = __ballot(lane < in_round && d > 0.0);
        if (!over) return -1;
        const int first = __ffsll((unsigned long long)over) - 1;
        const int64_t k = base + first;   // first i with D_i > 0
        const double d_k = __shfl(d, first);
        const double d_km1 = first > 0 ? __shfl(d, first - 1) : d_before;
        if (k >= 1 && fabs(d_km1) <= M) return -1;
        if (k <= n - 2 && fabs(d_k) <= M) return -1;
        return k;
    };
    uint64_t mp[RB], mq[RB];
    if (U < 0.5) {   // from the front
        int64_t na = 0, nc = 0;
        double d_prev = -UT;
        for (int64_t r0 = 0; r0 < rounds; r0 += RB) {
            n2v_classify_trip<RB>(c.col, a, n, rounds, prev, np_lds, np_lds_n, np_g, np_g_n,
                                  np_bits, r0, 1, lane, mp, mq);
            scanned += RB;
#pragma unroll
            for (int j = 0; j < RB; ++j) {
                const int64_t r = r0 + j;
                if (r >= rounds) break;
                const int64_t end = (r + 1) * WAVE < n ? (r + 1) * WAVE : n;
                const int64_t ea = na + __popcll(mp[j]), ec = nc + __popcll(mq[j]);
                const double d_end = n2v_w(ea, end - ea - ec, ec, ip, iq) - UT;
                if (d_end > 0.0) return resolve(r, mp[j], mq[j], na, nc, d_prev);
                d_prev = d_end;
                na = ea;
                nc = ec;
            }
        }
        return -1;
    }
    int64_t sa = 0, sc = 0;   // from the back: the counts in the rounds after r
    for (int64_t r0 = rounds - 1; r0 >= 0; r0 -= RB) {
        n2v_classify_trip<RB>(c.col, a, n, rounds, prev, np_lds, np_lds_n, np_g, np_g_n, np_bits,
                              r0, -1, lane, mp, mq);
        scanned += RB;
#pragma unroll
        for (int j = 0; j < RB; ++j) {
            const int64_t r = r0 - j;
            if (r < 0) break;
            const int64_t ba = A - sa - __popcll(mp[j]), bc = C - sc - __popcll(mq[j]);
            const int64_t base = r * WAVE;
            const double d_before = n2v_w(ba, base - ba - bc, bc, ip, iq) - UT;
            if (!(d_before > 0.0)) return resolve(r, mp[j], mq[j], ba, bc, d_before);
            sa += __popcll(mp[j]);
            sc += __popcll(mq[j]);
        }
    }
    return -1;
}

__device__ __forceinline__ int64_t n2v_pick_counted(const ReplayCtx &c, int64_t a, int64_t n,
                                                    int32_t prev, const int32_t *np_lds,
                                                    int np_lds_n, const int32_t *np_g,
                                                    int64_t np_g_n, const uint32_t *np_bits,
                                                    double U, int64_t A, int64_t C, int lane,
                                                    uint32_t &scanned) {
    // a bitmap test is one independent load: more rounds per trip; a search is a chain
    return np_bits ? n2v_pick_counted_rb<DW_N2V_CN_RBB>(c, a, n, prev, np_lds, np_lds_n, np_g,
                                                        np_g_n, np_bits, U, A, C, lane, scanned)
                   : n2v_pick_counted_rb<DW_N2V_CN_RB>(c, a, n, prev, np_lds, np_lds_n, np_g,
                                                       np_g_n, np_bits, U, A, C, lane, scanned);
}

// cn[e] for every directed edge e = (t -> v = col[e]) of row t: bit 31 = [t in N(v)], bits 0-30
// = #{x in N(v) : x != t, x in N(t)} — the classes a node2vec step t -> v counts (above). With
// I = |N(t) ∩ N(v)|, counted over the shorter list against the other row (the same number from
// either side on a simple graph: no repeated neighbours, as networkx graphs and the deduplicated
// R-MAT lists; the positions path above assumes the same), C(t -> v) = I - [t in N(v) and t in
// N(t)] and C(v -> t) = I - [v in N(v)]: one count serves both directions of an undirected edge,
// so it is computed once, from the side t < v, and the reverse entry found through v's position
// table (adj_hpos). Membership in a row with a neighbour bitmap (dw_hub_bitmaps) is one 4-B test
// inside that row's V-bit map (L2-resident for the many edges that probe one hub), else a probe
// of the row's adjacency hash or a scan of its short list. One lane per edge when the shorter
// list has <= 16 entries, else the wave over that edge. The build is bound by random lines: at
// C3, sum over edges of min(deg) = 5.5e9 tests, 79% of edges with both degrees > 16.
__device__ __forceinline__ int64_t row_of_edge(const int64_t *__restrict__ row_ptr,
                                               int64_t n_rows, int64_t e) {
    int64_t lo = 0, hi = n_rows;   // last row with row_ptr[row] <= e
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (row_ptr[mid] <= e)
            lo = mid;
        else
            hi = mid;
    }
    return lo;
}

// One edge's positions in the compact index (dw_n2v_edge_index_build): uint16 when the target
// row has at most N2V_U16_MAX_DEG neighbours (every position fits), else int32 — half the
// bytes for all but the hubs' lists (C5: 116 GB instead of 222 GB of positions). `wide` follows
// from deg(v), which the step's record carries.
constexpr int64_t N2V_U16_MAX_DEG = 65536;
struct PosList {
    const uint8_t *__restrict__ p;
    bool wide;
    __device__ __forceinline__ int64_t operator[](int64_t i) const {
        return wide ? static_cast<int64_t>(reinterpret_cast<const int32_t *>(p)[i])
                    : static_cast<int64_t>(reinterpret_cast<const uint16_t *>(p)[i]);
    }
};

struct EdgeIndex {   // the membership tests' index (dw_edge_common_counts)
    const int32_t *col;
    const int64_t *adj_off;
    const int32_t *adj_hash;
    const int32_t *adj_hpos;
    const int32_t *hub_idx;    // row -> its bitmap, -1 (or NULL: no bitmaps)
    const uint32_t *hub_bits;
    int64_t hub_words;
};

__device__ __forceinline__ const uint32_t *row_bits(const EdgeIndex &x, int32_t row) {
    if (!x.hub_idx) return nullptr;
    const int32_t h = x.hub_idx[row];
    return h >= 0 ? x.hub_bits + h * x.hub_words : nullptr;
}

// y in N(row)? (bitmap, hash or list scan)
__device__ __forceinline__ bool edge_member(const EdgeIndex &x, const uint32_t *bits,
                                            const AdjRow &r, int32_t y, uint32_t &probes) {
    if (bits) return ((bits[y >> 5] >> (y & 31)) & 1u) != 0u;
    return lane_member(x.col, x.adj_hash, r, y, probes);
}

__global__ void __launch_bounds__(256)
    k_edge_common(EdgeIndex x, const int64_t *__restrict__ row_ptr, int64_t n_rows,
                  int64_t n_edges, uint32_t *__restrict__ cn) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    const int64_t n_waves = (int64_t)gridDim.x * blockDim.x / WAVE;
    uint32_t probes = 0;
    for (int64_t e0 = wave * WAVE; e0 < n_edges; e0 += n_waves * WAVE) {
        const int64_t e = e0 + lane;
        const bool valid = e < n_edges;
        int32_t t = 0, v = 0;
        AdjRow rt{0, 0, 0, 0}, rv{0, 0, 0, 0};
        const uint32_t *bt = nullptr, *bv = nullptr;
        if (valid) {
            t = static_cast<int32_t>(row_of_edge(row_ptr, n_rows, e));
            v = x.col[e];
            rt = adj_row(row_ptr, x.adj_off, t);
            rv = adj_row(row_ptr, x.adj_off, v);
            bt = row_bits(x, t);
            bv = row_bits(x, v);
        }
        // A = [t in N(v)]; an undirected edge's pair is counted from its t < v side
        const bool A = valid && edge_member(x, bv, rv, t, probes);
        const bool mine = valid && (t <= v || !A);
        int64_t rev = -1;   // the entry of v -> t, written here too
        if (mine && A && t < v) {
            const int64_t pos = lane_position(x.col, x.adj_hash, x.adj_hpos, rv, t, probes);
            rev = pos >= 0 ? rv.a + pos : -1;
        }
        const bool self_t = mine && A && edge_member(x, bt, rt, t, probes);
        const bool self_v = rev >= 0 && edge_member(x, bv, rv, v, probes);
        const bool t_short = rt.n <= rv.n;
        const AdjRow rs = t_short ? rt : rv, rl = t_short ? rv : rt;
        const uint32_t *bl = t_short ? bv : bt;
        uint32_t I = 0;
        const bool small = rs.n <= 16;
        if (mine && small)
            for (int64_t k = 0; k < rs.n; ++k)
                if (edge_member(x, bl, rl, x.col[rs.a + k], probes)) ++I;
        uint64_t heavy = __ballot(mine && !small);
        while (heavy) {   // one edge at a time, the wave over its shorter list
            const int src = __ffsll((unsigned long long)heavy) - 1;
            heavy &= heavy - 1;
            const int64_t sa_ = __shfl(rs.a, src), sn = __shfl(rs.n, src);
            const AdjRow l{__shfl(rl.a, src), __shfl(rl.n, src), __shfl(rl.h, src),
                           static_cast<uint32_t>(__shfl(static_cast<int32_t>(rl.nb), src))};
            const uint32_t *b = reinterpret_cast<const uint32_t *>(
                __shfl(reinterpret_cast<unsigned long long>(bl), src));
            uint32_t cnt = 0;
            for (int64_t k = lane; k < sn; k += WAVE)
                if (edge_member(x, b, l, x.col[sa_ + k], probes)) ++cnt;
#pragma unroll
            for (int off = WAVE / 2; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, WAVE);
            if (lane == src) I = cnt;
        }
        if (mine) cn[e] = (A ? 0x80000000u : 0u) | ((I - (self_t ? 1u : 0u)) & 0x7FFFFFFFu);
        if (rev >= 0) cn[rev] = 0x80000000u | ((I - (self_v ? 1u : 0u)) & 0x7FFFFFFFu);
    }
}

// ---- the per-edge position index (dw_n2v_edge_index_build) ----------------------------------
// A step t -> v over edge e needs, of N(v)'s classes, only WHERE the 1/p neighbour (t itself)
// and the C(e) 1/q neighbours sit: every other neighbour weighs 1. So per directed edge the
// index keeps t's position in N(v) (or -1) and the sorted positions in N(v) of the common
// neighbours; the pick is then a binary search over those C positions (log2 C dependent loads)
// and an ALU-only search inside the gap between two of them. Positions are found over the
// shorter list, as the counts were: N(t) shorter — each y in N(t) \ {t} probed into v's hash,
// read back through adj_hpos (unsorted; the segmented sort orders them); N(v) shorter — each
// of its entries tested against N(t) in order. One lane per edge when the shorter list has
// <= 16 entries, else the wave over that edge (ballot compaction keeps the list order). An
// edge whose positions do not add up to its counted C sets DW_S_BAD_CSR.
// (edges [e_begin, e_end) of a chunk: pos is the chunk's scratch, entry i of edge e at
// off[e] - base + i)
__global__ void __launch_bounds__(256)
    k_edge_cn_positions(EdgeIndex x, const int64_t *__restrict__ row_ptr, int64_t n_rows,
                        int64_t e_begin, int64_t e_end, const uint32_t *__restrict__ cn,
                        const int64_t *__restrict__ off, int64_t base, int32_t *__restrict__ pos,
                        int32_t *__restrict__ pos_t, int32_t *status) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    const int64_t n_waves = (int64_t)gridDim.x * blockDim.x / WAVE;
    const uint64_t lt = (1ull << lane) - 1;   // lanes below this one
    const int64_t n_edges = e_end;
    uint32_t probes = 0;
    for (int64_t e0 = e_begin + wave * WAVE; e0 < n_edges; e0 += n_waves * WAVE) {
        const int64_t e = e0 + lane;
        const bool valid = e < n_edges;
        int32_t t = 0;
        AdjRow rt{0, 0, 0, 0}, rv{0, 0, 0, 0};
        const uint32_t *bt = nullptr;
        uint32_t w = 0;
        int64_t o = 0;
        if (valid) {
            t = static_cast<int32_t>(row_of_edge(row_ptr, n_rows, e));
            const int32_t v = x.col[e];
            rt = adj_row(row_ptr, x.adj_off, t);
            rv = adj_row(row_ptr, x.adj_off, v);
            bt = row_bits(x, t);
            w = cn[e];
            o = off[e] - base;
            int32_t pt = -1;
            if (w >> 31) {
                const int64_t p = lane_position(x.col, x.adj_hash, x.adj_hpos, rv, t, probes);
                if (p < 0) dw::status_or(status, DW_S_BAD_CSR);
                pt = static_cast<int32_t>(p);
            }
            pos_t[e] = pt;
        }
        const int64_t C = w & 0x7FFFFFFFu;
        const bool t_short = rt.n <= rv.n;
        const bool small = (t_short ? rt.n : rv.n) <= 16;
        if (valid && C > 0 && small) {
            int64_t k = 0;
            if (t_short) {
                for (int64_t j = 0; j < rt.n; ++j) {
                    const int32_t y = x.col[rt.a + j];
                    if (y == t) continue;   // x == prev: the 1/p class, never a common neighbour
                    const int64_t p = lane_position(x.col, x.adj_hash, x.adj_hpos, rv, y, probes);
                    if (p >= 0) {
                        if (k < C) pos[o + k] = static_cast<int32_t>(p);
                        ++k;
                    }
                }
            } else {
                for (int64_t i = 0; i < rv.n; ++i) {
                    const int32_t y = x.col[rv.a + i];
                    if (y != t && edge_member(x, bt, rt, y, probes)) {
                        if (k < C) pos[o + k] = static_cast<int32_t>(i);
                        ++k;
                    }
                }
            }
            if (k != C) dw::status_or(status, DW_S_BAD_CSR);
        }
        uint64_t heavy = __ballot(valid && C > 0 && !small);
        while (heavy) {   // one edge at a time, the wave over its shorter list
            const int src = __ffsll((unsigned long long)heavy) - 1;
            heavy &= heavy - 1;
            const bool ts = __shfl(t_short ? 1 : 0, src) != 0;
            const int32_t tt = __shfl(t, src);
            const AdjRow l_t{__shfl(rt.a, src), __shfl(rt.n, src), __shfl(rt.h, src),
                             static_cast<uint32_t>(__shfl(static_cast<int32_t>(rt.nb), src))};
            const AdjRow l_v{__shfl(rv.a, src), __shfl(rv.n, src), __shfl(rv.h, src),
                             static_cast<uint32_t>(__shfl(static_cast<int32_t>(rv.nb), src))};
            const uint32_t *b = reinterpret_cast<const uint32_t *>(
                __shfl(reinterpret_cast<unsigned long long>(bt), src));
            const int64_t oo = __shfl(o, src), cc = __shfl(C, src);
            int64_t k = 0;
            const int64_t len = ts ? l_t.n : l_v.n;
            for (int64_t j0 = 0; j0 < len; j0 += WAVE) {
                const int64_t j = j0 + lane;
                int64_t p = -1;
                if (j < len) {
                    if (ts) {
                        const int32_t y = x.col[l_t.a + j];
                        if (y != tt)
                            p = lane_position(x.col, x.adj_hash, x.adj_hpos, l_v, y, probes);
                    } else {
                        const int32_t y = x.col[l_v.a + j];
                        if (y != tt && edge_member(x, b, l_t, y, probes)) p = j;
                    }
                }
                const uint64_t hit = __ballot(p >= 0);
                const int64_t slot = k + __popcll(hit & lt);
                if (p >= 0 && slot < cc) pos[oo + slot] = static_cast<int32_t>(p);
                k += __popcll(hit);
            }
            if (lane == src && k != cc) dw::status_or(status, DW_S_BAD_CSR);
        }
    }
}

// The sorted positions of a chunk's edges into the compact index: edge e's list at byte
// boff[e] as uint16 (deg(col[e]) <= N2V_U16_MAX_DEG) or int32; one lane per edge for short
// lists, the wave over a long one (coalesced stores).
__global__ void __launch_bounds__(256)
    k_n2v_pos_compact(const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
                      int64_t e_begin, int64_t e_end, const int64_t *__restrict__ off,
                      int64_t base, const int64_t *__restrict__ boff,
                      const int32_t *__restrict__ sorted, uint8_t *__restrict__ out) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    const int64_t n_waves = (int64_t)gridDim.x * blockDim.x / WAVE;
    for (int64_t e0 = e_begin + wave * WAVE; e0 < e_end; e0 += n_waves * WAVE) {
        const int64_t e = e0 + lane;
        int64_t a = 0, c = 0, b = 0;
        bool wide = false;
        if (e < e_end) {
            a = off[e] - base;
            c = off[e + 1] - off[e];
            b = boff[e];
            const int32_t v = col[e];
            wide = row_ptr[v + 1] - row_ptr[v] > N2V_U16_MAX_DEG;
            if (c <= 32) {
                for (int64_t i = 0; i < c; ++i) {
                    if (wide)
                        reinterpret_cast<int32_t *>(out + b)[i] = sorted[a + i];
                    else
                        reinterpret_cast<uint16_t *>(out + b)[i] =
                            static_cast<uint16_t>(sorted[a + i]);
                }
            }
        }
        uint64_t heavy = __ballot(e < e_end && c > 32);
        while (heavy) {
            const int src = __ffsll((unsigned long long)heavy) - 1;
            heavy &= heavy - 1;
            const int64_t ha = __shfl(a, src), hc = __shfl(c, src), hb = __shfl(b, src);
            const bool hw = __shfl(wide ? 1 : 0, src) != 0;
            for (int64_t i = lane; i < hc; i += WAVE) {
                if (hw)
                    reinterpret_cast<int32_t *>(out + hb)[i] = sorted[ha + i];
                else
                    reinterpret_cast<uint16_t *>(out + hb)[i] = static_cast<uint16_t>(sorted[ha + i]);
            }
        }
    }
}

// The walker's 32-B edge record: {x, deg(x), row_ptr[x] lo, hi} (the edge-inline CSR entry)
// then {byte offset of its positions lo, hi, counts word, t's position in N(x)} — one line per
// step.
__global__ void k_n2v_edge_records(const int64_t *__restrict__ row_ptr,
                                   const int32_t *__restrict__ col, const uint32_t *__restrict__ cn,
                                   const int64_t *__restrict__ off,
                                   const int32_t *__restrict__ pos_t, int64_t n_edges,
                                   int4 *__restrict__ rec) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n_edges; e += stride) {
        const int32_t v = col[e];
        const int64_t a = row_ptr[v];
        const int64_t o = off[e];
        rec[2 * e] = int4{v, static_cast<int32_t>(row_ptr[v + 1] - a),
                          static_cast<int32_t>(static_cast<uint32_t>(a)),
                          static_cast<int32_t>(a >> 32)};
        rec[2 * e + 1] = int4{static_cast<int32_t>(static_cast<uint32_t>(o)),
                              static_cast<int32_t>(o >> 32), static_cast<int32_t>(cn[e]),
                              pos_t[e]};
    }
}

struct CnCount64 {   // C(e) of a counts word, widened for the offsets' scan
    __host__ __device__ __forceinline__ int64_t operator()(uint32_t w) const {
        return static_cast<int64_t>(w & 0x7FFFFFFFu);
    }
};

struct CnBytes {     // edge e's bytes in the compact index: C(e) entries of 2 or 4 B, to 4 B
    const uint32_t *cn;
    const int64_t *row_ptr;
    const int32_t *col;
    __host__ __device__ __forceinline__ int64_t operator()(int64_t e) const {
        const int32_t v = col[e];
        const int64_t w = row_ptr[v + 1] - row_ptr[v] > N2V_U16_MAX_DEG ? 4 : 2;
        return ((static_cast<int64_t>(cn[e] & 0x7FFFFFFFu) * w) + 3) & ~int64_t(3);
    }
};

#define DW_WALK_HIP_OK(expr, what)                                                  \
    do {                                                                            \
        hipError_t e_ = (expr);                                                     \
        if (e_ != hipSuccess) {                                                     \
            ::dw::set_error("%s: %s", what, hipGetErrorString(e_));                 \
            return DW_E_HIP;                                                        \
        }                                                                           \
    } while (0)

// The adjacency index of the probe-the-shorter-list steps (dw_walk_replay_indexed; adj_off ==
// NULL: every step classifies N(v)) and the optional traffic counters (uint64[4] += {bytes,
// hash probes, list entries read, steps}).
struct N2VIndex {
    const int64_t *adj_off;
    const int32_t *adj_hash;
    const int32_t *adj_hpos;
    int32_t b_factor;
    unsigned long long *counters;
    const int32_t *hub_idx;    // row -> its neighbour bitmap (dw_hub_bitmaps), or -1
    const uint32_t *hub_bits;  // [n_hubs][hub_words]
    int64_t hub_words;
    const uint32_t *edge_cn;   // per-edge class counts (dw_edge_common_counts), or NULL
};

__device__ __forceinline__ uint32_t ceil_log2(int64_t x) {
    uint32_t k = 0;
    while ((int64_t(1) << k) < x) ++k;
    return k;
}

// COUNTS: the launch has the per-edge class counts (ix.edge_cn): every step after the first
// takes n2v_pick_counted, so the full classification (node2vec_pick_exact) and its class-mask
// cache are not compiled in; CH then only sizes the serial fallback's weight cache (hub rows
// past it recompute their weights in lane 0) and, with the N(prev) stage, the positions buffer.
template <int CH, int NCAP, bool COUNTS>
__device__ __forceinline__ void walk_replay_body(ReplayCtx c, int64_t n_rows,
                                                 const int32_t *__restrict__ starts,
                                                 int64_t n_walks, int32_t L,
                                                 const double *__restrict__ uniforms,
                                                 int32_t *__restrict__ out, int32_t *status,
                                                 int fast, N2VIndex ix) {
    // per wave: CH doubles (the serial replay's weights / the exact picks' ballots) followed by
    // the NCAP-entry N(prev) stage; the ballots take both halves when nothing is staged
    __shared__ uint64_t s_lds[REPLAY_WAVES][CH + NCAP / 2];
    __shared__ int64_t s_pick[REPLAY_WAVES];
    const int lane = threadIdx.x & (WAVE - 1);
    const int wv = threadIdx.x / WAVE;
    double *buf = reinterpret_cast<double *>(s_lds[wv]);
    int32_t *nprev_lds = reinterpret_cast<int32_t *>(s_lds[wv] + CH);
    const int64_t n_waves = (int64_t)gridDim.x * REPLAY_WAVES;
    const bool counted = ix.counters != nullptr;
    uint32_t probes = 0, loads = 0, steps = 0;   // counted launches only
    for (int64_t wk = (int64_t)blockIdx.x * REPLAY_WAVES + wv; wk < n_walks; wk += n_waves) {
        int32_t v = starts[wk], prev = -1;
        int64_t e_in = -1;   // the edge prev -> v (its class counts: ix.edge_cn)
        int32_t s = 1;
        int32_t *o = out + wk * (int64_t)L;
        if (lane == 0) o[0] = v;
        const double *u = uniforms + wk * (int64_t)(L - 1);
        for (; s < L; ++s) {
            if (v < 0 || (int64_t)v >= n_rows) {
                if (lane == 0) dw::status_or(status, DW_S_BAD_CSR);
                break;
            }
            const int64_t a = c.row_ptr[v];
            const int64_t n = c.row_ptr[v + 1] - a;
            if (n <= 0) {  // random.choices on an empty population -> IndexError
                if (lane == 0) dw::status_or(status, DW_S_ISOLATED_NODE);
                break;
            }
            const double uu = u[s - 1];
            int64_t pa = 0, pn = 0;
            if (c.node2vec && prev >= 0) {
                pa = c.row_ptr[prev];
                pn = c.row_ptr[prev + 1] - pa;
            }
            if (counted && lane == 0) ++steps;
            // N(prev) much the shorter list: its members' positions in N(v) (v's hash)
            // (positions: the wave's buffer and N(prev) stage, contiguous: 2 CH + NCAP entries)
            if (fast && ix.adj_off && c.node2vec && prev >= 0 && pn <= 2 * CH + NCAP &&
                pn * (int64_t)ix.b_factor < n) {
                const int64_t h = ix.adj_off[v];
                const AdjRow rv{a, n, h, static_cast<uint32_t>((ix.adj_off[v + 1] - h) >> 4)};
                const AdjRow rt{pa, pn, 0, 0};
                const int64_t fp = n2v_pick_positions(
                    c.col, ix.adj_hash, ix.adj_hpos, rv, rt, prev, uu, c.inv_p, c.inv_q,
                    reinterpret_cast<int32_t *>(buf), lane, probes, loads);
                dw::wave_lds_sync();
                if (fp >= 0) {
                    const int32_t child = c.col[a + fp];
                    if (lane == 0) o[s] = child;
                    prev = v;
                    v = child;
                    e_in = a + fp;
                    continue;
                }
            }
            // N(prev), sorted, for the adjacency test
            const int32_t *np_lds = nullptr;
            int np_lds_n = 0;
            const int32_t *np_g = nullptr;
            int64_t np_g_n = 0;
            const uint32_t *np_bits = nullptr;
            if (c.node2vec && prev >= 0 && ix.hub_idx) {
                const int32_t hb = ix.hub_idx[prev];
                if (hb >= 0) np_bits = ix.hub_bits + hb * ix.hub_words;
            }
            // the class counts of prev -> v known: only the rounds up to the crossing classified
            const bool known =
                (COUNTS || ix.edge_cn != nullptr) && fast && c.node2vec && prev >= 0 && e_in >= 0;
            if (c.node2vec && prev >= 0) {
                if (counted && lane == 0 && !known)   // N(v) read; N(prev) staged, bit-tested
                    loads += static_cast<uint32_t>(   // or searched
                        n + (np_bits ? n
                                     : pn <= NCAP ? pn
                                                  : n * static_cast<int64_t>(ceil_log2(pn + 1))));
                if (np_bits) {
                    np_g = c.col_sorted + pa;   // (the serial fallback's search)
                    np_g_n = pn;
                } else if (pn <= NCAP) {
                    for (int64_t e = lane; e < pn; e += WAVE) nprev_lds[e] = c.col_sorted[pa + e];
                    dw::wave_lds_sync();
                    np_lds = nprev_lds;
                    np_lds_n = static_cast<int>(pn);
                } else {
                    np_g = c.col_sorted + pa;
                    np_g_n = pn;
                }
            }
            if (fast) {  // unweighted: the exact pick without the serial sums (above)
                int64_t fp;
                if (known) {
                    const uint32_t w = ix.edge_cn[e_in];
                    uint32_t scanned = 0;
                    fp = n2v_pick_counted(c, a, n, prev, np_lds, np_lds_n, np_g, np_g_n, np_bits,
                                          uu, static_cast<int64_t>(w >> 31),
                                          static_cast<int64_t>(w & 0x7FFFFFFFu), lane, scanned);
                    if (counted && lane == 0) {   // the counts word; N(v) up to the crossing
                        const int64_t ne = (int64_t)scanned * WAVE < n ? (int64_t)scanned * WAVE : n;
                        loads += static_cast<uint32_t>(
                            1 + ne + (np_bits ? ne
                                              : pn <= NCAP ? pn
                                                           : ne * static_cast<int64_t>(
                                                                      ceil_log2(pn + 1))));
                    }
                } else if constexpr (COUNTS) {
                    fp = (!c.node2vec || prev < 0) ? uniform_pick_exact(uu, n) : -1;
                } else {
                    fp = (!c.node2vec || prev < 0)
                             ? uniform_pick_exact(uu, n)
                             : node2vec_pick_exact(c, a, n, prev, np_lds, np_lds_n, np_g, np_g_n,
                                                   uu, reinterpret_cast<uint64_t *>(buf),
                                                   np_lds ? CH : CH + NCAP / 2, lane, np_bits);
                }
                if (fp >= 0) {
                    const int32_t child = c.col[a + fp];
                    if (lane == 0) o[s] = child;
                    prev = v;
                    v = child;
                    e_in = a + fp;
                    dw::wave_lds_sync();  // N(prev) / masks are rewritten next step
                    continue;
                }
                dw::wave_lds_sync();
            }
            if (n <= CH) {
                for (int64_t i = lane; i < n; i += WAVE)
                    buf[i] = step_weight(c, a + i, prev, np_lds, np_lds_n, np_g, np_g_n);
                dw::wave_lds_sync();
                if (lane == 0) {
                    double sum = 0.0;  // sum(neighbor_weights), left to right
                    for (int64_t i = 0; i < n; ++i) sum = sum + buf[i];
                    if (sum == 0.0) {
                        dw::status_or(status, DW_S_ZERO_WEIGHT);
                        s_pick[wv] = -1;
                    } else {
                        double cum = 0.0;  // itertools.accumulate(nw / sum)
                        for (int64_t i = 0; i < n; ++i) {
                            const double nw = buf[i] / sum;
                            cum = (i == 0) ? nw : cum + nw;
                            buf[i] = cum;
                        }
                        const double total = buf[n - 1] + 0.0;
                        s_pick[wv] = bisect_right_lds(buf, uu * total, n - 1);
                    }
                }
            } else {  // hub row: lane 0 recomputes the weights on the fly (same arithmetic)
                if (lane == 0) {
                    double sum = 0.0;
                    for (int64_t i = 0; i < n; ++i)
                        sum = sum + step_weight(c, a + i, prev, np_lds, np_lds_n, np_g, np_g_n);
                    if (sum == 0.0) {
                        dw::status_or(status, DW_S_ZERO_WEIGHT);
                        s_pick[wv] = -1;
                    } else {
                        double total = 0.0;
                        for (int64_t i = 0; i < n; ++i) {
                            const double nw =
                                step_weight(c, a + i, prev, np_lds, np_lds_n, np_g, np_g_n) / sum;
                            total = (i == 0) ? nw : total + nw;
                        }
                        total = total + 0.0;
                        const double x = uu * total;
                        int64_t pick = n - 1;  // bisect_right(cum, x, 0, n-1)
                        double cum = 0.0;
                        for (int64_t i = 0; i < n - 1; ++i) {
                            const double nw =
                                step_weight(c, a + i, prev, np_lds, np_lds_n, np_g, np_g_n) / sum;
                            cum = (i == 0) ? nw : cum + nw;
                            if (x < cum) {
                                pick = i;
                                break;
                            }
                        }
                        s_pick[wv] = pick;
                    }
                }
            }
            dw::wave_lds_sync();
            const int64_t pick = s_pick[wv];
            dw::wave_lds_sync();
            if (pick < 0) break;
            const int32_t child = c.col[a + pick];
            if (lane == 0) o[s] = child;
            prev = v;
            v = child;
            e_in = a + pick;
        }
        if (lane == 0)
            for (; s < L; ++s) o[s] = -1;  // marks an aborted walk
    }
    if (counted) {   // per step: row_ptr pairs of v and prev (32 B), the uniform, the pick and
                     // the output (16); per probe a 64-B bucket; per list entry 4 B
        unsigned long long v4[3] = {(unsigned long long)probes, (unsigned long long)loads,
                                    (unsigned long long)steps};
        for (int k = 0; k < 3; ++k)
            for (int off = WAVE / 2; off > 0; off >>= 1) v4[k] += __shfl_xor(v4[k], off, WAVE);
        if (lane == 0) {
            atomicAdd(ix.counters + 0, v4[0] * 64ull + v4[1] * 4ull + v4[2] * 48ull);
            atomicAdd(ix.counters + 1, v4[0]);
            atomicAdd(ix.counters + 2, v4[1]);
            atomicAdd(ix.counters + 3, v4[2]);
        }
    }
}

template <int CH, int NCAP>
__global__ void __launch_bounds__(REPLAY_WAVES *WAVE)
    k_walk_replay(ReplayCtx c, int64_t n_rows, const int32_t *__restrict__ starts,
                  int64_t n_walks, int32_t L, const double *__restrict__ uniforms,
                  int32_t *__restrict__ out, int32_t *status, int fast, N2VIndex ix) {
    walk_replay_body<CH, NCAP, false>(c, n_rows, starts, n_walks, L, uniforms, out, status, fast,
                                      ix);
}

// The COUNTS form is latency-bound on each walker's dependent chain and its LDS (4.6 KiB per
// wave) allows 34 walkers per CU, so its registers are bounded for more waves per SIMD
#ifndef DW_N2V_CN_WAVES
#define DW_N2V_CN_WAVES 5
#endif
template <int CH, int NCAP>
__global__ void __launch_bounds__(REPLAY_WAVES *WAVE)
    __attribute__((amdgpu_waves_per_eu(DW_N2V_CN_WAVES, 8)))
    k_walk_replay_cn(ReplayCtx c, int64_t n_rows, const int32_t *__restrict__ starts,
                     int64_t n_walks, int32_t L, const double *__restrict__ uniforms,
                     int32_t *__restrict__ out, int32_t *status, int fast, N2VIndex ix) {
    walk_replay_body<CH, NCAP, true>(c, n_rows, starts, n_walks, L, uniforms, out, status, fast,
                                     ix);
}

// ---- node2vec over the position index: one lane per walker ----------------------------------
// With t's position pt and the sorted common-neighbour positions P[0..C) of the step's edge,
// the prefix counts at neighbour i are a_i = [pt <= i] and c_i = #{P <= i}: the pick (the
// first i with D_i = W(a_i, i + 1 - a_i - c_i, c_i) - U T > 0, T = W(A, n - A - C, C)) is
// found by a binary search over j of D at P[j] (c = j + 1), then inside the gap
// (P[j-1], P[j]] where c is j (j + 1 at P[j] itself) by a search with no loads. The D values,
// T, M and the bracketing test are the expressions of node2vec_pick_exact on the same
// integers, so the pick — or the hand-over where the margin fails — is the same.
// EXACT = false (the Philox walker, k_walk_node2vec_positions): no margin tests — the pick is
// the first i at which the fp64 D_i turns positive, an exact draw from W_i / T up to the fp64
// rounding of D (relative 2^-50), the same expressions as the oracle's (oracle/philox.py).
// ---- the exact serial pick, run by run ---------------------------------------------------
// Where the margin cannot decide, the pick is the reference's own arithmetic: sum(w) left to
// right, normalized = w / s, accumulate, bisect_right (random_walk_generator.py:109-111,
// random.choices). Over N(v) the weights are 1 except at t's position (1/p) and the C common
// positions (1/q), so each sequential fp64 sum is a few runs of equal terms, and a run of m equal
// terms y advances in one step per binade of the running sum S: within [B, 2B) (ulp u) every
// addition rounds alike, fl(S + y) = S + D u with D = floor(y / u) (+1 when the remainder
// exceeds u / 2; on a tie the even neighbour, constant once S / u is even). The pick then costs
// O(C + log n) instead of O(n) dependent adds with an adjacency test each (a 393K-neighbour
// hub's serial replay took ~0.5 s in one lane). tests/test_serial_runs.py restates ff_run /
// runs_pass / the pick and checks them bit for bit against the sequential sums and the
// oracle's choices_index.
// ff_run's constants for one term y in one binade [lo, hi) of S (not a tie, D >= 1): every
// addition there adds D ulps, so a run that stays inside costs a multiply and a compare. A pass
// keeps one (its runs all add the same term).
struct RunBinade {
    double lo = 1.0, hi = 0.0, u = 0.0, iu = 0.0, D = 0.0;
};

// m additions of y (> 0) to S: returns the first addition (1-based) after which S > x (S left
// there), or 0 (S after all m).
__device__ int64_t ff_run(double &S, const double y, const int64_t m, const double x,
                          RunBinade &bc) {
    int64_t done = 0;
    while (done < m) {
        if (S >= bc.lo && S < bc.hi) {   // the cached binade: does the rest of the run fit?
            const double room = (bc.hi - S) * bc.iu;   // exact: ulps to the binade's top
            const double left = static_cast<double>(m - done);
            if (left * bc.D <= room) {
                const double Sj = S + (left * bc.D) * bc.u;   // exact (on the grid, <= hi)
                if (x < Sj) {
                    const int64_t js =
                        x < S ? 1
                              : static_cast<int64_t>((x - S) * bc.iu) /
                                        static_cast<int64_t>(bc.D) + 1;
                    S = S + static_cast<double>(js) * bc.D * bc.u;
                    return done + js;
                }
                S = Sj;
                return 0;
            }
        }
        if (S > 0.0 && y < S) {
            const int e =
                static_cast<int>((__double_as_longlong(S) >> 52) & 0x7FF) - 1022;   // S in [2^(e-1), 2^e)
            const double B2 = ldexp(1.0, e);
            const double u = ldexp(1.0, e - 53), iu = ldexp(1.0, 53 - e);
            const double qd = floor(y * iu);             // (powers of two: exact)
            const double r = y - qd * u;                 // exact
            const int64_t q = static_cast<int64_t>(qd);
            const int64_t k = static_cast<int64_t>(S * iu);
            const bool tie = r == 0.5 * u;
            if (!tie || (k & 1) == 0) {
                const int64_t D = q + ((r > 0.5 * u || (tie && (q & 1))) ? 1 : 0);
                if (D == 0) return S > x ? done + 1 : 0;   // the rest add nothing
                if (!tie) bc = RunBinade{0.5 * B2, B2, u, iu, static_cast<double>(D)};
                const int64_t jmax = static_cast<int64_t>((B2 - S) * iu) / D;
                if (jmax > 0) {
                    const int64_t j = jmax < m - done ? jmax : m - done;
                    const double Sj = S + static_cast<double>(j * D) * u;
                    if (x < B2 && x < Sj) {   // the crossing is inside the chunk
                        const int64_t js =
                            x < S ? 1 : static_cast<int64_t>((x - S) * iu) / D + 1;
                        S = S + static_cast<double>(js * D) * u;
                        return done + js;
                    }
                    S = Sj;
                    done += j;
                    continue;
                }
            }
        }
        const double t = S + y;   // one addition as it is
        ++done;
        if (t == S) return t > x ? done : 0;
        S = t;
        if (S > x) return done;
    }
    return 0;
}

// The fp64 left-to-right sum of the n terms (`one`, vp at pt, vq at the ascending P[0..C)) in
// S; returns the first index < hi whose partial sum exceeds x, or -1. The positions are read
// four ahead (independent loads in flight while the runs are summed).
__device__ int64_t runs_pass(PosList P, int64_t C, int64_t pt, double vp, double vq, int64_t n,
                             int64_t hi, double one, double x, double &S, uint32_t &loads) {
    S = 0.0;
    RunBinade bc;
    int64_t i = 0, j = 0;   // j: the P entries consumed
    bool p_left = pt >= 0;
    auto ld = [&](int64_t k) -> int64_t { return k < C ? P[k] : n; };
    int64_t q0 = ld(0), q1 = ld(1), q2 = ld(2), q3 = ld(3);
    loads += (P.wide ? 2u : 1u) * static_cast<uint32_t>(C < 4 ? C : 4);
    while (true) {
        int64_t pos;
        double val;
        if (p_left && pt < q0) {
            pos = pt;
            val = vp;
            p_left = false;
        } else if (j < C) {
            pos = q0;
            val = vq;
            ++j;
            q0 = q1;
            q1 = q2;
            q2 = q3;
            q3 = ld(j + 3);
            if (j + 3 < C) loads += P.wide ? 2u : 1u;
        } else {
            pos = n;
            val = 0.0;
        }
        const int64_t end = pos < hi ? pos : hi;
        if (end > i) {
            const int64_t k = ff_run(S, one, end - i, x, bc);
            if (k) return i + k - 1;
        }
        if (pos >= hi) return -1;
        S = S + val;
        if (S > x) return pos;
        i = pos + 1;
    }
}

// runs_pass for long lists (tests/test_serial_runs.py seq_pass_bs): inside one binade of S
// (ulp u, none of `one` / vq a tie or above its bottom) every addition adds a fixed number of
// ulps, D1 for a one and Dq for a special, so k(t) = S / u after the elements [i, t) is
// k0 + D1 (ones) + Dq (specials) — increasing in t. The binade's end and the crossing of x are
// then a binary search over P and a division in the run of ones before the special found; the
// element that leaves the binade, t's position and any tie are added as they are. O(binades x
// log C) loads per pass (~20 binades from the first term to the sum) instead of O(C).
__device__ __forceinline__ int64_t k_mul_sat(int64_t d, int64_t c) {   // d, c >= 0; capped 2^60
    return (c > 0 && d > (int64_t(1) << 60) / c) ? (int64_t(1) << 60) : d * c;
}

__device__ int64_t runs_pass_bs(PosList P, int64_t C, int64_t pt, double vp, double vq,
                                int64_t n, int64_t hi, double one, double x, double &S,
                                uint32_t &loads) {
    const uint32_t unit = P.wide ? 2u : 1u;
    S = 0.0;
    int64_t i = 0, j = 0;
    bool p_left = pt >= 0;
    const int64_t KT = int64_t(1) << 53;
    while (i < hi) {
        const int64_t seg_end = (p_left && pt < hi) ? pt : hi;
        if (S > 0.0 && i < seg_end) {
            const int e =
                static_cast<int>((__double_as_longlong(S) >> 52) & 0x7FF) - 1022;   // S in [2^(e-1), 2^e)
            const double u = ldexp(1.0, e - 53), iu = ldexp(1.0, 53 - e);
            const double B = ldexp(1.0, e - 1);
            int64_t D1 = 0, Dq = 0;
            bool ok = one < B && vq < B;
            if (ok) {
                const double q1 = floor(one * iu), r1 = one - q1 * u;
                const double qq = floor(vq * iu), rq = vq - qq * u;
                ok = r1 != 0.5 * u && rq != 0.5 * u;
                D1 = static_cast<int64_t>(q1) + (r1 > 0.5 * u ? 1 : 0);
                Dq = static_cast<int64_t>(qq) + (rq > 0.5 * u ? 1 : 0);
                ok = ok && D1 > 0 && Dq > 0;
            }
            if (ok) {
                const int64_t k0 = static_cast<int64_t>(S * iu);
                const bool xin = x < 2.0 * B;   // (x >= S >= B: x on this binade's grid)
                const int64_t XT = xin ? static_cast<int64_t>(x * iu) : KT;
                const int64_t LIM = XT < KT ? XT : KT;
                auto k_after = [&](int64_t jj) -> int64_t {   // k after special jj (>= j)
                    const int64_t pj = P[jj];
                    loads += unit;
                    return k0 + k_mul_sat(D1, pj + 1 - i - (jj + 1 - j)) +
                           k_mul_sat(Dq, jj + 1 - j);
                };
                int64_t lo = j, up = C;   // jc: the first special at or past seg_end
                while (lo < up) {
                    const int64_t mid = (lo + up) >> 1;
                    loads += unit;
                    if (P[mid] < seg_end)
                        lo = mid + 1;
                    else
                        up = mid;
                }
                const int64_t jc = lo;
                lo = j, up = jc;          // jf: the first special whose k passes LIM
                while (lo < up) {
                    const int64_t mid = (lo + up) >> 1;
                    if (k_after(mid) > LIM)
                        up = mid;
                    else
                        lo = mid + 1;
                }
                const int64_t jf = lo;
                const int64_t t0 = jf > j ? P[jf - 1] + 1 : i;
                const int64_t kb = jf > j ? k_after(jf - 1) : k0;
                const int64_t nxt = jf < jc ? P[jf] : seg_end;
                const int64_t run = nxt - t0;   // the ones before special jf
                const int64_t fit = (LIM - kb) / D1;
                const int64_t m = run < fit ? run : fit;
                if (xin && m < run && kb + D1 * (m + 1) <= KT) {   // a one crosses x
                    S = static_cast<double>(kb + D1 * (m + 1)) * u;
                    return t0 + m;
                }
                if (xin && m == run && jf < jc) {
                    const int64_t kf = k_after(jf);
                    if (kf <= KT) {                                  // special jf crosses x
                        S = static_cast<double>(kf) * u;
                        return nxt;
                    }
                }
                if (t0 + m > i) {   // progress inside the binade
                    S = static_cast<double>(kb + D1 * m) * u;
                    i = t0 + m;
                    j = jf;
                    continue;
                }
            }
        }
        // one element as it is
        double val = one;
        if (p_left && pt == i) {
            val = vp;
            p_left = false;
        } else if (j < C) {
            loads += unit;
            if (P[j] == i) {
                val = vq;
                ++j;
            }
        }
        S = S + val;
        if (S > x) return i;
        ++i;
    }
    return -1;
}

// The reference's pick over N(v) (n neighbours; t at pt or -1; the 1/q neighbours at P), by
// its own fp64 arithmetic: the serial replay the margin tests fall back to.
constexpr int64_t RUNS_BS_MIN = 48;   // lists longer than this: by binades
__device__ int64_t n2v_pick_serial_runs(PosList P, int64_t C, int64_t pt, int64_t n, double U,
                                        double ip, double iq, uint32_t &loads) {
    const double inf = __builtin_huge_val();
    double s, total, S;
    // (short lists run by run; long ones by binades)
    auto pass = [&](double vp, double vq, int64_t hi, double one, double x, double &out) {
        return C > RUNS_BS_MIN ? runs_pass_bs(P, C, pt, vp, vq, n, hi, one, x, out, loads)
                               : runs_pass(P, C, pt, vp, vq, n, hi, one, x, out, loads);
    };
    pass(ip, iq, n, 1.0, inf, s);                                      // sum(w)
    const double n1 = 1.0 / s, np = ip / s, nq = iq / s;              // normalized
    pass(np, nq, n, n1, inf, total);                                  // accumulate
    total = total + 0.0;
    const int64_t k = pass(np, nq, n - 1, n1, U * total, S);
    return k < 0 ? n - 1 : k;                                         // bisect_right(.., 0, n-1)
}

// lines (counted launches; NULL otherwise): += the 128-B lines the search's dependent loads
// move to — a probe in the line of the one before it is a cache hit, not another random line
template <bool EXACT = true>
__device__ __forceinline__ int64_t n2v_pick_pos(PosList P, int64_t C, int64_t pt, int64_t n,
                                                double U, double ip, double iq,
                                                uint32_t &loads,   // += 2-B units read (1 per uint16 entry, 2 per int32)
                                                uint32_t *lines = nullptr) {
    uint64_t last_line = ~0ull;
    auto touch = [&](int64_t i) {
        if (!lines) return;
        const uint64_t ln = (reinterpret_cast<uint64_t>(P.p) + static_cast<uint64_t>(i) *
                                                                   (P.wide ? 4u : 2u)) >> 7;
        if (ln != last_line) {
            ++*lines;
            last_line = ln;
        }
    };
    const int64_t A = pt >= 0 ? 1 : 0;
    const double T = n2v_w(A, n - A - C, C, ip, iq);
    const double UT = U * T;
    const double M = EXACT ? exact_margin(n, T) : 0.0;
    if (EXACT && !(T - UT > 0.0)) return -1;   // D_{n-1} <= 0: rounding at the top end
    auto D = [&](int64_t i, int64_t c) {
        const int64_t a = (pt >= 0 && pt <= i) ? 1 : 0;
        return n2v_w(a, (i + 1) - a - c, c, ip, iq) - UT;
    };
    int64_t lo = 0, hi = C;           // first j with D(P[j], j + 1) > 0, else C
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        loads += P.wide ? 2u : 1u;
        touch(mid);
        if (D(P[mid], mid + 1) > 0.0)
            hi = mid;
        else
            lo = mid + 1;
    }
    const int64_t j = lo;
    const int64_t pj = j < C ? P[j] : n - 1;   // D(pj) > 0
    int64_t a = j > 0 ? P[j - 1] + 1 : 0;       // D(P[j-1]) <= 0
    if (j > 0) {
        loads += P.wide ? 2u : 1u;
        touch(j - 1);
    }
    int64_t b = pj;
    while (a < b) {                   // i < pj: c_i = j
        const int64_t mid = (a + b) >> 1;
        if (D(mid, j) > 0.0)
            b = mid;
        else
            a = mid + 1;
    }
    const int64_t k = a;
    if constexpr (EXACT) {
        const double d_k = D(k, (j < C && k == pj) ? j + 1 : j);
        if (k >= 1 && fabs(D(k - 1, j)) <= M) return -1;
        if (k <= n - 2 && fabs(d_k) <= M) return -1;
    }
    return k;
}

// The walks of dw_walk_replay_indexed, one lane per walker over the 32-B edge records
// (k_n2v_edge_records): a step is the record of the edge it arrived by (its next row and its
// index entry in one line), the search of its positions, and nothing else. The uniforms are
// staged in LDS per tile of steps as in k_walk_replay_uniform_inline. A pick the margin leaves
// open is made by the reference's arithmetic itself, run by run (n2v_pick_serial_runs).
// 8 staged steps per tile (17 KiB of LDS per block): the walk is latency-bound, so blocks
// per CU count for more than the uniforms' reload rate
constexpr int RP_T = 8;
template <bool COUNT>
__global__ void __launch_bounds__(256)
    k_walk_replay_n2v_pos(const int64_t *__restrict__ row_ptr, const int4 *__restrict__ rec,
                          const uint8_t *__restrict__ pos, int64_t n_rows,
                          const int32_t *__restrict__ starts, int64_t n_walks, int32_t L,
                          const double *__restrict__ uniforms, double ip, double iq,
                          int32_t *__restrict__ out, int32_t *status,
                          unsigned long long *counters) {
    __shared__ double tile[256][RP_T + 1];
    const int tid = threadIdx.x;
    const int64_t n_chunks = (n_walks + 255) / 256;
    const int64_t UL = L - 1;
    uint32_t loads = 0, steps = 0, serial = 0, lines = 0;
    for (int64_t ch = blockIdx.x; ch < n_chunks; ch += gridDim.x) {
        const int64_t w0 = ch * 256;
        const int n_here = (n_walks - w0 < 256) ? static_cast<int>(n_walks - w0) : 256;
        const int64_t wk = w0 + tid;
        const bool live = tid < n_here;
        int32_t v = live ? starts[wk] : 0;
        int32_t *o = out + wk * (int64_t)L;
        bool ok = live && v >= 0 && (int64_t)v < n_rows;
        if (live && !ok) dw::status_or(status, DW_S_BAD_CSR);
        int64_t a = ok ? row_ptr[v] : 0;
        int64_t n = ok ? row_ptr[v + 1] - a : 0;
        int32_t prev = -1;
        int64_t e_in = -1, p_off = 0;
        uint32_t cw = 0;   // the counts word of e_in
        int32_t pt = -1;
        const bool pack = (L & 3) == 0;
        int32_t q0 = v, q1 = -1, q2 = -1;
        if (live && !pack) o[0] = v;
        for (int64_t t0 = 0; t0 < UL; t0 += RP_T) {
            const int tn = (UL - t0 < RP_T) ? static_cast<int>(UL - t0) : RP_T;
            __syncthreads();
#pragma unroll 4
            for (int it = 0; it < RP_T; ++it) {
                const int e = it * 256 + tid;
                const int wl = e / RP_T, sl = e % RP_T;
                if (wl < n_here && sl < tn) tile[wl][sl] = uniforms[(w0 + wl) * UL + t0 + sl];
            }
            __syncthreads();
            if (!live) continue;
            for (int j = 0; j < tn; ++j) {
                const int32_t st = static_cast<int32_t>(t0) + 1 + j;
                int32_t node = -1;
                if (ok) {
                    if (n <= 0) {
                        dw::status_or(status, DW_S_ISOLATED_NODE);
                        ok = false;
                    } else {
                        const double U = tile[tid][j];
                        if (COUNT) ++steps;
                        const PosList PL{pos + p_off, n > N2V_U16_MAX_DEG};
                        const int64_t C = prev < 0 ? 0 : (cw & 0x7FFFFFFFu);
                        const int64_t ptv = (prev >= 0 && (cw >> 31)) ? pt : -1;
                        int64_t k = prev < 0 ? uniform_pick_exact(U, n)
                                             : n2v_pick_pos(PL, C, ptv, n, U, ip, iq, loads,
                                                            COUNT ? &lines : nullptr);
                        if (k < 0) {   // the margin cannot decide: the reference's arithmetic
                            k = n2v_pick_serial_runs(PL, C, ptv, n, U, ip, iq, loads);
                            if (COUNT) ++serial;
                        }
                        {
                            const int64_t e = a + k;
                            const int4 r0 = rec[2 * e], r1 = rec[2 * e + 1];
                            prev = v;
                            v = r0.x;
                            n = r0.y;
                            a = static_cast<int64_t>(static_cast<uint32_t>(r0.z)) |
                                (static_cast<int64_t>(r0.w) << 32);
                            p_off = static_cast<int64_t>(static_cast<uint32_t>(r1.x)) |
                                    (static_cast<int64_t>(r1.y) << 32);
                            cw = static_cast<uint32_t>(r1.z);
                            pt = r1.w;
                            e_in = e;
                            node = v;
                        }
                    }
                }
                if (!pack) {
                    o[st] = node;
                } else {
                    switch (st & 3) {
                        case 0: q0 = node; break;
                        case 1: q1 = node; break;
                        case 2: q2 = node; break;
                        default:
                            reinterpret_cast<int4 *>(o)[st >> 2] = int4{q0, q1, q2, node};
                    }
                }
            }
        }
    }
    if (COUNT) {   // per step the 32-B record, the uniform and the output (44 B); the positions
                   // read (2-B units); the serial picks; the searches' line moves
        unsigned long long v2[4] = {(unsigned long long)loads, (unsigned long long)steps,
                                    (unsigned long long)serial, (unsigned long long)lines};
        for (int k = 0; k < 4; ++k)
            for (int off = WAVE / 2; off > 0; off >>= 1) v2[k] += __shfl_xor(v2[k], off, WAVE);
        if ((tid & (WAVE - 1)) == 0) {
            atomicAdd(counters + 0, v2[0] * 2ull + v2[1] * 44ull);
            atomicAdd(counters + 1, v2[2]);
            atomicAdd(counters + 2, v2[0]);
            atomicAdd(counters + 3, v2[1]);
            atomicAdd(counters + 4, v2[3]);
        }
    }
}

// =============================================================================================
// Fast walkers
// =============================================================================================

// One first-order draw from row [a, a+n): uniform neighbour, or Vose alias when weighted.
__device__ __forceinline__ int64_t first_order_pick(uint32_t r0, uint32_t r1, int64_t a,
                                                    int64_t n, const uint32_t *prob_thr,
                                                    const int32_t *alias) {
    int64_t i = dw::bounded32(r0, static_cast<uint32_t>(n));
    if (prob_thr) {
        const uint32_t t = prob_thr[a + i];
        if (t != ALWAYS && r1 >= t) i = alias[a + i];
    }
    return i;
}

__global__ void __launch_bounds__(256)
    k_walk_deepwalk_fast(const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
                         const uint32_t *__restrict__ prob_thr, const int32_t *__restrict__ alias,
                         int64_t n_rows, const int32_t *__restrict__ starts, int64_t n_walks,
                         int32_t L, uint32_t k0, uint32_t k1, uint64_t walk_id0,
                         int32_t *__restrict__ out, int32_t *status,
                         const dw_step_scalars *__restrict__ dyn) {
    const int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (w >= n_walks) return;
    const uint64_t wid = (dyn ? dyn->walk_id0 : walk_id0) + static_cast<uint64_t>(w);
    int32_t *o = out + w * (int64_t)L;
    int32_t v = starts[w];
    o[0] = v;
    int32_t s = 1;
    for (; s < L; ++s) {
        if (v < 0 || (int64_t)v >= n_rows) {
            dw::status_or(status, DW_S_BAD_CSR);
            break;
        }
        const int64_t a = row_ptr[v];
        const int64_t n = row_ptr[v + 1] - a;
        if (n <= 0) {
            dw::status_or(status, DW_S_ISOLATED_NODE);
            break;
        }
        const dw::U4 r = dw::philox(dw::U4{static_cast<uint32_t>(wid),
                                           static_cast<uint32_t>(wid >> 32),
                                           static_cast<uint32_t>(s) << 8, dw::TAG_DEEPWALK},
                                    k0, k1);
        v = col[a + first_order_pick(r.x, r.y, a, n, prob_thr, alias)];
        o[s] = v;
    }
    for (; s < L; ++s) o[s] = -1;
}

// DeepWalk over the edge-inline CSR (dw_edges_inline_build): entry e of row u is the int4
// {x, deg(x), row_ptr[x] (lo, hi)}, so the pick of the next node also yields its row — one
// dependent load per step where the CSR walk needs two (row_ptr, then col). Same Philox draws
// and picks as k_walk_deepwalk_fast: bit-identical walks.
// DeepWalk, one lane per walker; the walk leaves in 16-B stores of 4 steps when L % 4 == 0.
__global__ void __launch_bounds__(256)
    k_walk_deepwalk_inline(const int64_t *__restrict__ row_ptr, const int4 *__restrict__ edges,
                           const uint32_t *__restrict__ prob_thr, const int32_t *__restrict__ alias,
                           int64_t n_rows, const int32_t *__restrict__ starts, int64_t n_walks,
                           int32_t L, uint32_t k0, uint32_t k1, uint64_t walk_id0,
                           int32_t *__restrict__ out, int32_t *status,
                           const dw_step_scalars *__restrict__ dyn) {
    const int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (w >= n_walks) return;
    const uint64_t wid = (dyn ? dyn->walk_id0 : walk_id0) + static_cast<uint64_t>(w);
    int32_t *o = out + w * (int64_t)L;
    int32_t v = starts[w];
    bool ok = v >= 0 && (int64_t)v < n_rows;
    if (!ok) dw::status_or(status, DW_S_BAD_CSR);
    int64_t a = ok ? row_ptr[v] : 0;
    int64_t n = ok ? row_ptr[v + 1] - a : 0;
    auto draw = [&](int32_t s) {
        return dw::philox(dw::U4{static_cast<uint32_t>(wid), static_cast<uint32_t>(wid >> 32),
                                 static_cast<uint32_t>(s) << 8, dw::TAG_DEEPWALK},
                          k0, k1);
    };
    dw::U4 r = draw(1);   // the draw of the coming step: computed while the previous load flies
    auto step = [&](int32_t s) -> int32_t {   // node at step s >= 1 (-1 once the walk aborted)
        if (!ok) return -1;
        if (n <= 0) {
            dw::status_or(status, DW_S_ISOLATED_NODE);
            ok = false;
            return -1;
        }
        const int4 e = edges[a + first_order_pick(r.x, r.y, a, n, prob_thr, alias)];
        r = draw(s + 1);   // independent of e: overlaps the load's latency
        a = static_cast<int64_t>(static_cast<uint32_t>(e.z)) | (static_cast<int64_t>(e.w) << 32);
        n = e.y;
        return e.x;
    };
    if ((L & 3) == 0) {
        int4 *o4 = reinterpret_cast<int4 *>(o);
        for (int32_t s0 = 0; s0 < L; s0 += 4) {
            int4 pk;
            pk.x = s0 == 0 ? v : step(s0);
            pk.y = step(s0 + 1);
            pk.z = step(s0 + 2);
            pk.w = step(s0 + 3);
            o4[s0 >> 2] = pk;
        }
    } else {
        o[0] = v;
        for (int32_t s = 1; s < L; ++s) o[s] = step(s);
    }
}

// node2vec (Philox) over the per-edge position index (dw_n2v_edge_index_build), one lane per
// walker: the exact replay walker's step (k_walk_replay_n2v_pos) with its uniform drawn from
// Philox instead of CPython's stream — one 32-B edge record per step (the next row and the
// step's index entry), log2 C dependent 2- or 4-B position loads, no rejection rounds and no
// adjacency tests. The first step picks bounded32(r.x, n) (the unbiased first step,
// random_walk_generator.py:97), later steps U = 53 bits of (r.x, r.y) (genrand_res53's split)
// against the prefix weights of the reference rule (:100-108) through n2v_pick_pos<false>.
// Counter (walk id lo, hi, step << 8, TAG_N2V_POS); restated in oracle/philox.py
// (fast_walks_positions). The next step's draw is computed while the record load is in flight.
// COUNT: realised bytes (the 32-B record and 4-B output per step, 2 or 4 B per position load,
// the start's row_ptr pair) and steps into counters[0], counters[1], the searches' 128-B line
// moves in counters[2], the positions read in 2-B units in counters[3].
template <bool COUNT>
__global__ void __launch_bounds__(256)
    k_walk_node2vec_positions(const int64_t *__restrict__ row_ptr, const int4 *__restrict__ rec,
                              const uint8_t *__restrict__ pos, int64_t n_rows,
                              const int32_t *__restrict__ starts, int64_t n_walks, int32_t L,
                              double ip, double iq, uint32_t k0, uint32_t k1, uint64_t walk_id0,
                              int32_t *__restrict__ out, int32_t *status,
                              const dw_step_scalars *__restrict__ dyn,
                              unsigned long long *counters) {
    const int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    uint32_t loads = 0, steps = 0, lines = 0;
    if (w < n_walks) {
        const uint64_t wid = (dyn ? dyn->walk_id0 : walk_id0) + static_cast<uint64_t>(w);
        int32_t *o = out + w * (int64_t)L;
        int32_t v = starts[w];
        bool ok = v >= 0 && (int64_t)v < n_rows;
        if (!ok) dw::status_or(status, DW_S_BAD_CSR);
        int64_t a = ok ? row_ptr[v] : 0;
        int64_t n = ok ? row_ptr[v + 1] - a : 0;
        bool second = false;                 // a previous node exists (steps >= 2)
        int64_t p_off = 0;
        uint32_t cw = 0;                     // the counts word of the edge taken
        int32_t pt = -1;                     // the previous node's position in N(v)
        auto draw = [&](int32_t s) {
            return dw::philox(dw::U4{static_cast<uint32_t>(wid), static_cast<uint32_t>(wid >> 32),
                                     static_cast<uint32_t>(s) << 8, dw::TAG_N2V_POS},
                              k0, k1);
        };
        dw::U4 r = draw(1);
        auto step = [&](int32_t s) -> int32_t {   // node at step s >= 1 (-1 once aborted)
            if (!ok) return -1;
            if (n <= 0) {
                dw::status_or(status, DW_S_ISOLATED_NODE);
                ok = false;
                return -1;
            }
            int64_t k;
            if (!second) {
                k = dw::bounded32(r.x, static_cast<uint32_t>(n));
            } else {
                const double U = static_cast<double>((static_cast<uint64_t>(r.x >> 5) << 26) |
                                                     static_cast<uint64_t>(r.y >> 6)) *
                                 0x1p-53;
                k = n2v_pick_pos<false>(PosList{pos + p_off, n > N2V_U16_MAX_DEG},
                                        cw & 0x7FFFFFFFu, (cw >> 31) ? pt : -1, n, U, ip, iq,
                                        loads, COUNT ? &lines : nullptr);
            }
            const int64_t e = a + k;
            const int4 r0 = rec[2 * e], r1 = rec[2 * e + 1];
            r = draw(s + 1);   // independent of the record: overlaps its latency
            if (COUNT) ++steps;
            v = r0.x;
            n = r0.y;
            a = static_cast<int64_t>(static_cast<uint32_t>(r0.z)) |
                (static_cast<int64_t>(r0.w) << 32);
            p_off = static_cast<int64_t>(static_cast<uint32_t>(r1.x)) |
                    (static_cast<int64_t>(r1.y) << 32);
            cw = static_cast<uint32_t>(r1.z);
            pt = r1.w;
            second = true;
            return v;
        };
        if ((L & 3) == 0) {
            int4 *o4 = reinterpret_cast<int4 *>(o);
            const int32_t v0 = v;
            for (int32_t s0 = 0; s0 < L; s0 += 4) {
                int4 pk;
                pk.x = s0 == 0 ? v0 : step(s0);
                pk.y = step(s0 + 1);
                pk.z = step(s0 + 2);
                pk.w = step(s0 + 3);
                o4[s0 >> 2] = pk;
            }
        } else {
            o[0] = v;
            for (int32_t s = 1; s < L; ++s) o[s] = step(s);
        }
    }
    if (COUNT) {
        const int lane = threadIdx.x & (WAVE - 1);
        unsigned long long v3[4] = {
            (unsigned long long)loads * 2ull + (unsigned long long)steps * 36ull +
                (w < n_walks ? 20ull : 0ull),
            (unsigned long long)steps, (unsigned long long)lines, (unsigned long long)loads};
        for (int k = 0; k < 4; ++k)
            for (int off = WAVE / 2; off > 0; off >>= 1) v3[k] += __shfl_xor(v3[k], off, WAVE);
        if (lane == 0) {
            atomicAdd(counters + 0, v3[0]);
            atomicAdd(counters + 1, v3[1]);
            atomicAdd(counters + 2, v3[2]);
            atomicAdd(counters + 3, v3[3]);
        }
    }
}

// One block per hub row: its neighbours as bits of a V-bit map (the bit-exact node2vec replay's
// membership test against a hub prev: one 4-B load instead of a search of its sorted list).
__global__ void __launch_bounds__(256)
    k_hub_bitmaps(const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
                  const int32_t *__restrict__ hub_rows, int64_t hub_words,
                  uint32_t *__restrict__ bits) {
    const int32_t r = hub_rows[blockIdx.x];
    uint32_t *b = bits + blockIdx.x * hub_words;
    for (int64_t e = row_ptr[r] + threadIdx.x; e < row_ptr[r + 1]; e += blockDim.x) {
        const int32_t x = col[e];
        atomicOr(b + (x >> 5), 1u << (x & 31));
    }
}

__global__ void k_edges_inline(const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
                               int64_t nnz, int4 *__restrict__ edges) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nnz; e += stride) {
        const int32_t x = col[e];
        const int64_t a = row_ptr[x];
        edges[e] = int4{x, static_cast<int32_t>(row_ptr[x + 1] - a),
                        static_cast<int32_t>(static_cast<uint32_t>(a)),
                        static_cast<int32_t>(a >> 32)};
    }
}

// dw_step_starts / dw_step_scalars_advance: the per-step values of a replayed training step.
__global__ void __launch_bounds__(256)
    k_step_starts(const dw_step_scalars *__restrict__ dyn, const int32_t *__restrict__ epoch,
                  int64_t n_epoch, int32_t *__restrict__ out, int64_t n) {
    const uint64_t base = dyn->walk_id0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += stride)
        out[k] = epoch[(base + static_cast<uint64_t>(k)) % static_cast<uint64_t>(n_epoch)];
}

// One block: thread 0 moves the block to the next step; then (epoch != NULL) the block's
// threads write that step's start nodes, as k_step_starts would (one launch instead of two).
__global__ void __launch_bounds__(256)
    k_step_advance(dw_step_scalars *dyn, const float *__restrict__ hist, int64_t hist_rows,
                   uint64_t walks_per_step, uint64_t centres_per_step, int32_t *status,
                   const int32_t *__restrict__ epoch, int64_t n_epoch,
                   int32_t *__restrict__ starts_out, int64_t n) {
    __shared__ uint64_t next_wid;
    if (threadIdx.x == 0) {
        const uint64_t wid = dyn->walk_id0 + walks_per_step;
        dyn->walk_id0 = wid;
        next_wid = wid;
        dyn->noise_offset += centres_per_step;
        const int64_t s = ++dyn->step;
        if (s >= hist_rows)
            dw::status_or(status, DW_S_BAD_INDEX);
        else
            for (int k = 0; k < 8; ++k) dyn->adam[k] = hist[8 * s + k];
    }
    if (!epoch) return;
    __syncthreads();
    const uint64_t base = next_wid;
    for (int64_t k = threadIdx.x; k < n; k += blockDim.x)
        starts_out[k] = epoch[(base + static_cast<uint64_t>(k)) % static_cast<uint64_t>(n_epoch)];
}

// dw_step_scalars_expand: one block; thread 0 writes the blocks of the next n_steps steps and
// moves `base` past them, then the block's threads write the first one's start nodes (for all
// the steps' walks: n = n_steps * walks per step).
__global__ void __launch_bounds__(256)
    k_step_expand(dw_step_scalars *base, dw_step_scalars *steps, int64_t n_steps,
                  const float *__restrict__ hist, int64_t hist_rows, uint64_t walks_per_step,
                  uint64_t centres_per_step, int32_t *status, const int32_t *__restrict__ epoch,
                  int64_t n_epoch, int32_t *__restrict__ starts_out, int64_t n) {
    __shared__ uint64_t first_wid;
    if (threadIdx.x == 0) {
        dw_step_scalars b = *base;
        first_wid = b.walk_id0;
        for (int64_t j = 0; j <= n_steps; ++j) {
            if (j > 0) {  // the advance of dw_step_scalars_advance
                b.walk_id0 += walks_per_step;
                b.noise_offset += centres_per_step;
                const int64_t s = ++b.step;
                if (s >= hist_rows)
                    dw::status_or(status, DW_S_BAD_INDEX);
                else
                    for (int k = 0; k < 8; ++k) b.adam[k] = hist[8 * s + k];
            }
            if (j < n_steps) steps[j] = b;
        }
        *base = b;
    }
    if (!epoch) return;
    __syncthreads();
    const uint64_t w0 = first_wid;
    for (int64_t k = threadIdx.x; k < n; k += blockDim.x)
        starts_out[k] = epoch[(w0 + static_cast<uint64_t>(k)) % static_cast<uint64_t>(n_epoch)];
}

constexpr int N2V_WAVES = 4;     // waves per block
// (Occupancy: the hashed variant compiles to 73 VGPRs, 6 waves/SIMD. Forcing 8 waves/SIMD
// (amdgpu_waves_per_eu) spills to scratch and measured 16% slower at C3.)

struct N2VThr {
    uint32_t p, q, one;  // accept iff r < thr (ALWAYS = unconditional)
};

// The G-bit slice of a wave ballot that belongs to this lane's group.
template <int G>
__device__ __forceinline__ uint32_t group_ballot(bool pred, int q) {
    return static_cast<uint32_t>((__ballot(pred) >> (G * q)) & ((1ull << G) - 1ull));
}

// Membership of a group-uniform key in a sorted int32 list [0, n), the N2V_G lanes of a group
// cooperating: N2V_G-ary search — lane j reads splitter j of the current range, one ballot picks
// the segment, until <= N2V_G entries remain and one load + ballot decides. ceil(log_G n)
// dependent loads (6 at G=8 for the largest C3 hub, 44,848 neighbours), no LDS staging.
template <int N2V_G>
__device__ __forceinline__ bool group_contains(const int32_t *__restrict__ list, int64_t n,
                                               int32_t key, int gl, int q, uint32_t &bytes) {
    int64_t lo = 0, len = n;
    while (len > N2V_G) {
        const int64_t idx = lo + (static_cast<int64_t>(gl) * len) / N2V_G;
        const int32_t sv = list[idx];
        bytes += 4 * N2V_G;
        if (group_ballot<N2V_G>(sv == key, q)) return true;
        const int c = __popc(group_ballot<N2V_G>(sv < key, q));  // splitters below key: 0 .. c-1
        if (c == 0) return false;                          // key < list[lo]
        const int64_t s0 = lo + (static_cast<int64_t>(c - 1) * len) / N2V_G;
        const int64_t s1 = (c == N2V_G) ? lo + len : lo + (static_cast<int64_t>(c) * len) / N2V_G;
        lo = s0;
        len = s1 - s0;
    }
    const bool hit = gl < len && list[lo + gl] == key;
    bytes += 4 * static_cast<uint32_t>(len);
    return group_ballot<N2V_G>(hit, q) != 0u;
}

// Membership of a group-uniform key in a row's adjacency hash (dw_adj_hash_build): the group
// reads one 64-B bucket (16 slots, 16/N2V_G per lane); a hit -> true, a free slot -> false
// (slots fill in probe order and never empty), else the next bucket. At load <= 3/4 the first
// bucket almost always decides; nb probes bound the loop.
template <int N2V_G>
__device__ __forceinline__ bool group_hash_contains(const int32_t *__restrict__ tab, uint32_t nb,
                                                    int32_t key, int gl, int q, uint32_t &bytes) {
    constexpr int PER = 16 / N2V_G;
    uint32_t b = dw::adj_bucket(key, nb);
    for (uint32_t t = 0; t < nb; ++t) {
        const int32_t *slot = tab + (int64_t)b * 16 + gl * PER;
        bytes += 64;
        bool hit = false, free_slot = false;
        if constexpr (PER == 4) {
            const int4 e = *reinterpret_cast<const int4 *>(slot);
            hit = e.x == key || e.y == key || e.z == key || e.w == key;
            free_slot = e.x < 0 || e.y < 0 || e.z < 0 || e.w < 0;
        } else if constexpr (PER == 2) {
            const int2 e = *reinterpret_cast<const int2 *>(slot);
            hit = e.x == key || e.y == key;
            free_slot = e.x < 0 || e.y < 0;
        } else {
            const int32_t e = *slot;
            hit = e == key;
            free_slot = e < 0;
        }
        if (group_ballot<N2V_G>(hit, q)) return true;
        if (group_ballot<N2V_G>(free_slot, q)) return false;
        if (++b == nb) b = 0;
    }
    return false;
}

// Membership in a short UNSORTED list (a row without an adjacency hash, degree <= 8): the group
// reads it N2V_G entries at a time.
template <int N2V_G>
__device__ __forceinline__ bool small_contains(const int32_t *__restrict__ list, int64_t n,
                                               int32_t key, int gl, int q, uint32_t &bytes) {
    bytes += 4 * static_cast<uint32_t>(n);
    bool hit = false;
    for (int64_t t = gl; t < n; t += N2V_G) hit = hit || list[t] == key;
    return group_ballot<N2V_G>(hit, q) != 0u;
}

// N2V_G lanes per walker (8 by default: 8 walkers per wave — the walk is latency-bound, so
// walkers in flight matter more than proposals per instruction). A rejection round draws
// proposals j = 0..63 (Philox counter lane field j; oracle/philox.py fast_walks) and picks the
// LOWEST accepting j; the group evaluates them N2V_G at a time in j order and stops at the first block holding an
// acceptance, which selects the same j as evaluating all 64 at once. A proposal x != prev is
// accepted iff r < thr(x in N(prev) ? q : one); when r is below both thresholds (accept) or
// not below either (reject) the adjacency test cannot change the outcome, so only the
// "ambiguous" proposals BELOW the block's first certain acceptance are tested, in j order,
// each by one group-cooperative search of N(prev): HASH = false, an N2V_G-ary search of the
// sorted list `nbr` (col_sorted); HASH = true, one probe of prev's adjacency hash, or for a row
// without one (degree <= DW_ADJ_HASH_MIN_DEG) one load of its list `nbr` (= col, unsorted).
// STATS (dw_walk_fast_counted, a diagnostic launch; the walks are the same): every walker's
// realised load/store bytes, steps, proposal blocks and adjacency tests, summed per wave and
// added to counters[0..3] once per wave.
template <int N2V_G, bool HASH, bool STATS>
__global__ void __launch_bounds__(N2V_WAVES *WAVE)
    k_walk_node2vec_fast(const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
                         const int32_t *__restrict__ nbr, const int64_t *__restrict__ adj_off,
                         const int32_t *__restrict__ adj_hash,
                         const uint32_t *__restrict__ prob_thr, const int32_t *__restrict__ alias,
                         int64_t n_rows, const int32_t *__restrict__ starts, int64_t n_walks,
                         int32_t L, N2VThr thr, uint32_t k0, uint32_t k1, uint64_t walk_id0,
                         int32_t *__restrict__ out, int32_t *status,
                         unsigned long long *counters, const dw_step_scalars *__restrict__ dyn) {
    if (dyn) walk_id0 = dyn->walk_id0;
    uint32_t c_bytes = 0, c_steps = 0, c_blocks = 0, c_tests = 0;   // STATS only
    const uint32_t pick_bytes = prob_thr ? 12u : 4u;   // col (+ prob_thr, alias) per proposal
    const int lane = threadIdx.x & (WAVE - 1);
    const int q = lane / N2V_G, gl = lane & (N2V_G - 1);
    const int wv = threadIdx.x / WAVE;
    constexpr int GPW = WAVE / N2V_G;  // walkers per wave
    const int64_t n_slots = (int64_t)gridDim.x * N2V_WAVES * GPW;
    // thresholds as 33-bit bounds: accept iff r < T (ALWAYS -> 2^32)
    const uint64_t Tp = thr.p == ALWAYS ? (1ull << 32) : thr.p;
    const uint64_t Tq = thr.q == ALWAYS ? (1ull << 32) : thr.q;
    const uint64_t T1 = thr.one == ALWAYS ? (1ull << 32) : thr.one;
    const uint64_t Tlo = Tq < T1 ? Tq : T1, Thi = Tq < T1 ? T1 : Tq;
    const bool adj_wins = Tq > T1;  // in the ambiguous band: accept iff (x in N(prev)) == adj_wins

    for (int64_t base = ((int64_t)blockIdx.x * N2V_WAVES + wv) * GPW; base < n_walks;
         base += n_slots) {
        const int64_t w = base + q;
        if (w >= n_walks) continue;
        const uint64_t wid = walk_id0 + static_cast<uint64_t>(w);
        const uint32_t c0 = static_cast<uint32_t>(wid), c1 = static_cast<uint32_t>(wid >> 32);
        int32_t *o = out + w * (int64_t)L;
        int32_t v = starts[w];
        int32_t prev = -1;
        int64_t pa = 0, pn = 0;  // CSR range of prev (carried from the previous step)
        int64_t ph = 0;          // prev's adjacency-hash buckets (HASH), with their count pnb
        uint32_t pnb = 0;
        if (gl == 0) o[0] = v;
        int32_t s = 1;
        for (; s < L; ++s) {
            if (v < 0 || (int64_t)v >= n_rows) {
                if (gl == 0) dw::status_or(status, DW_S_BAD_CSR);
                break;
            }
            const int64_t a = row_ptr[v];
            const int64_t n = row_ptr[v + 1] - a;
            int64_t h = 0;
            uint32_t nb = 0;
            if constexpr (HASH) {   // independent of the row_ptr loads: same latency slot
                h = adj_off[v];
                nb = static_cast<uint32_t>((adj_off[v + 1] - h) >> 4);
            }
            if (n <= 0) {
                if (gl == 0) dw::status_or(status, DW_S_ISOLATED_NODE);
                break;
            }
            if constexpr (STATS) {
                c_steps += 1;
                c_bytes += (HASH ? 32u : 16u) + 4u;   // row_ptr (+ adj_off) pairs, the output
            }
            int32_t nxt;
            if (prev < 0) {  // first step: prev_node is None -> unbiased (random_walk_generator.py:97)
                const dw::U4 r = dw::philox(
                    dw::U4{c0, c1, static_cast<uint32_t>(s) << 8, dw::TAG_NODE2VEC}, k0, k1);
                nxt = col[a + first_order_pick(r.x, r.y, a, n, prob_thr, alias)];
                if constexpr (STATS) c_bytes += pick_bytes;
            } else {
                nxt = -1;
                for (uint32_t round = 0; round < DW_MAX_REJECTION_ROUNDS && nxt < 0; ++round) {
                    for (int blk = 0; blk < WAVE / N2V_G; ++blk) {
                        const uint32_t j = static_cast<uint32_t>(blk * N2V_G + gl);
                        const dw::U4 r = dw::philox(
                            dw::U4{c0, c1, (static_cast<uint32_t>(s) << 8) | j,
                                   dw::TAG_NODE2VEC ^ round},
                            k0, k1);
                        const int32_t x = col[a + first_order_pick(r.x, r.y, a, n, prob_thr, alias)];
                        if constexpr (STATS) {
                            c_blocks += 1;
                            c_bytes += N2V_G * pick_bytes;
                        }
                        const uint64_t u = r.z;
                        const bool sure = (x == prev) ? (u < Tp) : (u < Tlo);
                        const bool amb = x != prev && u >= Tlo && u < Thi;
                        const uint32_t m_sure = group_ballot<N2V_G>(sure, q);
                        const int f = m_sure ? __ffs(m_sure) - 1 : N2V_G;
                        uint32_t m_amb = group_ballot<N2V_G>(amb, q);
                        if (f < N2V_G) m_amb &= (1u << f) - 1u;
                        int win = f;
                        while (m_amb) {  // group-uniform loop over the candidates that matter
                            const int l = __ffs(m_amb) - 1;
                            const int32_t xl = __shfl(x, q * N2V_G + l, WAVE);
                            bool adj;
                            uint32_t tb = 0;
                            if (HASH && pnb > 0)
                                adj = group_hash_contains<N2V_G>(adj_hash + ph, pnb, xl, gl, q, tb);
                            else
                                adj = HASH ? small_contains<N2V_G>(nbr + pa, pn, xl, gl, q, tb)
                                           : group_contains<N2V_G>(nbr + pa, pn, xl, gl, q, tb);
                            if constexpr (STATS) {
                                c_tests += 1;
                                c_bytes += tb;
                            }
                            if (adj == adj_wins) {
                                win = l;
                                break;
                            }
                            m_amb &= m_amb - 1u;
                        }
                        if (win < N2V_G) {
                            nxt = __shfl(x, q * N2V_G + win, WAVE);
                            break;
                        }
                    }
                }
                if (nxt < 0) {
                    if (gl == 0) dw::status_or(status, DW_S_REJECTION_CAP);
                    break;
                }
            }
            if (gl == 0) o[s] = nxt;
            prev = v;
            pa = a;
            pn = n;
            ph = h;
            pnb = nb;
            v = nxt;
        }
        if (gl == 0)
            for (; s < L; ++s) o[s] = -1;
    }
    if constexpr (STATS) {   // one group lane counts; sum the wave, one atomic per counter
        uint32_t v4[4] = {gl == 0 ? c_bytes : 0u, gl == 0 ? c_steps : 0u,
                          gl == 0 ? c_blocks : 0u, gl == 0 ? c_tests : 0u};
        for (int k = 0; k < 4; ++k) {
            unsigned long long x = v4[k];
            for (int off = WAVE / 2; off > 0; off >>= 1) x += __shfl_xor(x, off, WAVE);
            if (lane == 0) atomicAdd(counters + k, x);
        }
    }
}

inline uint32_t accept_threshold(double alpha, double alpha_max) {
    const double r = alpha / alpha_max;
    if (r >= 1.0) return ALWAYS;
    double t = floor(r * 4294967296.0);
    if (t < 0.0) t = 0.0;
    if (t > 4294967294.0) t = 4294967294.0;
    return static_cast<uint32_t>(t);
}

// Walkers of k_walk_node2vec_fast<G> the device keeps resident at once.
inline int64_t node2vec_capacity(const void *kern, int g) {
    int dev = 0, n_cu = 0, bpc = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n_cu <= 0)
        n_cu = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, kern, N2V_WAVES * WAVE, 0) !=
            hipSuccess || bpc <= 0)
        bpc = 6;
    return (int64_t)bpc * n_cu * N2V_WAVES * (WAVE / g);
}

template <bool HASH>
int launch_node2vec(const int64_t *row_ptr, const int32_t *col, const int32_t *nbr,
                    const int64_t *adj_off, const int32_t *adj_hash, const uint32_t *prob_thr,
                    const int32_t *alias, int64_t n_rows, const int32_t *starts, int64_t n_walks,
                    int32_t walk_length, double p, double q, uint32_t k0, uint32_t k1,
                    uint64_t walk_id0, int32_t *out, int32_t *status, void *stream,
                    unsigned long long *counters = nullptr) {
    DW_REQUIRE(p > 0.0 && q > 0.0, "dw_walk_fast: p and q must be positive");
    const double ip = 1.0 / p, iq = 1.0 / q;
    double amax = 1.0;
    if (ip > amax) amax = ip;
    if (iq > amax) amax = iq;
    N2VThr thr{accept_threshold(ip, amax), accept_threshold(iq, amax), accept_threshold(1.0, amax)};
    // Lanes per walker G (4, 8 or 16; the walks do not depend on it): the walker is
    // latency-bound, so a batch that fits on the chip at 16 lanes per walker (fewer blocks of
    // proposals per step) runs at 16, one that fits at 8 at 8, a larger one at 4 (the most
    // walkers in flight). Measured at C3, 1M walks: G=4 116M, G=8 101M, G=16 79M walks/s;
    // 8,192 walks: 17M / 27M / 32M.
    // resident walkers at 16 and 8 lanes (occupancy query once per process: one GPU model)
    static const int64_t cap16 = node2vec_capacity(
        reinterpret_cast<const void *>(&k_walk_node2vec_fast<16, HASH, false>), 16);
    static const int64_t cap8 = node2vec_capacity(
        reinterpret_cast<const void *>(&k_walk_node2vec_fast<8, HASH, false>), 8);
    const int group = n_walks <= cap16 ? 16 : n_walks <= cap8 ? 8 : 4;
    const int64_t per_block = N2V_WAVES * (WAVE / group);
    int64_t blocks = (n_walks + per_block - 1) / per_block;
    if (blocks > 8192) blocks = 8192;
#define DW_N2V_LAUNCH(G, ST)                                                                   \
    hipLaunchKernelGGL((k_walk_node2vec_fast<G, HASH, ST>), dim3((unsigned)blocks),            \
                       dim3(N2V_WAVES * WAVE), 0, dw::as_stream(stream), row_ptr, col, nbr,    \
                       adj_off, adj_hash, prob_thr, alias, n_rows, starts, n_walks, walk_length, \
                       thr, k0, k1, walk_id0, out, status, counters, dw::bound_step_scalars())
    if (counters) {
        if (group == 4)
            DW_N2V_LAUNCH(4, true);
        else if (group == 8)
            DW_N2V_LAUNCH(8, true);
        else
            DW_N2V_LAUNCH(16, true);
    } else if (group == 4)
        DW_N2V_LAUNCH(4, false);
    else if (group == 8)
        DW_N2V_LAUNCH(8, false);
    else
        DW_N2V_LAUNCH(16, false);
#undef DW_N2V_LAUNCH
    DW_LAUNCH_CHECK(HASH ? "dw_walk_fast_indexed/node2vec" : "dw_walk_fast/node2vec");
    return DW_OK;
}

}  // namespace

extern "C" {

int dw_walk_replay(const int64_t *row_ptr, const int32_t *col, const int32_t *col_sorted,
                   const double *weights, int64_t n_rows, const int32_t *starts, int64_t n_walks,
                   int32_t walk_length, int32_t method, double p, double q,
                   const double *uniforms, int32_t *out, int32_t *status, void *stream) {
    DW_REQUIRE(walk_length >= 1, "dw_walk_replay: Minimum walk length is 1!");
    DW_REQUIRE(method == DW_METHOD_DEEPWALK || method == DW_METHOD_NODE2VEC,
               "dw_walk_replay: unknown method %d", method);
    DW_REQUIRE(n_walks >= 0 && n_rows >= 0, "dw_walk_replay: negative size");
    if (n_walks == 0) return DW_OK;
    DW_REQUIRE(row_ptr && col && starts && out && status, "dw_walk_replay: null pointer");
    DW_REQUIRE(walk_length == 1 || uniforms, "dw_walk_replay: uniforms is null");
    DW_REQUIRE(method == DW_METHOD_DEEPWALK || col_sorted,
               "dw_walk_replay: node2vec needs col_sorted");
    DW_REQUIRE(method == DW_METHOD_DEEPWALK || (p != 0.0 && q != 0.0),
               "dw_walk_replay: p and q must be non-zero");
    ReplayCtx c;
    c.row_ptr = row_ptr;
    c.col = col;
    c.col_sorted = col_sorted;
    c.w = weights;
    c.node2vec = method == DW_METHOD_NODE2VEC;
    c.inv_p = c.node2vec ? 1.0 / p : 1.0;  // `1 / self._p` (host IEEE division)
    c.inv_q = c.node2vec ? 1.0 / q : 1.0;
    int64_t blocks = (n_walks + REPLAY_WAVES - 1) / REPLAY_WAVES;
    if (blocks > 16384) blocks = 16384;
    // unweighted graphs take the exact picks without the serial sums (k_walk_replay_uniform,
    // node2vec_pick_exact); DW_REPLAY_SERIAL=1 keeps the serial replay everywhere (tests compare
    // the two bit for bit)
    const char *ser = getenv("DW_REPLAY_SERIAL");
    const bool serial_only = ser && ser[0] == '1';
    const bool fast = !weights && !serial_only && c.inv_p > 0.0 && c.inv_q > 0.0 &&
                      c.inv_p < 1e300 && c.inv_q < 1e300;
    if (!c.node2vec && !weights) {
        int64_t ublocks = (n_walks + 255) / 256;
        if (ublocks > 65536) ublocks = 65536;
        hipLaunchKernelGGL(k_walk_replay_uniform, dim3((unsigned)ublocks), dim3(256), 0,
                           dw::as_stream(stream), row_ptr, col, n_rows, starts, n_walks,
                           walk_length, uniforms, out, status, serial_only ? 1 : 0);
        DW_LAUNCH_CHECK("dw_walk_replay");
        return DW_OK;
    }
    if (fast)
        hipLaunchKernelGGL((k_walk_replay<REPLAY_CH_EXACT, REPLAY_NCAP_EXACT>), dim3((unsigned)blocks),
                           dim3(REPLAY_WAVES * WAVE), 0, dw::as_stream(stream), c, n_rows, starts,
                           n_walks, walk_length, uniforms, out, status, 1, N2VIndex{});
    else
        hipLaunchKernelGGL((k_walk_replay<REPLAY_CH, REPLAY_NCAP>), dim3((unsigned)blocks),
                           dim3(REPLAY_WAVES * WAVE), 0, dw::as_stream(stream), c, n_rows, starts,
                           n_walks, walk_length, uniforms, out, status, 0, N2VIndex{});
    DW_LAUNCH_CHECK("dw_walk_replay");
    return DW_OK;
}

int dw_walk_replay_indexed(const int64_t *row_ptr, const int32_t *col, const int32_t *col_sorted,
                           const int64_t *adj_off, const int32_t *adj_hash,
                           const int32_t *adj_hpos, const int32_t *hub_idx,
                           const uint32_t *hub_bits, int64_t hub_words,
                           const uint32_t *edge_cn, int64_t n_rows,
                           const int32_t *starts, int64_t n_walks, int32_t walk_length, double p,
                           double q, const double *uniforms, int32_t *out, int32_t *status,
                           uint64_t *counters, void *stream) {
    DW_REQUIRE(walk_length >= 1, "dw_walk_replay_indexed: Minimum walk length is 1!");
    DW_REQUIRE(n_walks >= 0 && n_rows >= 0, "dw_walk_replay_indexed: negative size");
    if (n_walks == 0) return DW_OK;
    DW_REQUIRE(row_ptr && col && col_sorted && adj_off && adj_hash && adj_hpos && starts && out &&
                   status,
               "dw_walk_replay_indexed: null pointer");
    DW_REQUIRE(walk_length == 1 || uniforms, "dw_walk_replay_indexed: uniforms is null");
    DW_REQUIRE(p > 0.0 && q > 0.0, "dw_walk_replay_indexed: p and q must be positive");
    ReplayCtx c;
    c.row_ptr = row_ptr;
    c.col = col;
    c.col_sorted = col_sorted;
    c.w = nullptr;
    c.node2vec = true;
    c.inv_p = 1.0 / p;   // `1 / self._p` (host IEEE division)
    c.inv_q = 1.0 / q;
    DW_REQUIRE(c.inv_p < 1e300 && c.inv_q < 1e300, "dw_walk_replay_indexed: p, q too small");
    const char *ser = getenv("DW_REPLAY_SERIAL");   // the serial arithmetic everywhere (tests)
    if (ser && ser[0] == '1' && !counters)
        return dw_walk_replay(row_ptr, col, col_sorted, nullptr, n_rows, starts, n_walks,
                              walk_length, DW_METHOD_NODE2VEC, p, q, uniforms, out, status,
                              stream);
    int64_t blocks = (n_walks + REPLAY_WAVES - 1) / REPLAY_WAVES;
    if (blocks > 16384) blocks = 16384;
    // N(prev) mapped into N(v) when deg(v) > b_factor deg(prev). With the per-edge class counts
    // a classification scans ~deg(v)/4 entries, so the mapping pays only for a much shorter
    // N(prev): 64 (C3, 65,536 walks: 14.5 ms at 16, 13.5 at 64, 13.6 at 256, 17.8 at 4);
    // without the counts 16 (scripts/gpu_n2v_cn.sh, measured with a factor override since removed)
    const int32_t b_factor = edge_cn ? 64 : 16;
    DW_REQUIRE(!hub_idx || (hub_bits && hub_words >= (n_rows + 31) / 32),
               "dw_walk_replay_indexed: hub bitmaps need hub_bits of >= ceil(n_rows / 32) words");
    const N2VIndex ix{adj_off, adj_hash, adj_hpos, b_factor,
                      reinterpret_cast<unsigned long long *>(counters), hub_idx, hub_bits,
                      hub_words, edge_cn};
    // with the counts: their own kernel (no class-mask cache: 11.25 ms against 13.45 ms through
    // the general kernel for 65,536 C3 walks; profiles/r03_replay_rates.jsonl)
    if (edge_cn)
        hipLaunchKernelGGL((k_walk_replay_cn<REPLAY_CH_CN, REPLAY_NCAP_EXACT>),
                           dim3((unsigned)blocks), dim3(REPLAY_WAVES * WAVE), 0,
                           dw::as_stream(stream), c, n_rows, starts, n_walks, walk_length,
                           uniforms, out, status, 1, ix);
    else
        hipLaunchKernelGGL((k_walk_replay<REPLAY_CH_EXACT, REPLAY_NCAP_EXACT>),
                           dim3((unsigned)blocks), dim3(REPLAY_WAVES * WAVE), 0,
                           dw::as_stream(stream), c, n_rows, starts, n_walks, walk_length,
                           uniforms, out, status, 1, ix);
    DW_LAUNCH_CHECK("dw_walk_replay_indexed");
    return DW_OK;
}

int dw_edge_common_counts(const int64_t *row_ptr, const int32_t *col, const int64_t *adj_off,
                          const int32_t *adj_hash, const int32_t *adj_hpos,
                          const int32_t *hub_idx, const uint32_t *hub_bits, int64_t hub_words,
                          int64_t n_rows, int64_t n_edges, uint32_t *edge_cn, void *stream) {
    DW_REQUIRE(n_rows >= 0 && n_edges >= 0, "dw_edge_common_counts: negative size");
    if (n_edges == 0 || n_rows == 0) return DW_OK;
    DW_REQUIRE(row_ptr && col && adj_off && adj_hash && adj_hpos && edge_cn,
               "dw_edge_common_counts: null pointer");
    DW_REQUIRE(!hub_idx || (hub_bits && hub_words >= (n_rows + 31) / 32),
               "dw_edge_common_counts: hub bitmaps need hub_bits of >= ceil(n_rows / 32) words");
    int64_t blocks = (n_edges + 255) / 256;   // a wave per 64 edges
    if (blocks > 65536) blocks = 65536;
    const EdgeIndex x{col, adj_off, adj_hash, adj_hpos, hub_idx, hub_bits, hub_words};
    hipLaunchKernelGGL(k_edge_common, dim3((unsigned)blocks), dim3(256), 0, dw::as_stream(stream),
                       x, row_ptr, n_rows, n_edges, edge_cn);
    DW_LAUNCH_CHECK("dw_edge_common_counts");
    return DW_OK;
}

int dw_n2v_edge_offsets(const int64_t *row_ptr, const int32_t *col, const uint32_t *edge_cn,
                        int64_t n_edges, int64_t *off, int64_t *byte_off, void *tmp,
                        size_t *tmp_bytes, void *stream) {
    DW_REQUIRE(n_edges >= 0 && tmp_bytes, "dw_n2v_edge_offsets: bad arguments");
    DW_REQUIRE(n_edges < (int64_t(1) << 32), "dw_n2v_edge_offsets: too many edges");
    const auto in = rocprim::make_transform_iterator(edge_cn, CnCount64{});
    const auto inb = rocprim::make_transform_iterator(rocprim::make_counting_iterator<int64_t>(0),
                                                      CnBytes{edge_cn, row_ptr, col});
    const hipStream_t st = dw::as_stream(stream);
    size_t need = 0, need_b = 0;
    if (n_edges > 0) {
        DW_WALK_HIP_OK(rocprim::inclusive_scan(nullptr, need, in, static_cast<int64_t *>(nullptr),
                                               static_cast<size_t>(n_edges),
                                               rocprim::plus<int64_t>(), st),
                       "dw_n2v_edge_offsets: scan");
        DW_WALK_HIP_OK(rocprim::inclusive_scan(nullptr, need_b, inb,
                                               static_cast<int64_t *>(nullptr),
                                               static_cast<size_t>(n_edges),
                                               rocprim::plus<int64_t>(), st),
                       "dw_n2v_edge_offsets: byte scan");
        if (need_b > need) need = need_b;
    }
    if (!tmp) {
        *tmp_bytes = need > 0 ? need : 1;
        return DW_OK;
    }
    DW_REQUIRE(*tmp_bytes >= need, "dw_n2v_edge_offsets: tmp too small");
    DW_REQUIRE(off && byte_off && (n_edges == 0 || (edge_cn && row_ptr && col)),
               "dw_n2v_edge_offsets: null pointer");
    DW_WALK_HIP_OK(hipMemsetAsync(off, 0, sizeof(int64_t), st), "dw_n2v_edge_offsets: memset");
    DW_WALK_HIP_OK(hipMemsetAsync(byte_off, 0, sizeof(int64_t), st),
                   "dw_n2v_edge_offsets: memset");
    if (n_edges > 0) {
        DW_WALK_HIP_OK(rocprim::inclusive_scan(tmp, need, in, off + 1,
                                               static_cast<size_t>(n_edges),
                                               rocprim::plus<int64_t>(), st),
                       "dw_n2v_edge_offsets: scan");
        DW_WALK_HIP_OK(rocprim::inclusive_scan(tmp, need, inb, byte_off + 1,
                                               static_cast<size_t>(n_edges),
                                               rocprim::plus<int64_t>(), st),
                       "dw_n2v_edge_offsets: byte scan");
    }
    return DW_OK;
}

namespace {
struct MinusBase {   // a chunk's segment offsets relative to its first entry
    int64_t base;
    __host__ __device__ __forceinline__ int64_t operator()(int64_t o) const { return o - base; }
};
}  // namespace

int dw_n2v_edge_index_build(const int64_t *row_ptr, const int32_t *col, const int64_t *adj_off,
                            const int32_t *adj_hash, const int32_t *adj_hpos,
                            const int32_t *hub_idx, const uint32_t *hub_bits, int64_t hub_words,
                            const uint32_t *edge_cn, const int64_t *off, const int64_t *byte_off,
                            int64_t n_rows, int64_t n_edges, int64_t e_begin, int64_t e_end,
                            int64_t base, int64_t n_chunk_pos, uint8_t *pos, int32_t *scratch,
                            int32_t *pos_t, void *tmp, size_t *tmp_bytes, int32_t *status,
                            void *stream) {
    DW_REQUIRE(n_rows >= 0 && n_edges >= 0 && tmp_bytes && 0 <= e_begin && e_begin <= e_end &&
                   e_end <= n_edges && n_chunk_pos >= 0,
               "dw_n2v_edge_index_build: bad arguments");
    DW_REQUIRE(n_edges < (int64_t(1) << 31) && n_chunk_pos < (int64_t(1) << 31),
               "dw_n2v_edge_index_build: a chunk of < 2^31 entries (and edges) per call");
    const hipStream_t st = dw::as_stream(stream);
    uint32_t end_bit = 1;
    while (end_bit < 31 && (int64_t(1) << end_bit) < n_rows) ++end_bit;   // positions < deg <= V
    const int64_t n_seg = e_end - e_begin;
    size_t sort_bytes = 0;
    const auto sb = rocprim::make_transform_iterator(off + e_begin, MinusBase{base});
    const auto se = rocprim::make_transform_iterator(off + e_begin + 1, MinusBase{base});
    if (n_chunk_pos > 0)
        DW_WALK_HIP_OK(rocprim::segmented_radix_sort_keys(
                           nullptr, sort_bytes, static_cast<const int32_t *>(nullptr),
                           static_cast<int32_t *>(nullptr), static_cast<unsigned>(n_chunk_pos),
                           static_cast<unsigned>(n_seg > 0 ? n_seg : 1), sb, se, 0, end_bit, st),
                       "dw_n2v_edge_index_build: sort");
    // tmp: the unsorted positions (n_chunk_pos int32), then the segmented sort's storage
    const size_t un_bytes = ((static_cast<size_t>(n_chunk_pos) * 4 + 255) / 256) * 256;
    if (!tmp) {
        *tmp_bytes = un_bytes + sort_bytes + 256;
        return DW_OK;
    }
    DW_REQUIRE(*tmp_bytes >= un_bytes + sort_bytes, "dw_n2v_edge_index_build: tmp too small");
    if (n_seg == 0 || n_rows == 0) return DW_OK;
    DW_REQUIRE(row_ptr && col && adj_off && adj_hash && adj_hpos && edge_cn && off && byte_off &&
                   pos_t && status && (n_chunk_pos == 0 || (pos && scratch)),
               "dw_n2v_edge_index_build: null pointer");
    DW_REQUIRE(!hub_idx || (hub_bits && hub_words >= (n_rows + 31) / 32),
               "dw_n2v_edge_index_build: hub bitmaps need hub_bits of >= ceil(n_rows / 32) words");
    int32_t *unsorted = static_cast<int32_t *>(tmp);
    int64_t blocks = (n_seg + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    const EdgeIndex x{col, adj_off, adj_hash, adj_hpos, hub_idx, hub_bits, hub_words};
    hipLaunchKernelGGL(k_edge_cn_positions, dim3((unsigned)blocks), dim3(256), 0, st, x, row_ptr,
                       n_rows, e_begin, e_end, edge_cn, off, base, unsorted, pos_t, status);
    DW_LAUNCH_CHECK("dw_n2v_edge_index_build/positions");
    if (n_chunk_pos > 0) {
        DW_WALK_HIP_OK(rocprim::segmented_radix_sort_keys(
                           static_cast<char *>(tmp) + un_bytes, sort_bytes,
                           static_cast<const int32_t *>(unsorted), scratch,
                           static_cast<unsigned>(n_chunk_pos), static_cast<unsigned>(n_seg), sb,
                           se, 0, end_bit, st),
                       "dw_n2v_edge_index_build: sort");
        hipLaunchKernelGGL(k_n2v_pos_compact, dim3((unsigned)blocks), dim3(256), 0, st, row_ptr,
                           col, e_begin, e_end, off, base, byte_off, scratch, pos);
        DW_LAUNCH_CHECK("dw_n2v_edge_index_build/compact");
    }
    return DW_OK;
}

int dw_n2v_edge_records(const int64_t *row_ptr, const int32_t *col, const uint32_t *edge_cn,
                        const int64_t *byte_off, const int32_t *pos_t, int64_t n_edges,
                        int32_t *rec, void *stream) {
    DW_REQUIRE(n_edges >= 0, "dw_n2v_edge_records: bad size");
    if (n_edges == 0) return DW_OK;
    DW_REQUIRE(row_ptr && col && edge_cn && byte_off && pos_t && rec,
               "dw_n2v_edge_records: null pointer");
    int64_t blocks = (n_edges + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_n2v_edge_records, dim3((unsigned)blocks), dim3(256), 0,
                       dw::as_stream(stream), row_ptr, col, edge_cn, byte_off, pos_t, n_edges,
                       reinterpret_cast<int4 *>(rec));
    DW_LAUNCH_CHECK("dw_n2v_edge_records");
    return DW_OK;
}

int dw_walk_replay_positions(const int64_t *row_ptr, const int32_t *n2v_rec,
                             const uint8_t *n2v_pos, int64_t n_rows, const int32_t *starts,
                             int64_t n_walks, int32_t walk_length, double p, double q,
                             const double *uniforms, int32_t *out, int32_t *status,
                             uint64_t *counters, void *stream) {
    DW_REQUIRE(walk_length >= 1, "dw_walk_replay_positions: Minimum walk length is 1!");
    DW_REQUIRE(n_walks >= 0 && n_rows >= 0, "dw_walk_replay_positions: negative size");
    if (n_walks == 0) return DW_OK;
    DW_REQUIRE(row_ptr && n2v_rec && n2v_pos && starts && out && status,
               "dw_walk_replay_positions: null pointer");
    DW_REQUIRE(walk_length == 1 || uniforms, "dw_walk_replay_positions: uniforms is null");
    DW_REQUIRE(p > 0.0 && q > 0.0, "dw_walk_replay_positions: p and q must be positive");
    const double ip = 1.0 / p, iq = 1.0 / q;   // `1 / self._p` (host IEEE division)
    DW_REQUIRE(ip < 1e300 && iq < 1e300, "dw_walk_replay_positions: p, q too small");
    const hipStream_t st = dw::as_stream(stream);
    int64_t blocks = (n_walks + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    auto *cnt = reinterpret_cast<unsigned long long *>(counters);
    if (counters)
        hipLaunchKernelGGL(k_walk_replay_n2v_pos<true>, dim3((unsigned)blocks), dim3(256), 0, st,
                           row_ptr, reinterpret_cast<const int4 *>(n2v_rec), n2v_pos, n_rows,
                           starts, n_walks, walk_length, uniforms, ip, iq, out, status, cnt);
    else
        hipLaunchKernelGGL(k_walk_replay_n2v_pos<false>, dim3((unsigned)blocks), dim3(256), 0, st,
                           row_ptr, reinterpret_cast<const int4 *>(n2v_rec), n2v_pos, n_rows,
                           starts, n_walks, walk_length, uniforms, ip, iq, out, status, cnt);
    DW_LAUNCH_CHECK("dw_walk_replay_positions");
    return DW_OK;
}

int dw_hub_bitmaps(const int64_t *row_ptr, const int32_t *col, int64_t n_rows,
                   const int32_t *hub_rows, int64_t n_hubs, int64_t hub_words, uint32_t *bits,
                   void *stream) {
    DW_REQUIRE(n_hubs >= 0 && n_rows >= 0, "dw_hub_bitmaps: negative size");
    if (n_hubs == 0) return DW_OK;
    DW_REQUIRE(row_ptr && col && hub_rows && bits, "dw_hub_bitmaps: null pointer");
    DW_REQUIRE(hub_words >= (n_rows + 31) / 32, "dw_hub_bitmaps: hub_words too small");
    DW_REQUIRE(n_hubs < (int64_t(1) << 31), "dw_hub_bitmaps: too many hubs");
    hipError_t e = hipMemsetAsync(bits, 0, (size_t)n_hubs * hub_words * sizeof(uint32_t),
                                  dw::as_stream(stream));
    if (e != hipSuccess) {
        dw::set_error("dw_hub_bitmaps: memset: %s", hipGetErrorString(e));
        return DW_E_HIP;
    }
    hipLaunchKernelGGL(k_hub_bitmaps, dim3((unsigned)n_hubs), dim3(256), 0, dw::as_stream(stream),
                       row_ptr, col, hub_rows, hub_words, bits);
    DW_LAUNCH_CHECK("dw_hub_bitmaps");
    return DW_OK;
}

int dw_walk_replay_inline(const int64_t *row_ptr, const int32_t *edges, int64_t n_rows,
                          const int32_t *starts, int64_t n_walks, int32_t walk_length,
                          const double *uniforms, int32_t *out, int32_t *status, void *stream) {
    DW_REQUIRE(walk_length >= 1, "dw_walk_replay_inline: walk_length must be >= 1");
    DW_REQUIRE(n_walks >= 0 && n_rows >= 0, "dw_walk_replay_inline: negative size");
    if (n_walks == 0) return DW_OK;
    DW_REQUIRE(row_ptr && edges && starts && out && status,
               "dw_walk_replay_inline: null pointer");
    DW_REQUIRE(walk_length == 1 || uniforms, "dw_walk_replay_inline: uniforms is null");
    const char *ser = getenv("DW_REPLAY_SERIAL");
    const bool serial_only = ser && ser[0] == '1';
    int64_t blocks = (n_walks + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_walk_replay_uniform_inline, dim3((unsigned)blocks), dim3(256), 0,
                       dw::as_stream(stream), row_ptr, reinterpret_cast<const int4 *>(edges),
                       n_rows, starts, n_walks, walk_length, uniforms, out, status,
                       serial_only ? 1 : 0);
    DW_LAUNCH_CHECK("dw_walk_replay_inline");
    return DW_OK;
}

int dw_walk_fast(const int64_t *row_ptr, const int32_t *col, const int32_t *col_sorted,
                 const uint32_t *prob_thr, const int32_t *alias, int64_t n_rows,
                 const int32_t *starts, int64_t n_walks, int32_t walk_length, int32_t method,
                 double p, double q, uint64_t seed, uint64_t walk_id0, int32_t *out,
                 int32_t *status, void *stream) {
    DW_REQUIRE(walk_length >= 1, "dw_walk_fast: Minimum walk length is 1!");
    DW_REQUIRE(walk_length < (1 << 24), "dw_walk_fast: walk_length too large");
    DW_REQUIRE(method == DW_METHOD_DEEPWALK || method == DW_METHOD_NODE2VEC,
               "dw_walk_fast: unknown method %d", method);
    DW_REQUIRE(n_walks >= 0 && n_rows >= 0, "dw_walk_fast: negative size");
    if (n_walks == 0) return DW_OK;
    DW_REQUIRE(row_ptr && col && starts && out && status, "dw_walk_fast: null pointer");
    DW_REQUIRE((prob_thr == nullptr) == (alias == nullptr),
               "dw_walk_fast: prob_thr and alias must be both set or both null");
    const uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
    if (method == DW_METHOD_DEEPWALK) {
        const int64_t blocks = (n_walks + 255) / 256;
        DW_REQUIRE(blocks < (int64_t(1) << 31), "dw_walk_fast: too many walks");
        hipLaunchKernelGGL(k_walk_deepwalk_fast, dim3((unsigned)blocks), dim3(256), 0,
                           dw::as_stream(stream), row_ptr, col, prob_thr, alias, n_rows, starts,
                           n_walks, walk_length, k0, k1, walk_id0, out, status,
                           dw::bound_step_scalars());
        DW_LAUNCH_CHECK("dw_walk_fast/deepwalk");
        return DW_OK;
    }
    DW_REQUIRE(col_sorted, "dw_walk_fast: node2vec needs col_sorted");
    return launch_node2vec<false>(row_ptr, col, col_sorted, nullptr, nullptr, prob_thr, alias,
                                  n_rows, starts, n_walks, walk_length, p, q, k0, k1, walk_id0,
                                  out, status, stream);
}

int dw_walk_fast_indexed(const int64_t *row_ptr, const int32_t *col, const int32_t *edges,
                         const int64_t *adj_off, const int32_t *adj_hash,
                         const uint32_t *prob_thr, const int32_t *alias, int64_t n_rows,
                         const int32_t *starts, int64_t n_walks, int32_t walk_length,
                         int32_t method, double p, double q, uint64_t seed, uint64_t walk_id0,
                         int32_t *out, int32_t *status, void *stream) {
    DW_REQUIRE(walk_length >= 1 && walk_length < (1 << 24),
               "dw_walk_fast_indexed: walk_length must be in [1, 2^24)");
    DW_REQUIRE(method == DW_METHOD_DEEPWALK || method == DW_METHOD_NODE2VEC,
               "dw_walk_fast_indexed: unknown method %d", method);
    DW_REQUIRE(n_walks >= 0 && n_rows >= 0, "dw_walk_fast_indexed: negative size");
    if (n_walks == 0) return DW_OK;
    DW_REQUIRE(row_ptr && starts && out && status, "dw_walk_fast_indexed: null pointer");
    DW_REQUIRE((prob_thr == nullptr) == (alias == nullptr),
               "dw_walk_fast_indexed: prob_thr and alias must be both set or both null");
    const uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
    if (method == DW_METHOD_DEEPWALK) {
        DW_REQUIRE(edges, "dw_walk_fast_indexed: DeepWalk needs edges (dw_edges_inline_build)");
        const int64_t blocks = (n_walks + 255) / 256;
        DW_REQUIRE(blocks < (int64_t(1) << 31), "dw_walk_fast_indexed: too many walks");
        hipLaunchKernelGGL(k_walk_deepwalk_inline, dim3((unsigned)blocks), dim3(256), 0,
                           dw::as_stream(stream), row_ptr, reinterpret_cast<const int4 *>(edges),
                           prob_thr, alias, n_rows, starts, n_walks, walk_length, k0, k1,
                           walk_id0, out, status, dw::bound_step_scalars());
        DW_LAUNCH_CHECK("dw_walk_fast_indexed/deepwalk");
        return DW_OK;
    }
    DW_REQUIRE(col && adj_off && adj_hash,
               "dw_walk_fast_indexed: node2vec needs col, adj_off and adj_hash");
    return launch_node2vec<true>(row_ptr, col, col, adj_off, adj_hash, prob_thr, alias, n_rows,
                                 starts, n_walks, walk_length, p, q, k0, k1, walk_id0, out,
                                 status, stream);
}

int dw_walk_fast_counted(const int64_t *row_ptr, const int32_t *col, const int64_t *adj_off,
                         const int32_t *adj_hash, const uint32_t *prob_thr, const int32_t *alias,
                         int64_t n_rows, const int32_t *starts, int64_t n_walks,
                         int32_t walk_length, double p, double q, uint64_t seed,
                         uint64_t walk_id0, int32_t *out, int32_t *status,
                         uint64_t *counters, void *stream) {
    DW_REQUIRE(walk_length >= 1 && walk_length < (1 << 24),
               "dw_walk_fast_counted: walk_length must be in [1, 2^24)");
    DW_REQUIRE(n_walks >= 0 && n_rows >= 0, "dw_walk_fast_counted: negative size");
    if (n_walks == 0) return DW_OK;
    DW_REQUIRE(row_ptr && col && adj_off && adj_hash && starts && out && status && counters,
               "dw_walk_fast_counted: null pointer");
    DW_REQUIRE((prob_thr == nullptr) == (alias == nullptr),
               "dw_walk_fast_counted: prob_thr and alias must be both set or both null");
    const uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
    return launch_node2vec<true>(row_ptr, col, col, adj_off, adj_hash, prob_thr, alias, n_rows,
                                 starts, n_walks, walk_length, p, q, k0, k1, walk_id0, out,
                                 status, stream,
                                 reinterpret_cast<unsigned long long *>(counters));
}

int dw_walk_fast_positions(const int64_t *row_ptr, const int32_t *n2v_rec, const uint8_t *n2v_pos,
                           int64_t n_rows, const int32_t *starts, int64_t n_walks,
                           int32_t walk_length, double p, double q, uint64_t seed,
                           uint64_t walk_id0, int32_t *out, int32_t *status, uint64_t *counters,
                           void *stream) {
    DW_REQUIRE(walk_length >= 1 && walk_length < (1 << 24),
               "dw_walk_fast_positions: walk_length must be in [1, 2^24)");
    DW_REQUIRE(n_walks >= 0 && n_rows >= 0, "dw_walk_fast_positions: negative size");
    if (n_walks == 0) return DW_OK;
    DW_REQUIRE(row_ptr && n2v_rec && starts && out && status,
               "dw_walk_fast_positions: null pointer");
    DW_REQUIRE(p > 0.0 && q > 0.0, "dw_walk_fast_positions: p and q must be positive");
    const double ip = 1.0 / p, iq = 1.0 / q;
    DW_REQUIRE(ip < 1e300 && iq < 1e300, "dw_walk_fast_positions: p, q too small");
    const uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
    const int64_t blocks = (n_walks + 255) / 256;
    DW_REQUIRE(blocks < (int64_t(1) << 31), "dw_walk_fast_positions: too many walks");
    auto *cnt = reinterpret_cast<unsigned long long *>(counters);
    if (cnt)
        hipLaunchKernelGGL(k_walk_node2vec_positions<true>, dim3((unsigned)blocks), dim3(256), 0,
                           dw::as_stream(stream), row_ptr, reinterpret_cast<const int4 *>(n2v_rec),
                           n2v_pos, n_rows, starts, n_walks, walk_length, ip, iq, k0, k1, walk_id0,
                           out, status, dw::bound_step_scalars(), cnt);
    else
        hipLaunchKernelGGL(k_walk_node2vec_positions<false>, dim3((unsigned)blocks), dim3(256), 0,
                           dw::as_stream(stream), row_ptr, reinterpret_cast<const int4 *>(n2v_rec),
                           n2v_pos, n_rows, starts, n_walks, walk_length, ip, iq, k0, k1, walk_id0,
                           out, status, dw::bound_step_scalars(), cnt);
    DW_LAUNCH_CHECK("dw_walk_fast_positions");
    return DW_OK;
}

int dw_step_starts(const dw_step_scalars *dev, const int32_t *epoch_starts, int64_t n_epoch,
                   int32_t *starts_out, int64_t n, void *stream) {
    DW_REQUIRE(n >= 0 && n_epoch >= 1, "dw_step_starts: bad sizes");
    if (n == 0) return DW_OK;
    DW_REQUIRE(dev && epoch_starts && starts_out, "dw_step_starts: null pointer");
    int64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_step_starts, dim3((unsigned)blocks), dim3(256), 0, dw::as_stream(stream),
                       dev, epoch_starts, n_epoch, starts_out, n);
    DW_LAUNCH_CHECK("dw_step_starts");
    return DW_OK;
}

int dw_step_scalars_advance(dw_step_scalars *dev, const float *hist, int64_t hist_rows,
                            uint64_t walks_per_step, uint64_t centres_per_step, int32_t *status,
                            const int32_t *epoch_starts, int64_t n_epoch, int32_t *starts_out,
                            int64_t n, void *stream) {
    DW_REQUIRE(dev && hist && status && hist_rows >= 1, "dw_step_scalars_advance: bad arguments");
    DW_REQUIRE(!epoch_starts || (starts_out && n_epoch >= 1 && n >= 0),
               "dw_step_scalars_advance: bad start-node arguments");
    hipLaunchKernelGGL(k_step_advance, dim3(1), dim3(256), 0, dw::as_stream(stream), dev, hist,
                       hist_rows, walks_per_step, centres_per_step, status, epoch_starts, n_epoch,
                       starts_out, n);
    DW_LAUNCH_CHECK("dw_step_scalars_advance");
    return DW_OK;
}

int dw_step_scalars_expand(dw_step_scalars *base, dw_step_scalars *steps, int64_t n_steps,
                           const float *hist, int64_t hist_rows, uint64_t walks_per_step,
                           uint64_t centres_per_step, int32_t *status,
                           const int32_t *epoch_starts, int64_t n_epoch, int32_t *starts_out,
                           int64_t n, void *stream) {
    DW_REQUIRE(base && steps && hist && status && hist_rows >= 1 && n_steps >= 1 &&
                   n_steps <= 4096,
               "dw_step_scalars_expand: bad arguments");
    DW_REQUIRE(!epoch_starts || (starts_out && n_epoch >= 1 && n >= 0),
               "dw_step_scalars_expand: bad start-node arguments");
    hipLaunchKernelGGL(k_step_expand, dim3(1), dim3(256), 0, dw::as_stream(stream), base, steps,
                       n_steps, hist, hist_rows, walks_per_step, centres_per_step, status,
                       epoch_starts, n_epoch, starts_out, n);
    DW_LAUNCH_CHECK("dw_step_scalars_expand");
    return DW_OK;
}

int dw_edges_inline_build(const int64_t *row_ptr, const int32_t *col, int64_t n_rows, int64_t nnz,
                          int32_t *edges, void *stream) {
    DW_REQUIRE(n_rows >= 0 && nnz >= 0, "dw_edges_inline_build: negative size");
    if (nnz == 0) return DW_OK;
    DW_REQUIRE(row_ptr && col && edges, "dw_edges_inline_build: null pointer");
    int64_t blocks = (nnz + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_edges_inline, dim3((unsigned)blocks), dim3(256), 0, dw::as_stream(stream),
                       row_ptr, col, nnz, reinterpret_cast<int4 *>(edges));
    DW_LAUNCH_CHECK("dw_edges_inline_build");
    return DW_OK;
}

}  // extern "C"
