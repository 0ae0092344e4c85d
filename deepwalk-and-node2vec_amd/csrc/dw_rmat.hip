// Graph ingestion on gfx950: R-MAT edge lists and CSR built in HBM.
//
// Follows the generator spec of shallow_encoders/graph/rmat.py bit for bit:
//   * the uniforms are numpy's default_rng(seed).random() stream — PCG64 (128-bit LCG,
//     XSL-RR output, double = (x >> 11) * 2^-53) — level-major: draw l * n_edges + e is the
//     level-l uniform of edge e. The host hands over the 128-bit state before each level's
//     first draw and a 2^i jump table, so every thread jumps straight to its edges;
//   * src |= (r >= a+b), dst |= (a <= r < a+b) | (r >= a+b+c) at bit (scale-1-level);
//   * self-loops dropped, undirected duplicates removed keeping the FIRST draw (stable radix
//     sort of (min, max) keys carrying the draw index, the first of every run kept, then a
//     stream compaction in draw order);
//   * isolated nodes listed in increasing order (the host draws their patch edges from the
//     same numpy stream, advanced past the edge draws);
//   * CSR rows in edge-list order — what networkx's add_edges_from gives: each edge (u, v)
//     contributes u->v then v->u, stably sorted by source; column ids are vocabulary ids
//     (node + 1), row 0 is <unk>.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "dw_common.h"

namespace {

struct U128 {
    uint64_t lo, hi;
};

__device__ __forceinline__ U128 mul128(U128 a, U128 b) {
    return U128{a.lo * b.lo, __umul64hi(a.lo, b.lo) + a.lo * b.hi + a.hi * b.lo};
}

__device__ __forceinline__ U128 add128(U128 a, U128 b) {
    const uint64_t lo = a.lo + b.lo;
    return U128{lo, a.hi + b.hi + (lo < a.lo ? 1ull : 0ull)};
}

constexpr uint64_t PCG_MULT_LO = 0x4385DF649FCCF645ull;  // 0x2360ED051FC65DA4_4385DF649FCCF645
constexpr uint64_t PCG_MULT_HI = 0x2360ED051FC65DA4ull;

// numpy PCG64: state = state * M + inc, then the XSL-RR output of the NEW state.
__device__ __forceinline__ double pcg64_next_double(U128 &s, U128 inc) {
    s = add128(mul128(s, U128{PCG_MULT_LO, PCG_MULT_HI}), inc);
    const uint64_t x = s.hi ^ s.lo;
    const unsigned r = static_cast<unsigned>(s.hi >> 58);
    const uint64_t out = (x >> r) | (x << ((64u - r) & 63u));
    return static_cast<double>(out >> 11) * 0x1.0p-53;
}

constexpr int RMAT_EDGES_PER_THREAD = 16;

// One thread = RMAT_EDGES_PER_THREAD consecutive edges, all levels; per level one jump from
// the level's base state (<= log2(n_edges) table steps) then sequential draws.
__global__ void __launch_bounds__(256)
    k_rmat_draw(int32_t scale, int64_t n, const uint64_t *__restrict__ level_state,
                const uint64_t *__restrict__ jump, U128 inc, double t1, double t2, double t3,
                uint64_t *__restrict__ edges) {
    const int64_t e0 =
        (blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x) * RMAT_EDGES_PER_THREAD;
    if (e0 >= n) return;
    uint32_t src[RMAT_EDGES_PER_THREAD], dst[RMAT_EDGES_PER_THREAD];
#pragma unroll
    for (int j = 0; j < RMAT_EDGES_PER_THREAD; ++j) src[j] = dst[j] = 0u;
    for (int l = 0; l < scale; ++l) {
        U128 s{level_state[2 * l], level_state[2 * l + 1]};
        uint64_t k = static_cast<uint64_t>(e0);
        for (int i = 0; k != 0; ++i, k >>= 1)
            if (k & 1ull)
                s = add128(mul128(s, U128{jump[4 * i], jump[4 * i + 1]}),
                           U128{jump[4 * i + 2], jump[4 * i + 3]});
        const uint32_t bit = 1u << (scale - 1 - l);
#pragma unroll
        for (int j = 0; j < RMAT_EDGES_PER_THREAD; ++j) {
            if (e0 + j < n) {
                const double r = pcg64_next_double(s, inc);
                if (r >= t2) src[j] |= bit;
                if ((r >= t1 && r < t2) || r >= t3) dst[j] |= bit;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < RMAT_EDGES_PER_THREAD; ++j)
        if (e0 + j < n) edges[e0 + j] = (static_cast<uint64_t>(src[j]) << 32) | dst[j];
}

__global__ void __launch_bounds__(256)
    k_rmat_keys(const uint64_t *__restrict__ edges, int64_t n, int32_t scale,
                uint64_t *__restrict__ keys, uint32_t *__restrict__ idx) {
    const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
    if (i >= n) return;
    const uint64_t e = edges[i];
    const uint64_t u = e >> 32, v = e & 0xFFFFFFFFull;
    keys[i] = u == v ? (1ull << (2 * scale))  // self-loop: sorts last, never kept
                     : ((u < v ? u : v) << scale) | (u < v ? v : u);
    idx[i] = static_cast<uint32_t>(i);
}

// keep[draw] = 1 for the first draw of every distinct undirected edge (runs of equal keys are
// in draw order: the radix sort is stable).
__global__ void __launch_bounds__(256)
    k_rmat_first(const uint64_t *__restrict__ keys, const uint32_t *__restrict__ idx, int64_t n,
                 uint64_t invalid, uint8_t *__restrict__ keep) {
    const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = keys[i];
    keep[idx[i]] = (k != invalid && (i == 0 || keys[i - 1] != k)) ? 1 : 0;
}

__global__ void __launch_bounds__(256)
    k_endpoint_degree(const uint64_t *__restrict__ edges, int64_t m, int64_t n_nodes,
                      uint32_t *__restrict__ deg, int32_t *status) {
    const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
    if (i >= m) return;
    const uint64_t e = edges[i];
    const uint64_t u = e >> 32, v = e & 0xFFFFFFFFull;
    if (u >= static_cast<uint64_t>(n_nodes) || v >= static_cast<uint64_t>(n_nodes)) {
        dw::status_or(status, DW_S_BAD_CSR);
        return;
    }
    atomicAdd(deg + u, 1u);
    atomicAdd(deg + v, 1u);
}

__global__ void __launch_bounds__(256)
    k_zero_flags(const uint32_t *__restrict__ deg, int64_t n, uint8_t *__restrict__ flag) {
    const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
    if (i < n) flag[i] = deg[i] == 0u ? 1 : 0;
}

// Directed CSR entries: edge i -> (u -> v+1) at 2i and (v -> u+1) at 2i+1.
__global__ void __launch_bounds__(256)
    k_csr_entries(const uint64_t *__restrict__ edges, int64_t m, uint32_t *__restrict__ keys,
                  uint32_t *__restrict__ vals) {
    const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
    if (i >= m) return;
    const uint64_t e = edges[i];
    const uint32_t u = static_cast<uint32_t>(e >> 32), v = static_cast<uint32_t>(e);
    keys[2 * i] = u;
    vals[2 * i] = v + 1u;
    keys[2 * i + 1] = v;
    vals[2 * i + 1] = u + 1u;
}

__global__ void k_row_ptr_head(int64_t *row_ptr) {
    row_ptr[0] = 0;
    row_ptr[1] = 0;
}

inline size_t a256(size_t x) { return (x + 255) & ~size_t(255); }

int bits_for(int64_t n) {  // bits of values < n
    int b = 1;
    while (b < 63 && (static_cast<uint64_t>(n - 1) >> b) != 0) ++b;
    return b;
}

inline unsigned grid_of(int64_t n) { return static_cast<unsigned>((n + 255) / 256); }

#define DW_HIP_OK(expr, what)                                                       \
    do {                                                                            \
        hipError_t e_ = (expr);                                                     \
        if (e_ != hipSuccess) {                                                     \
            ::dw::set_error("%s: %s", what, hipGetErrorString(e_));                 \
            return DW_E_HIP;                                                        \
        }                                                                           \
    } while (0)

// ---- workspace plans (one size serves the three calls) ----------------------------------------
struct RmatPlan {
    size_t raw, keys0, keys1, idx0, idx1, keep, sort_tmp, sel_tmp, total;
};

int plan_rmat(int32_t scale, int64_t n, RmatPlan *p) {
    size_t sort_tmp = 0, sel_tmp = 0;
    rocprim::double_buffer<uint64_t> kb(nullptr, nullptr);
    rocprim::double_buffer<uint32_t> vb(nullptr, nullptr);
    DW_HIP_OK(rocprim::radix_sort_pairs(nullptr, sort_tmp, kb, vb, static_cast<uint32_t>(n), 0,
                                        2 * scale + 1),
              "dw_rmat: sort size query");
    DW_HIP_OK(rocprim::select(nullptr, sel_tmp, static_cast<const uint64_t *>(nullptr),
                              static_cast<const uint8_t *>(nullptr),
                              static_cast<uint64_t *>(nullptr), static_cast<int64_t *>(nullptr),
                              static_cast<size_t>(n)),
              "dw_rmat: select size query");
    size_t off = 0;
    p->raw = off;   off += a256(n * 8);
    p->keys0 = off; off += a256(n * 8);
    p->keys1 = off; off += a256(n * 8);
    p->idx0 = off;  off += a256(n * 4);
    p->idx1 = off;  off += a256(n * 4);
    p->keep = off;  off += a256(n);
    p->sort_tmp = off; off += a256(sort_tmp);
    p->sel_tmp = off;  off += a256(sel_tmp);
    p->total = off;
    return DW_OK;
}

struct CsrPlan {
    size_t keys0, keys1, vals0, vals1, deg, flags, sort_tmp, scan_tmp, sel_tmp, total;
};

int plan_csr(int64_t m, int64_t n_nodes, CsrPlan *p) {
    const int64_t nnz = 2 * m;
    size_t sort_tmp = 0, scan_tmp = 0, sel_tmp = 0;
    rocprim::double_buffer<uint32_t> kb(nullptr, nullptr), vb(nullptr, nullptr);
    DW_HIP_OK(rocprim::radix_sort_pairs(nullptr, sort_tmp, kb, vb,
                                        static_cast<uint32_t>(nnz > 0 ? nnz : 1), 0,
                                        bits_for(n_nodes)),
              "dw_csr_from_edges: sort size query");
    DW_HIP_OK(rocprim::inclusive_scan(nullptr, scan_tmp, static_cast<const uint32_t *>(nullptr),
                                      static_cast<int64_t *>(nullptr),
                                      static_cast<size_t>(n_nodes), rocprim::plus<int64_t>()),
              "dw_csr_from_edges: scan size query");
    DW_HIP_OK(rocprim::select(nullptr, sel_tmp, rocprim::counting_iterator<int32_t>(0),
                              static_cast<const uint8_t *>(nullptr),
                              static_cast<int32_t *>(nullptr), static_cast<int64_t *>(nullptr),
                              static_cast<size_t>(n_nodes)),
              "dw_graph_isolated: select size query");
    size_t off = 0;
    p->keys0 = off; off += a256(nnz * 4);
    p->keys1 = off; off += a256(nnz * 4);
    p->vals0 = off; off += a256(nnz * 4);
    p->vals1 = off; off += a256(nnz * 4);
    p->deg = off;   off += a256(n_nodes * 4);
    p->flags = off; off += a256(n_nodes);
    p->sort_tmp = off; off += a256(sort_tmp);
    p->scan_tmp = off; off += a256(scan_tmp);
    p->sel_tmp = off;  off += a256(sel_tmp);
    p->total = off;
    return DW_OK;
}

}  // namespace

extern "C" {

int dw_ingest_workspace_bytes(int32_t scale, int64_t n_edges, int64_t n_nodes, size_t *bytes) {
    DW_REQUIRE(bytes && scale >= 1 && scale <= 31 && n_edges >= 0 && n_nodes >= 1,
               "dw_ingest_workspace_bytes: bad arguments");
    DW_REQUIRE(n_edges < (int64_t(1) << 31) && n_nodes < (int64_t(1) << 31),
               "dw_ingest_workspace_bytes: sizes must fit int32");
    RmatPlan r;
    CsrPlan c;
    int rc = plan_rmat(scale, n_edges > 0 ? n_edges : 1, &r);
    if (rc != DW_OK) return rc;
    rc = plan_csr(n_edges > 0 ? n_edges : 1, n_nodes, &c);
    if (rc != DW_OK) return rc;
    *bytes = r.total > c.total ? r.total : c.total;
    return DW_OK;
}

int dw_rmat_edges(int32_t scale, int64_t n_edges, const uint64_t *level_state,
                  const uint64_t *jump, uint64_t inc_lo, uint64_t inc_hi, double t1, double t2,
                  double t3, uint64_t *edges, int64_t *n_unique, void *workspace,
                  size_t workspace_bytes, void *stream) {
    DW_REQUIRE(scale >= 1 && scale <= 31 && n_edges >= 1 && n_edges < (int64_t(1) << 31),
               "dw_rmat_edges: bad sizes");
    DW_REQUIRE(level_state && jump && edges && n_unique && workspace,
               "dw_rmat_edges: null pointer");
    RmatPlan p;
    int rc = plan_rmat(scale, n_edges, &p);
    if (rc != DW_OK) return rc;
    DW_REQUIRE(workspace_bytes >= p.total, "dw_rmat_edges: workspace too small (%zu < %zu)",
               workspace_bytes, p.total);
    hipStream_t st = dw::as_stream(stream);
    char *w = static_cast<char *>(workspace);
    uint64_t *raw = reinterpret_cast<uint64_t *>(w + p.raw);
    const int64_t n_threads = (n_edges + RMAT_EDGES_PER_THREAD - 1) / RMAT_EDGES_PER_THREAD;
    hipLaunchKernelGGL(k_rmat_draw, dim3(grid_of(n_threads)), dim3(256), 0, st, scale, n_edges,
                       level_state, jump, U128{inc_lo, inc_hi}, t1, t2, t3, raw);
    DW_LAUNCH_CHECK("dw_rmat_edges/draw");
    uint64_t *k0 = reinterpret_cast<uint64_t *>(w + p.keys0);
    uint64_t *k1 = reinterpret_cast<uint64_t *>(w + p.keys1);
    uint32_t *i0 = reinterpret_cast<uint32_t *>(w + p.idx0);
    uint32_t *i1 = reinterpret_cast<uint32_t *>(w + p.idx1);
    uint8_t *keep = reinterpret_cast<uint8_t *>(w + p.keep);
    hipLaunchKernelGGL(k_rmat_keys, dim3(grid_of(n_edges)), dim3(256), 0, st, raw, n_edges,
                       scale, k0, i0);
    DW_LAUNCH_CHECK("dw_rmat_edges/keys");
    rocprim::double_buffer<uint64_t> kb(k0, k1);
    rocprim::double_buffer<uint32_t> vb(i0, i1);
    size_t sort_tmp = p.sel_tmp - p.sort_tmp;
    DW_HIP_OK(rocprim::radix_sort_pairs(w + p.sort_tmp, sort_tmp, kb, vb,
                                        static_cast<uint32_t>(n_edges), 0, 2 * scale + 1, st),
              "dw_rmat_edges: sort");
    hipLaunchKernelGGL(k_rmat_first, dim3(grid_of(n_edges)), dim3(256), 0, st, kb.current(),
                       vb.current(), n_edges, 1ull << (2 * scale), keep);
    DW_LAUNCH_CHECK("dw_rmat_edges/first");
    size_t sel_tmp = p.total - p.sel_tmp;
    DW_HIP_OK(rocprim::select(w + p.sel_tmp, sel_tmp, static_cast<const uint64_t *>(raw),
                              static_cast<const uint8_t *>(keep), edges, n_unique,
                              static_cast<size_t>(n_edges), st),
              "dw_rmat_edges: compaction");
    return DW_OK;
}

int dw_graph_isolated(const uint64_t *edges, int64_t n_edges, int64_t n_nodes,
                      int32_t *isolated, int64_t *n_isolated, int32_t *status, void *workspace,
                      size_t workspace_bytes, void *stream) {
    DW_REQUIRE(n_edges >= 0 && n_nodes >= 1 && n_nodes < (int64_t(1) << 31),
               "dw_graph_isolated: bad sizes");
    DW_REQUIRE(isolated && n_isolated && status && workspace && (edges || n_edges == 0),
               "dw_graph_isolated: null pointer");
    CsrPlan p;
    int rc = plan_csr(n_edges > 0 ? n_edges : 1, n_nodes, &p);
    if (rc != DW_OK) return rc;
    DW_REQUIRE(workspace_bytes >= p.total, "dw_graph_isolated: workspace too small");
    hipStream_t st = dw::as_stream(stream);
    char *w = static_cast<char *>(workspace);
    uint32_t *deg = reinterpret_cast<uint32_t *>(w + p.deg);
    uint8_t *flags = reinterpret_cast<uint8_t *>(w + p.flags);
    DW_HIP_OK(hipMemsetAsync(deg, 0, n_nodes * 4, st), "dw_graph_isolated: memset");
    if (n_edges > 0) {
        hipLaunchKernelGGL(k_endpoint_degree, dim3(grid_of(n_edges)), dim3(256), 0, st, edges,
                           n_edges, n_nodes, deg, status);
        DW_LAUNCH_CHECK("dw_graph_isolated/degree");
    }
    hipLaunchKernelGGL(k_zero_flags, dim3(grid_of(n_nodes)), dim3(256), 0, st, deg, n_nodes,
                       flags);
    DW_LAUNCH_CHECK("dw_graph_isolated/flags");
    size_t sel_tmp = p.total - p.sel_tmp;
    DW_HIP_OK(rocprim::select(w + p.sel_tmp, sel_tmp, rocprim::counting_iterator<int32_t>(0),
                              static_cast<const uint8_t *>(flags), isolated, n_isolated,
                              static_cast<size_t>(n_nodes), st),
              "dw_graph_isolated: compaction");
    return DW_OK;
}

int dw_csr_from_edges(const uint64_t *edges, int64_t n_edges, int64_t n_nodes,
                      int64_t *row_ptr, int32_t *col, int32_t *status, void *workspace,
                      size_t workspace_bytes, void *stream) {
    DW_REQUIRE(n_edges >= 0 && n_nodes >= 1 && n_nodes < (int64_t(1) << 31) &&
                   2 * n_edges < (int64_t(1) << 31),
               "dw_csr_from_edges: bad sizes");
    DW_REQUIRE(row_ptr && status && workspace && (n_edges == 0 || (edges && col)),
               "dw_csr_from_edges: null pointer");
    CsrPlan p;
    int rc = plan_csr(n_edges > 0 ? n_edges : 1, n_nodes, &p);
    if (rc != DW_OK) return rc;
    DW_REQUIRE(workspace_bytes >= p.total, "dw_csr_from_edges: workspace too small");
    hipStream_t st = dw::as_stream(stream);
    char *w = static_cast<char *>(workspace);
    uint32_t *deg = reinterpret_cast<uint32_t *>(w + p.deg);
    DW_HIP_OK(hipMemsetAsync(deg, 0, n_nodes * 4, st), "dw_csr_from_edges: memset");
    hipLaunchKernelGGL(k_row_ptr_head, dim3(1), dim3(1), 0, st, row_ptr);
    DW_LAUNCH_CHECK("dw_csr_from_edges/head");
    if (n_edges > 0) {
        hipLaunchKernelGGL(k_endpoint_degree, dim3(grid_of(n_edges)), dim3(256), 0, st, edges,
                           n_edges, n_nodes, deg, status);
        DW_LAUNCH_CHECK("dw_csr_from_edges/degree");
        const int64_t nnz = 2 * n_edges;
        uint32_t *k0 = reinterpret_cast<uint32_t *>(w + p.keys0);
        uint32_t *k1 = reinterpret_cast<uint32_t *>(w + p.keys1);
        uint32_t *v0 = reinterpret_cast<uint32_t *>(w + p.vals0);
        uint32_t *v1 = reinterpret_cast<uint32_t *>(w + p.vals1);
        hipLaunchKernelGGL(k_csr_entries, dim3(grid_of(n_edges)), dim3(256), 0, st, edges,
                           n_edges, k0, v0);
        DW_LAUNCH_CHECK("dw_csr_from_edges/entries");
        rocprim::double_buffer<uint32_t> kb(k0, k1), vb(v0, v1);
        size_t sort_tmp = p.scan_tmp - p.sort_tmp;
        DW_HIP_OK(rocprim::radix_sort_pairs(w + p.sort_tmp, sort_tmp, kb, vb,
                                            static_cast<uint32_t>(nnz), 0, bits_for(n_nodes),
                                            st),
                  "dw_csr_from_edges: sort");
        DW_HIP_OK(hipMemcpyAsync(col, vb.current(), nnz * 4, hipMemcpyDeviceToDevice, st),
                  "dw_csr_from_edges: copy");
    }
    size_t scan_tmp = p.sel_tmp - p.scan_tmp;
    DW_HIP_OK(rocprim::inclusive_scan(w + p.scan_tmp, scan_tmp, static_cast<const uint32_t *>(deg),
                                      row_ptr + 2, static_cast<size_t>(n_nodes),
                                      rocprim::plus<int64_t>(), st),
              "dw_csr_from_edges: scan");
    return DW_OK;
}

}  // extern "C"
