// CSR utilities on gfx950: validation, sorted neighbour copy, per-row alias tables.
//
// The reference keeps its graph as a networkx dict-of-dicts and walks it from Python
// (shallow_encoders/graph/random_walk_generator.py:41-53). On the device the graph is a CSR in
// HBM (row_ptr int64, col int32, optional float64 weights) in vocabulary-id space.
#include <hipcub/hipcub.hpp>

#include "dw_common.h"

namespace {

__global__ void k_csr_validate(const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
                               int64_t n_rows, int64_t nnz, int32_t *status) {
    const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    if (tid == 0) {
        if (row_ptr[0] != 0 || row_ptr[n_rows] != nnz) dw::status_or(status, DW_S_BAD_CSR);
    }
    for (int64_t r = tid; r < n_rows; r += stride)
        if (row_ptr[r] > row_ptr[r + 1]) dw::status_or(status, DW_S_BAD_CSR);
    for (int64_t e = tid; e < nnz; e += stride) {
        const int32_t c = col[e];
        if (c < 0 || (int64_t)c >= n_rows) dw::status_or(status, DW_S_BAD_CSR);
    }
}

// key = row << 32 | col: one global radix sort orders every row's neighbours ascending.
__global__ void k_make_keys(const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
                            int64_t n_rows, uint64_t *__restrict__ keys) {
    const int64_t stride = (int64_t)gridDim.x * (blockDim.x / 64);
    const int lane = threadIdx.x & 63;
    for (int64_t r = blockIdx.x * (int64_t)(blockDim.x / 64) + threadIdx.x / 64; r < n_rows;
         r += stride) {
        const int64_t a = row_ptr[r], b = row_ptr[r + 1];
        for (int64_t e = a + lane; e < b; e += 64)
            keys[e] = (static_cast<uint64_t>(r) << 32) | static_cast<uint32_t>(col[e]);
    }
}

// adjacent equal entries within a row of the sorted copy: a repeated neighbour
__global__ void k_csr_simple(const int64_t *__restrict__ row_ptr,
                             const int32_t *__restrict__ col_sorted, int64_t n_rows,
                             int32_t *status) {
    const int64_t stride = (int64_t)gridDim.x * (blockDim.x / 64);
    const int lane = threadIdx.x & 63;
    bool dup = false;
    for (int64_t r = blockIdx.x * (int64_t)(blockDim.x / 64) + threadIdx.x / 64; r < n_rows;
         r += stride) {
        const int64_t a = row_ptr[r], b = row_ptr[r + 1];
        for (int64_t e = a + 1 + lane; e < b; e += 64) dup = dup || col_sorted[e] == col_sorted[e - 1];
    }
    if (__ballot(dup) != 0ull && lane == 0) dw::status_or(status, DW_S_DUP_NEIGHBOR);
}

__global__ void k_keys_to_col(const uint64_t *__restrict__ keys, int64_t nnz,
                              int32_t *__restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nnz; e += stride)
        out[e] = static_cast<int32_t>(keys[e] & 0xFFFFFFFFull);
}

// Vose alias construction, one thread per row (rows are independent; hubs are serial but rare).
// Small-list grows from the row's front of work_idx, large-list from its back: they never meet.
__global__ void k_alias_build(const int64_t *__restrict__ row_ptr, const double *__restrict__ w,
                              int64_t n_rows, uint32_t *__restrict__ prob_thr,
                              int32_t *__restrict__ alias, double *__restrict__ scaled,
                              int32_t *__restrict__ stack, int32_t *status) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n_rows; r += stride) {
        const int64_t a = row_ptr[r], b = row_ptr[r + 1];
        const int64_t n = b - a;
        if (n == 0) continue;
        double sum = 0.0;
        for (int64_t e = a; e < b; ++e) sum += w ? w[e] : 1.0;
        if (!(sum > 0.0)) {
            dw::status_or(status, DW_S_ZERO_WEIGHT);
            for (int64_t e = a; e < b; ++e) {
                prob_thr[e] = 0xFFFFFFFFu;
                alias[e] = static_cast<int32_t>(e - a);
            }
            continue;
        }
        int64_t ns = 0, nl = 0;
        for (int64_t e = a; e < b; ++e) {
            const double s = (w ? w[e] : 1.0) * static_cast<double>(n) / sum;
            scaled[e] = s;
            alias[e] = static_cast<int32_t>(e - a);
            if (s < 1.0)
                stack[a + ns++] = static_cast<int32_t>(e - a);
            else
                stack[b - 1 - nl++] = static_cast<int32_t>(e - a);
        }
        while (ns > 0 && nl > 0) {
            const int32_t l = stack[a + --ns];
            const int32_t g = stack[b - 1 - --nl];
            const double pl = scaled[a + l];
            prob_thr[a + l] = static_cast<uint32_t>(fmin(floor(pl * 4294967296.0), 4294967295.0));
            alias[a + l] = g;
            const double pg = (scaled[a + g] + pl) - 1.0;
            scaled[a + g] = pg;
            if (pg < 1.0)
                stack[a + ns++] = g;
            else
                stack[b - 1 - nl++] = g;
        }
        while (nl > 0) {
            const int32_t g = stack[b - 1 - --nl];
            prob_thr[a + g] = 0xFFFFFFFFu;
        }
        while (ns > 0) {
            const int32_t l = stack[a + --ns];
            prob_thr[a + l] = 0xFFFFFFFFu;
        }
    }
}


// ---- per-row adjacency hash (node2vec "x in N(prev)" tests in one probe) ---------------------
// Row u of degree > DW_ADJ_HASH_MIN_DEG owns nb(u) = ceil(4 deg / 48) buckets of 16 int32 slots
// (load <= 3/4) at adj_off[u]; rows of lower degree own none (a single load of their unsorted
// neighbour list decides). Key x goes to bucket dw::adj_bucket(x, nb) and the first free slot
// of that bucket or the next ones (cyclically): slots only go empty -> full, so a bucket with a
// free slot ends every probe sequence through it.
__global__ void k_adj_counts(const int64_t *__restrict__ row_ptr, int64_t n_rows,
                             int64_t *__restrict__ counts) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r <= n_rows; r += stride)
        counts[r] = r < n_rows ? 16 * dw::adj_buckets(row_ptr[r + 1] - row_ptr[r]) : 0;
}

__global__ void k_adj_insert(const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
                             int64_t n_rows, const int64_t *__restrict__ adj_off,
                             int32_t *__restrict__ tab, int32_t *status) {
    const int64_t stride = (int64_t)gridDim.x * (blockDim.x / 64);
    const int lane = threadIdx.x & 63;
    for (int64_t r = blockIdx.x * (int64_t)(blockDim.x / 64) + threadIdx.x / 64; r < n_rows;
         r += stride) {
        const int64_t off = adj_off[r];
        const uint32_t nb = static_cast<uint32_t>((adj_off[r + 1] - off) / 16);
        if (nb == 0) continue;
        const int64_t a = row_ptr[r], b = row_ptr[r + 1];
        for (int64_t e = a + lane; e < b; e += 64) {
            const int32_t x = col[e];
            uint32_t bk = dw::adj_bucket(x, nb);
            bool done = false;
            for (uint32_t t = 0; t < nb && !done; ++t) {
                int32_t *slots = tab + off + (int64_t)bk * 16;
                for (int j = 0; j < 16; ++j) {
                    const int32_t old = atomicCAS(slots + j, -1, x);
                    // inserted, or a repeated neighbour merged (membership is all the Philox
                    // walker asks; the exact replay refuses such rows, dw_csr_check_simple)
                    if (old == -1 || old == x) {
                        done = true;
                        break;
                    }
                }
                if (++bk == nb) bk = 0;
            }
            if (!done) dw::status_or(status, DW_S_BAD_CSR);   // cannot happen at load <= 3/4
        }
    }
}

// adj_hpos[slot] = the index of the slot's key in its row's insertion order (networkx
// neighbour order): the bit-exact node2vec replay maps a neighbour of prev to its position in
// N(v) with one probe (dw_walk_replay's "probe the shorter list" step).
__global__ void k_adj_positions(const int64_t *__restrict__ row_ptr,
                                const int32_t *__restrict__ col, int64_t n_rows,
                                const int64_t *__restrict__ adj_off,
                                const int32_t *__restrict__ tab, int32_t *__restrict__ hpos,
                                int32_t *status) {
    const int64_t stride = (int64_t)gridDim.x * (blockDim.x / 64);
    const int lane = threadIdx.x & 63;
    for (int64_t r = blockIdx.x * (int64_t)(blockDim.x / 64) + threadIdx.x / 64; r < n_rows;
         r += stride) {
        const int64_t off = adj_off[r];
        const uint32_t nb = static_cast<uint32_t>((adj_off[r + 1] - off) / 16);
        if (nb == 0) continue;
        const int64_t a = row_ptr[r], b = row_ptr[r + 1];
        for (int64_t e = a + lane; e < b; e += 64) {
            const int32_t x = col[e];
            uint32_t bk = dw::adj_bucket(x, nb);
            bool done = false;
            for (uint32_t t = 0; t < nb && !done; ++t) {
                const int64_t s0 = off + (int64_t)bk * 16;
                for (int j = 0; j < 16; ++j)
                    if (tab[s0 + j] == x) {
                        hpos[s0 + j] = static_cast<int32_t>(e - a);
                        done = true;
                        break;
                    }
                if (++bk == nb) bk = 0;
            }
            if (!done) dw::status_or(status, DW_S_BAD_CSR);
        }
    }
}

inline int grid_for(int64_t work, int block, int cap = 8192) {
    int64_t g = (work + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return static_cast<int>(g);
}

}  // namespace

extern "C" {

int dw_csr_validate(const int64_t *row_ptr, const int32_t *col, int64_t n_rows, int64_t nnz,
                    int32_t *status, void *stream) {
    DW_REQUIRE(row_ptr && status, "dw_csr_validate: null pointer");
    DW_REQUIRE(n_rows >= 0 && nnz >= 0, "dw_csr_validate: negative size");
    DW_REQUIRE(nnz == 0 || col, "dw_csr_validate: col is null");
    hipLaunchKernelGGL(k_csr_validate, dim3(grid_for(n_rows > nnz ? n_rows : nnz, 256)), dim3(256),
                       0, dw::as_stream(stream), row_ptr, col, n_rows, nnz, status);
    DW_LAUNCH_CHECK("dw_csr_validate");
    return DW_OK;
}

int dw_csr_sort_copy(const int64_t *row_ptr, const int32_t *col, int64_t n_rows, int64_t nnz,
                     int32_t *col_sorted, void *temp, size_t *temp_bytes, void *stream) {
    DW_REQUIRE(temp_bytes, "dw_csr_sort_copy: temp_bytes is null");
    DW_REQUIRE(n_rows >= 0 && nnz >= 0, "dw_csr_sort_copy: negative size");
    DW_REQUIRE(n_rows < (int64_t(1) << 31), "dw_csr_sort_copy: n_rows must fit int32");
    int end_bit = 32;
    while (end_bit < 64 && (uint64_t(n_rows) >> (end_bit - 32)) != 0) ++end_bit;
    const size_t keys_bytes = ((size_t)nnz * sizeof(uint64_t) + 255) & ~size_t(255);
    size_t cub_bytes = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortKeys(nullptr, cub_bytes, (uint64_t *)nullptr,
                                                     (uint64_t *)nullptr, (int)nnz, 0, end_bit,
                                                     dw::as_stream(stream));
    if (e != hipSuccess) {
        dw::set_error("dw_csr_sort_copy: hipcub size query: %s", hipGetErrorString(e));
        return DW_E_HIP;
    }
    const size_t need = 2 * keys_bytes + cub_bytes;
    if (temp == nullptr) {
        *temp_bytes = need;
        return DW_OK;
    }
    DW_REQUIRE(*temp_bytes >= need, "dw_csr_sort_copy: temp too small (%zu < %zu)", *temp_bytes,
               need);
    DW_REQUIRE(nnz < (int64_t(1) << 31), "dw_csr_sort_copy: nnz must fit int32 for hipcub");
    if (nnz == 0) return DW_OK;
    DW_REQUIRE(row_ptr && col && col_sorted, "dw_csr_sort_copy: null pointer");
    char *base = static_cast<char *>(temp);
    uint64_t *k_in = reinterpret_cast<uint64_t *>(base);
    uint64_t *k_out = reinterpret_cast<uint64_t *>(base + keys_bytes);
    void *cub_tmp = base + 2 * keys_bytes;
    hipLaunchKernelGGL(k_make_keys, dim3(grid_for(n_rows * 64, 256)), dim3(256), 0,
                       dw::as_stream(stream), row_ptr, col, n_rows, k_in);
    DW_LAUNCH_CHECK("dw_csr_sort_copy/keys");
    e = hipcub::DeviceRadixSort::SortKeys(cub_tmp, cub_bytes, k_in, k_out, (int)nnz, 0, end_bit,
                                          dw::as_stream(stream));
    if (e != hipSuccess) {
        dw::set_error("dw_csr_sort_copy: hipcub sort: %s", hipGetErrorString(e));
        return DW_E_HIP;
    }
    hipLaunchKernelGGL(k_keys_to_col, dim3(grid_for(nnz, 256)), dim3(256), 0,
                       dw::as_stream(stream), k_out, nnz, col_sorted);
    DW_LAUNCH_CHECK("dw_csr_sort_copy/extract");
    return DW_OK;
}

int dw_csr_check_simple(const int64_t *row_ptr, const int32_t *col_sorted, int64_t n_rows,
                        int64_t nnz, int32_t *status, void *stream) {
    DW_REQUIRE(n_rows >= 0 && nnz >= 0, "dw_csr_check_simple: negative size");
    DW_REQUIRE(row_ptr && status, "dw_csr_check_simple: null pointer");
    if (nnz == 0 || n_rows == 0) return DW_OK;
    DW_REQUIRE(col_sorted, "dw_csr_check_simple: col_sorted is null");
    hipLaunchKernelGGL(k_csr_simple, dim3(grid_for(n_rows * 64, 256)), dim3(256), 0,
                       dw::as_stream(stream), row_ptr, col_sorted, n_rows, status);
    DW_LAUNCH_CHECK("dw_csr_check_simple");
    return DW_OK;
}

int dw_adj_hash_offsets(const int64_t *row_ptr, int64_t n_rows, int64_t *adj_off, void *temp,
                        size_t *temp_bytes, void *stream) {
    DW_REQUIRE(temp_bytes, "dw_adj_hash_offsets: temp_bytes is null");
    DW_REQUIRE(n_rows >= 0 && n_rows < (int64_t(1) << 31),
               "dw_adj_hash_offsets: n_rows must be in [0, 2^31)");
    const size_t cnt_bytes = ((size_t)(n_rows + 1) * sizeof(int64_t) + 255) & ~size_t(255);
    size_t cub_bytes = 0;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, cub_bytes, (int64_t *)nullptr,
                                                    (int64_t *)nullptr, (int)(n_rows + 1),
                                                    dw::as_stream(stream));
    if (e != hipSuccess) {
        dw::set_error("dw_adj_hash_offsets: hipcub size query: %s", hipGetErrorString(e));
        return DW_E_HIP;
    }
    const size_t need = cnt_bytes + cub_bytes;
    if (temp == nullptr) {
        *temp_bytes = need;
        return DW_OK;
    }
    DW_REQUIRE(*temp_bytes >= need, "dw_adj_hash_offsets: temp too small (%zu < %zu)",
               *temp_bytes, need);
    DW_REQUIRE(row_ptr && adj_off, "dw_adj_hash_offsets: null pointer");
    int64_t *counts = static_cast<int64_t *>(temp);
    hipLaunchKernelGGL(k_adj_counts, dim3(grid_for(n_rows + 1, 256)), dim3(256), 0,
                       dw::as_stream(stream), row_ptr, n_rows, counts);
    DW_LAUNCH_CHECK("dw_adj_hash_offsets/counts");
    e = hipcub::DeviceScan::ExclusiveSum(static_cast<char *>(temp) + cnt_bytes, cub_bytes, counts,
                                         adj_off, (int)(n_rows + 1), dw::as_stream(stream));
    if (e != hipSuccess) {
        dw::set_error("dw_adj_hash_offsets: hipcub scan: %s", hipGetErrorString(e));
        return DW_E_HIP;
    }
    return DW_OK;
}

int dw_adj_hash_positions(const int64_t *row_ptr, const int32_t *col, int64_t n_rows,
                          const int64_t *adj_off, const int32_t *adj_hash, int64_t n_slots,
                          int32_t *adj_hpos, int32_t *status, void *stream) {
    DW_REQUIRE(n_rows >= 0 && n_slots >= 0, "dw_adj_hash_positions: negative size");
    DW_REQUIRE(row_ptr && adj_off && status, "dw_adj_hash_positions: null pointer");
    if (n_slots == 0) return DW_OK;
    DW_REQUIRE(col && adj_hash && adj_hpos, "dw_adj_hash_positions: null pointer");
    hipError_t e = hipMemsetAsync(adj_hpos, 0xFF, (size_t)n_slots * sizeof(int32_t),
                                  dw::as_stream(stream));
    if (e != hipSuccess) {
        dw::set_error("dw_adj_hash_positions: memset: %s", hipGetErrorString(e));
        return DW_E_HIP;
    }
    hipLaunchKernelGGL(k_adj_positions, dim3(grid_for(n_rows * 64, 256)), dim3(256), 0,
                       dw::as_stream(stream), row_ptr, col, n_rows, adj_off, adj_hash, adj_hpos,
                       status);
    DW_LAUNCH_CHECK("dw_adj_hash_positions");
    return DW_OK;
}

int dw_adj_hash_build(const int64_t *row_ptr, const int32_t *col, int64_t n_rows,
                      const int64_t *adj_off, int64_t n_slots, int32_t *adj_hash, int32_t *status,
                      void *stream) {
    DW_REQUIRE(n_rows >= 0 && n_slots >= 0, "dw_adj_hash_build: negative size");
    DW_REQUIRE(row_ptr && adj_off && status, "dw_adj_hash_build: null pointer");
    if (n_slots == 0) return DW_OK;
    DW_REQUIRE(col && adj_hash, "dw_adj_hash_build: null pointer");
    hipError_t e = hipMemsetAsync(adj_hash, 0xFF, (size_t)n_slots * sizeof(int32_t),
                                  dw::as_stream(stream));
    if (e != hipSuccess) {
        dw::set_error("dw_adj_hash_build: memset: %s", hipGetErrorString(e));
        return DW_E_HIP;
    }
    hipLaunchKernelGGL(k_adj_insert, dim3(grid_for(n_rows * 64, 256)), dim3(256), 0,
                       dw::as_stream(stream), row_ptr, col, n_rows, adj_off, adj_hash, status);
    DW_LAUNCH_CHECK("dw_adj_hash_build");
    return DW_OK;
}

int dw_alias_build(const int64_t *row_ptr, const double *weights, int64_t n_rows, int64_t nnz,
                   uint32_t *prob_thr, int32_t *alias, double *work_prob, int32_t *work_idx,
                   int32_t *status, void *stream) {
    DW_REQUIRE(row_ptr && prob_thr && alias && work_prob && work_idx,
               "dw_alias_build: null pointer");
    DW_REQUIRE(n_rows >= 0 && nnz >= 0, "dw_alias_build: negative size");
    hipLaunchKernelGGL(k_alias_build, dim3(grid_for(n_rows, 64)), dim3(64), 0,
                       dw::as_stream(stream), row_ptr, weights, n_rows, prob_thr, alias, work_prob,
                       work_idx, status);
    DW_LAUNCH_CHECK("dw_alias_build");
    return DW_OK;
}

}  // extern "C"
