// Microbenchmark: the SGNS records as sorted today (u32 row key + u64 {coef, centre} value,
// 21 key bits) vs packed into one u64 key-only record {row << 22 | centre << 1 | label} sorted
// on bits [22, 43) — the form in which pass 2 would recompute the coefficient.
//   hipcc -O3 --offload-arch=gfx950 scripts/microbench/sort_keys_bench.hip -o /tmp/skb
#include <string.h>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>
#include <stdint.h>
#include <string.h>
#include <stdio.h>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);              \
            return 1;                                                            \
        }                                                                        \
    } while (0)

__device__ uint32_t mix(uint32_t i) {
    uint32_t x = i * 2654435761u;
    x ^= x >> 13;
    x *= 0x5bd1e995;
    x ^= x >> 15;
    return x;
}
__global__ void fill_pairs(uint32_t *k, uint64_t *v, int n, uint32_t V) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        k[i] = mix(i) % V;
        v[i] = i;
    }
}
struct alignas(8) Rec {   // packed record: row key + {centre, label} payload
    uint32_t payload;
    uint32_t row;
};
static const unsigned kBegin = 0, kEnd = 21;
struct RowOnly {          // rocprim decomposer: the sort sees only the row word
    __host__ __device__ rocprim::tuple<uint32_t &> operator()(Rec &r) const {
        return rocprim::tuple<uint32_t &>{r.row};
    }
};
__global__ void fill_keys(Rec *k, int n, uint32_t V) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) k[i] = Rec{static_cast<uint32_t>(i), mix(i) % V};
}

template <unsigned Bits, unsigned BS, unsigned IPT>
using OS = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<BS, IPT>,
                                        rocprim::kernel_config<BS, IPT>, Bits,
                                        rocprim::block_radix_rank_algorithm::match>>;

template <unsigned Bits, unsigned HBS, unsigned HIPT, unsigned BS, unsigned IPT>
using OS2 = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<HBS, HIPT>,
                                        rocprim::kernel_config<BS, IPT>, Bits,
                                        rocprim::block_radix_rank_algorithm::match>>;

template <class Cfg>
int pairs(const char *name, int n, void *tmp, size_t cap) {
    uint32_t *k0, *k1;
    uint64_t *v0, *v1;
    CK(hipMalloc(&k0, n * 4ull));
    CK(hipMalloc(&k1, n * 4ull));
    CK(hipMalloc(&v0, n * 8ull));
    CK(hipMalloc(&v1, n * 8ull));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e9;
    for (int it = 0; it < 6; ++it) {
        hipLaunchKernelGGL(fill_pairs, dim3((n + 255) / 256), dim3(256), 0, 0, k0, v0, n, 1048577u);
        rocprim::double_buffer<uint32_t> kb(k0, k1);
        rocprim::double_buffer<uint64_t> vb(v0, v1);
        size_t tb = 0;
        CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tb, kb, vb, n, 0, 21));
        if (tb > cap) return printf("cap\n"), 1;
        hipEventRecord(a);
        CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, kb, vb, n, 0, 21));
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (it > 0 && ms < best) best = ms;
    }
    printf("%-44s n=%d  %.3f ms\n", name, n, best);
    hipFree(k0); hipFree(k1); hipFree(v0); hipFree(v1);
    return 0;
}

__global__ void fill_p32(uint32_t *k, uint32_t *v, int n, uint32_t V) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        k[i] = mix(i) % V;
        v[i] = i;
    }
}

template <class Cfg>
int pairs32(const char *name, int n, void *tmp, size_t cap) {
    uint32_t *k0, *k1, *v0, *v1;
    CK(hipMalloc(&k0, n * 4ull));
    CK(hipMalloc(&k1, n * 4ull));
    CK(hipMalloc(&v0, n * 4ull));
    CK(hipMalloc(&v1, n * 4ull));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e9;
    for (int it = 0; it < 6; ++it) {
        hipLaunchKernelGGL(fill_p32, dim3((n + 255) / 256), dim3(256), 0, 0, k0, v0, n, 1048577u);
        rocprim::double_buffer<uint32_t> kb(k0, k1), vb(v0, v1);
        size_t tb = 0;
        CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tb, kb, vb, n, 0, 21));
        if (tb > cap) return printf("cap\n"), 1;
        hipEventRecord(a);
        CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, kb, vb, n, 0, 21));
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (it > 0 && ms < best) best = ms;
    }
    printf("%-44s n=%d  %.3f ms\n", name, n, best);
    hipFree(k0); hipFree(k1); hipFree(v0); hipFree(v1);
    return 0;
}

template <class Cfg>
int keys(const char *name, int n, void *tmp, size_t cap) {
    Rec *k0, *k1;
    CK(hipMalloc(&k0, n * 8ull));
    CK(hipMalloc(&k1, n * 8ull));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e9;
    for (int it = 0; it < 6; ++it) {
        hipLaunchKernelGGL(fill_keys, dim3((n + 255) / 256), dim3(256), 0, 0, k0, n, 1048577u);
        rocprim::double_buffer<Rec> kb(k0, k1);
        size_t tb = 0;
        CK(rocprim::radix_sort_keys<Cfg>(nullptr, tb, kb, n, RowOnly{}, kBegin, kEnd, hipStream_t(0)));
        if (tb > cap) return printf("cap\n"), 1;
        hipEventRecord(a);
        CK(rocprim::radix_sort_keys<Cfg>(tmp, tb, kb, n, RowOnly{}, kBegin, kEnd, hipStream_t(0)));
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (it > 0 && ms < best) best = ms;
        if (it == 1) {   // sorted on the row field, stable (payload ascending within a row)
            static Rec h[1 << 16];
            CK(hipMemcpy(h, kb.current() + n / 2, sizeof(h), hipMemcpyDeviceToHost));
            for (int i = 1; i < (1 << 16); ++i)
                if (h[i].row < h[i - 1].row ||
                    (h[i].row == h[i - 1].row && h[i].payload < h[i - 1].payload)) {
                    printf("%s: NOT SORTED/STABLE at %d\n", name, i);
                    break;
                }
        }
    }
    printf("%-44s n=%d  %.3f ms\n", name, n, best);
    hipFree(k0); hipFree(k1);
    return 0;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 34406400;
    const size_t cap = 1024ull << 20;
    void *tmp;
    CK(hipMalloc(&tmp, cap));
    pairs<OS<11, 1024, 16>>("pairs u32/u64 11-bit 1024x16 (product)", n, tmp, cap);
    pairs32<OS<11, 1024, 16>>("pairs u32/u32 11-bit 1024x16", n, tmp, cap);
    pairs32<OS<11, 1024, 20>>("pairs u32/u32 11-bit 1024x20", n, tmp, cap);
    pairs32<OS<11, 1024, 24>>("pairs u32/u32 11-bit 1024x24", n, tmp, cap);
    pairs32<OS<11, 512, 24>>("pairs u32/u32 11-bit 512x24", n, tmp, cap);
    keys<OS<10, 1024, 16>>("keys Rec row-only 10-bit 1024x16 (3 passes)", n, tmp, cap);
    pairs<OS<11, 1024, 16>>("pairs (again)", n, tmp, cap);
    return 0;
}
