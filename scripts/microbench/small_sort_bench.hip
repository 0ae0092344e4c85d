// Records sort at the reference's 64-walk batch on C3 (269K records, 21-bit rows; the lazy
// owner step, profiles/r03_*): rocprim onesweep configs, whole call timed (lookback-state
// memsets included).
//   hipcc -O3 --offload-arch=gfx950 scripts/microbench/small_sort_bench.hip -o scripts/microbench/small_sort_bench
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/rocprim.hpp>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);              \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

__global__ void fill(uint32_t *k, uint64_t *v, int n, uint32_t V) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        uint32_t x = i * 2654435761u;
        x ^= x >> 13;
        x *= 0x5bd1e995;
        x ^= x >> 15;
        k[i] = x % V;
        v[i] = i;
    }
}

template <unsigned Bits, unsigned BS, unsigned IPT, unsigned MERGE = 0>
using OS = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<BS, IPT>,
                                        rocprim::kernel_config<BS, IPT>, Bits,
                                        rocprim::block_radix_rank_algorithm::match>,
    MERGE>;

template <class Cfg>
void run(const char *name, uint32_t *k0, uint32_t *k1, uint64_t *v0, uint64_t *v1, int n,
         unsigned bits, void *tmp, size_t cap) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e9;
    for (int it = 0; it < 20; ++it) {
        hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, 0, k0, v0, n, 1048577u);
        rocprim::double_buffer<uint32_t> kb(k0, k1);
        rocprim::double_buffer<uint64_t> vb(v0, v1);
        size_t tb = 0;
        CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tb, kb, vb, n, 0, bits));
        if (tb > cap) {
            printf("%s: temp %zu > cap\n", name, tb);
            return;
        }
        CK(hipEventRecord(a));
        CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, kb, vb, n, 0, bits));
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (it > 2 && ms < best) best = ms;
    }
    printf("{\"config\": \"%s\", \"n\": %d, \"us\": %.2f}\n", name, n, best * 1e3);
    fflush(stdout);
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 268800;
    uint32_t *k0, *k1;
    uint64_t *v0, *v1;
    CK(hipMalloc(&k0, n * 4));
    CK(hipMalloc(&k1, n * 4));
    CK(hipMalloc(&v0, n * 8));
    CK(hipMalloc(&v1, n * 8));
    const size_t cap = 256ull << 20;
    void *tmp;
    CK(hipMalloc(&tmp, cap));
    run<OS<8, 256, 8, 128 * 1024>>("8-bit 256x8 (product small)", k0, k1, v0, v1, n, 21, tmp, cap);
    run<OS<11, 1024, 4>>("11-bit 1024x4", k0, k1, v0, v1, n, 21, tmp, cap);
    run<OS<11, 1024, 8>>("11-bit 1024x8", k0, k1, v0, v1, n, 21, tmp, cap);
    run<OS<11, 1024, 16>>("11-bit 1024x16 (product large)", k0, k1, v0, v1, n, 21, tmp, cap);
    run<OS<11, 512, 8>>("11-bit 512x8", k0, k1, v0, v1, n, 21, tmp, cap);
    run<OS<11, 256, 8>>("11-bit 256x8", k0, k1, v0, v1, n, 21, tmp, cap);
    run<OS<8, 512, 8>>("8-bit 512x8", k0, k1, v0, v1, n, 21, tmp, cap);
    run<OS<7, 256, 8>>("7-bit 256x8", k0, k1, v0, v1, n, 21, tmp, cap);
    run<OS<8, 256, 8, 512 * 1024>>("8-bit 256x8, merge <= 512K", k0, k1, v0, v1, n, 21, tmp, cap);
    return 0;
}
