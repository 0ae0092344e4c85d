// Microbenchmark: the SGNS records sort (34.4M {u32 row, u64 value} pairs, one C3 step) at 21
// key bits (rows 0..2^20, V = 2^20 + 1) against 20 key bits (the last row kept out of the sort),
// over onesweep digit widths / tiles. Keys are refilled before every timed sort.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 scripts/microbench/sort_bits_bench.hip \
//         -o scripts/microbench/sort_bits_bench
#include <hip/hip_runtime.h>
#include <string.h>
#include <rocprim/device/device_radix_sort.hpp>
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

__global__ void fill(uint32_t *k, uint64_t *v, int n, uint32_t V, uint32_t salt) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        uint32_t x = (i ^ salt) * 2654435761u;
        x ^= x >> 13;
        x *= 0x5bd1e995;
        x ^= x >> 15;
        k[i] = static_cast<uint32_t>((static_cast<uint64_t>(x) * V) >> 32);
        v[i] = i;
    }
}

template <unsigned Bits, unsigned BS, unsigned IPT>
using OS = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<BS, IPT>,
                                        rocprim::kernel_config<BS, IPT>, Bits,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;

template <class Cfg>
void run(const char *name, uint32_t *k0, uint32_t *k1, uint64_t *v0, uint64_t *v1, int n,
         uint32_t V, unsigned bits, void *tmp, size_t cap) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e9, sum = 0;
    int cnt = 0;
    for (int it = 0; it < 8; ++it) {
        hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, 0, k0, v0, n, V, it * 77u);
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
        if (it > 1) {
            best = ms < best ? ms : best;
            sum += ms;
            ++cnt;
        }
        if (it == 2) {
            static uint32_t host[1 << 16];
            CK(hipMemcpy(host, kb.current() + n / 2, sizeof(host), hipMemcpyDeviceToHost));
            for (int i = 1; i < (1 << 16); ++i)
                if (host[i] < host[i - 1]) {
                    printf("%s: NOT SORTED\n", name);
                    break;
                }
        }
    }
    printf("%-34s bits=%u  best %.3f ms  mean %.3f ms\n", name, bits, best, sum / cnt);
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 34406400;
    uint32_t *k0, *k1;
    uint64_t *v0, *v1;
    CK(hipMalloc(&k0, n * 4ull));
    CK(hipMalloc(&k1, n * 4ull));
    CK(hipMalloc(&v0, n * 8ull));
    CK(hipMalloc(&v1, n * 8ull));
    const size_t cap = 512ull << 20;
    void *tmp;
    CK(hipMalloc(&tmp, cap));
    const uint32_t V21 = (1u << 20) + 1, V20 = 1u << 20;
    if (argc > 2) {   // tile sweep of the product's 11-bit digits (21 bits)
        run<OS<11, 1024, 16>>("11-bit 1024x16 (product)", k0, k1, v0, v1, n, V21, 21, tmp, cap);
        run<OS<11, 1024, 12>>("11-bit 1024x12", k0, k1, v0, v1, n, V21, 21, tmp, cap);
        run<OS<11, 1024, 20>>("11-bit 1024x20", k0, k1, v0, v1, n, V21, 21, tmp, cap);
        run<OS<11, 1024, 24>>("11-bit 1024x24", k0, k1, v0, v1, n, V21, 21, tmp, cap);
        run<OS<11, 512, 32>>("11-bit 512x32", k0, k1, v0, v1, n, V21, 21, tmp, cap);
        run<OS<11, 768, 16>>("11-bit 768x16", k0, k1, v0, v1, n, V21, 21, tmp, cap);
        run<OS<11, 1024, 16>>("11-bit 1024x16 (product, again)", k0, k1, v0, v1, n, V21, 21,
                              tmp, cap);
        return 0;
    }
    run<OS<11, 1024, 16>>("11-bit 1024x16 (product)", k0, k1, v0, v1, n, V21, 21, tmp, cap);
    run<OS<11, 1024, 16>>("11-bit 1024x16", k0, k1, v0, v1, n, V20, 20, tmp, cap);
    run<OS<10, 1024, 16>>("10-bit 1024x16", k0, k1, v0, v1, n, V20, 20, tmp, cap);
    run<OS<10, 1024, 20>>("10-bit 1024x20", k0, k1, v0, v1, n, V20, 20, tmp, cap);
    run<OS<10, 1024, 12>>("10-bit 1024x12", k0, k1, v0, v1, n, V20, 20, tmp, cap);
    run<OS<10, 512, 16>>("10-bit 512x16", k0, k1, v0, v1, n, V20, 20, tmp, cap);
    run<OS<10, 1024, 24>>("10-bit 1024x24", k0, k1, v0, v1, n, V20, 20, tmp, cap);
    run<OS<11, 1024, 16>>("11-bit 1024x16 (product, again)", k0, k1, v0, v1, n, V21, 21, tmp,
                          cap);
    return 0;
}
