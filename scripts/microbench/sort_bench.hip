// Microbenchmark: device radix sort of SGNS gradient records (key = output row < V = 2^20 + 1,
// 21 bits; value = 64-bit {coef, centre}) — which onesweep digit width sorts them fastest.
//   hipcc -O3 --offload-arch=gfx950 scripts/microbench/sort_bench.hip -o scripts/microbench/sort_bench
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/rocprim.hpp>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);              \
            return 1;                                                            \
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

template <unsigned Bits, unsigned BS, unsigned IPT,
          rocprim::block_radix_rank_algorithm A = rocprim::block_radix_rank_algorithm::match>
using OS = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<BS, IPT>,
                                        rocprim::kernel_config<BS, IPT>, Bits, A>>;

template <class Cfg>
int run(const char *name, uint32_t *k0, uint32_t *k1, uint64_t *v0, uint64_t *v1, int n,
        unsigned bits, void *tmp, size_t cap) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e9;
    for (int it = 0; it < 6; ++it) {
        rocprim::double_buffer<uint32_t> kb(k0, k1);
        rocprim::double_buffer<uint64_t> vb(v0, v1);
        size_t tb = 0;
        CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tb, kb, vb, n, 0, bits));
        if (tb > cap) {
            printf("%s: temp %zu > cap\n", name, tb);
            return 0;
        }
        hipEventRecord(a);
        CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, kb, vb, n, 0, bits));
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (it > 0 && ms < best) best = ms;
        // verify sortedness once
        if (it == 1) {
            static uint32_t host[1 << 16];
            CK(hipMemcpy(host, kb.current() + n / 2, sizeof(host), hipMemcpyDeviceToHost));
            for (int i = 1; i < (1 << 16); ++i)
                if (host[i] < host[i - 1]) {
                    printf("%s: NOT SORTED\n", name);
                    break;
                }
        }
    }
    printf("%-40s n=%d  %.3f ms  %.2f Gitems/s\n", name, n, best, n / best / 1e6);
    return 0;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 34406400;
    const uint32_t V = 1048577;
    const unsigned bits = 21;
    uint32_t *k0, *k1;
    uint64_t *v0, *v1;
    CK(hipMalloc(&k0, n * 4));
    CK(hipMalloc(&k1, n * 4));
    CK(hipMalloc(&v0, n * 8));
    CK(hipMalloc(&v1, n * 8));
    const size_t cap = 512ull << 20;
    void *tmp;
    CK(hipMalloc(&tmp, cap));
    auto refill = [&] { hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, 0, k0, v0, n, V); };
    refill();
    run<rocprim::default_config>("default (8-bit digits, 3 passes)", k0, k1, v0, v1, n, bits, tmp, cap);
    refill();
    run<OS<7, 1024, 8>>("7-bit 1024x8", k0, k1, v0, v1, n, bits, tmp, cap);
    refill();
    run<OS<7, 1024, 12>>("7-bit 1024x12", k0, k1, v0, v1, n, bits, tmp, cap);
    refill();
    run<OS<7, 1024, 16>>("7-bit 1024x16", k0, k1, v0, v1, n, bits, tmp, cap);
    refill();
    run<OS<7, 512, 16>>("7-bit 512x16", k0, k1, v0, v1, n, bits, tmp, cap);
    refill();
    run<OS<6, 1024, 8>>("6-bit 1024x8 (4 passes)", k0, k1, v0, v1, n, bits, tmp, cap);
    refill();
    run<OS<8, 1024, 12>>("8-bit 1024x12", k0, k1, v0, v1, n, bits, tmp, cap);
    refill();
    run<OS<11, 1024, 16>>("11-bit 1024x16", k0, k1, v0, v1, n, bits, tmp, cap);
    // round 4: bigger tiles put more items per bucket run (fewer partial lines)
    refill();
    run<OS<11, 1024, 20>>("11-bit 1024x20", k0, k1, v0, v1, n, bits, tmp, cap);
    refill();
    run<OS<11, 1024, 24>>("11-bit 1024x24", k0, k1, v0, v1, n, bits, tmp, cap);
    refill();
    run<OS<11, 1024, 32>>("11-bit 1024x32", k0, k1, v0, v1, n, bits, tmp, cap);
    refill();
    run<OS<10, 1024, 24>>("10-bit 1024x24 (3 passes)", k0, k1, v0, v1, n, bits, tmp, cap);
    refill();
    run<OS<11, 1024, 16>>("11-bit 1024x16 (product, again)", k0, k1, v0, v1, n, bits, tmp, cap);
    return 0;
}
