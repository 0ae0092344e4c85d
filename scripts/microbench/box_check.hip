// Are the unscaled sqrt and division of the lazy replays' box (dw_common.h: sqrt_box, div_box)
// bit for bit sqrtf and the IEEE division there?
//   sqrt: every fp32 x in [2^-96, 2^20], and +0 (exhaustive, ~9.7e8 values);
//   div:  N random pairs, |n| in [2^-100, 2^60] (either sign; 1 in 4096 is +0),
//         d in [2^-27, 2^21), exponents uniform, mantissas random.
// Prints the mismatch counts (0 = the box forms may replace the scaled sequences).
//   hipcc -O3 --offload-arch=gfx950 -I include scripts/microbench/box_check.hip \
//         -o scripts/microbench/box_check
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../deepwalk-and-node2vec_amd/csrc/dw_common.h"

__device__ __forceinline__ uint32_t hash32(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return static_cast<uint32_t>(x);
}

__global__ void k_sqrt(uint32_t lo, uint32_t hi, unsigned long long *bad, unsigned int *first) {
    const uint64_t n = static_cast<uint64_t>(hi - lo) + 2;   // [lo, hi] and +0
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
         i += stride) {
        const uint32_t b = i == n - 1 ? 0u : lo + static_cast<uint32_t>(i);
        const float x = __uint_as_float(b);
        const float ref = sqrtf(x);
        const float got = dw::sqrt_box(x);
        if (__float_as_uint(ref) != __float_as_uint(got)) {
            atomicAdd(bad, 1ull);
            atomicMin(first, b);
        }
    }
}

__global__ void k_div(uint64_t n_pairs, unsigned long long *bad, unsigned long long *first) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n_pairs;
         i += stride) {
        const uint32_t h1 = hash32(i * 0x9E3779B97F4A7C15ull + 1);
        const uint32_t h2 = hash32(i ^ 0xD1B54A32D192ED03ull);
        const uint32_t h3 = hash32(i * 0xBF58476D1CE4E5B9ull + 7);
        float nu = ldexpf(1.0f + (h1 & 0x7FFFFF) * 0x1p-23f, static_cast<int>(h2 % 160) - 100);
        if (h1 >> 31) nu = -nu;
        if ((h2 >> 20) == 0) nu = 0.f;
        const float de =
            ldexpf(1.0f + (h3 & 0x7FFFFF) * 0x1p-23f, static_cast<int>((h3 >> 23) % 48) - 27);
        float ref;
        {
#pragma clang fp contract(off)
            ref = nu / de;
        }
        const float got = dw::div_box(nu, de);
        if (__float_as_uint(ref) != __float_as_uint(got)) {
            atomicAdd(bad, 1ull);
            atomicMin(first, static_cast<unsigned long long>(i));
        }
    }
}

int main(int argc, char **argv) {
    const uint64_t pairs = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 32);
    unsigned long long *dbad, hbad[2] = {0, 0}, *dfirst, hfirst = ~0ull;
    unsigned int *dfs, hfs = ~0u;
    hipMalloc(&dbad, 16);
    hipMalloc(&dfirst, 8);
    hipMalloc(&dfs, 4);
    hipMemcpy(dbad, hbad, 16, hipMemcpyHostToDevice);
    hipMemcpy(dfirst, &hfirst, 8, hipMemcpyHostToDevice);
    hipMemcpy(dfs, &hfs, 4, hipMemcpyHostToDevice);
    const float lo = 0x1p-96f, hi = 0x1p20f;
    uint32_t blo, bhi;
    memcpy(&blo, &lo, 4);
    memcpy(&bhi, &hi, 4);
    hipLaunchKernelGGL(k_sqrt, dim3(16384), dim3(256), 0, 0, blo, bhi, dbad, dfs);
    hipLaunchKernelGGL(k_div, dim3(16384), dim3(256), 0, 0, pairs, dbad + 1, dfirst);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("HIP error\n");
        return 2;
    }
    hipMemcpy(hbad, dbad, 16, hipMemcpyDeviceToHost);
    hipMemcpy(&hfirst, dfirst, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&hfs, dfs, 4, hipMemcpyDeviceToHost);
    printf("sqrt_box: %u values in [2^-96, 2^20] and +0: %llu mismatches", bhi - blo + 2, hbad[0]);
    if (hbad[0]) printf(" (first x bits 0x%08x)", hfs);
    printf("\ndiv_box: %llu random pairs: %llu mismatches", (unsigned long long)pairs, hbad[1]);
    if (hbad[1]) printf(" (first pair %llu)", hfirst);
    printf("\n");
    return (hbad[0] || hbad[1]) ? 1 : 0;
}
