// Exhaustive check of the reciprocal division the lazy replays and the graphed steps use for
// sqrt(v) / sqrt(bias_correction2) (dw_common.h dw::div_bc2s):
//   q = x * y;  r = fma(-c, q, x);  q' = fma(r, y, q)      (y = RN(1 / c), from the host)
// against the IEEE fp32 division x / c, for EVERY fp32 x in [1, 2) (all 2^23 mantissas) and
// x = 0, for every (c, y) pair in the input file (float32 pairs, as sharding.hist_row writes them
// for each step until c rounds to 1). Scaling x by 2^k is exact in every operation of both forms
// while x stays in [2^-64, 2^64] (c in [2^-10, 1]: no product leaves the normal range), so x in
// [1, 2) covers the whole range div_bc2s accepts. Prints one JSON line: pairs, checks, mismatches.
//   hipcc -O3 --offload-arch=gfx950 scripts/microbench/div_proof.hip -o scripts/microbench/div_proof
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void k_proof(const float2 *pairs, int64_t n_pairs, unsigned long long *bad,
                        unsigned long long *first) {
    // one thread per mantissa chunk of 64, looping over pairs in the grid's y dimension
    const int64_t pair = blockIdx.y;
    if (pair >= n_pairs) return;
    const float c = pairs[pair].x, y = pairs[pair].y;
    const uint32_t m0 = (blockIdx.x * blockDim.x + threadIdx.x) * 64u;
    unsigned long long nb = 0;
    for (uint32_t k = 0; k < 64; ++k) {
        const uint32_t mant = m0 + k;
        if (mant >= (1u << 23)) break;
        const float x = __uint_as_float(0x3F800000u | mant);
        float qd;
        {
#pragma clang fp contract(off)
            qd = x / c;
        }
        const float q0 = x * y;
        const float r = fmaf(-c, q0, x);
        const float q1 = fmaf(r, y, q0);
        if (__float_as_uint(q1) != __float_as_uint(qd)) ++nb;
    }
    if (m0 == 0) {   // x = 0 (and -0 is never a sqrt of v >= +0)
        const float x = 0.f;
        float qd;
        {
#pragma clang fp contract(off)
            qd = x / c;
        }
        const float q0 = x * y;
        const float q1 = fmaf(fmaf(-c, q0, x), y, q0);
        if (__float_as_uint(q1) != __float_as_uint(qd)) ++nb;
    }
    if (nb) {
        atomicAdd(bad, nb);
        atomicMin(first, static_cast<unsigned long long>(pair));
    }
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: div_proof pairs.bin\n");
        return 2;
    }
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    fseek(f, 0, SEEK_END);
    const long bytes = ftell(f);
    fseek(f, 0, SEEK_SET);
    const int64_t n = bytes / 8;
    float2 *h = (float2 *)malloc(n * 8);
    if (fread(h, 8, n, f) != (size_t)n) return 2;
    fclose(f);
    float2 *d;
    unsigned long long *dbad, *dfirst, hbad = 0, hfirst = ~0ull;
    hipMalloc(&d, n * 8);
    hipMalloc(&dbad, 8);
    hipMalloc(&dfirst, 8);
    hipMemcpy(d, h, n * 8, hipMemcpyHostToDevice);
    hipMemcpy(dbad, &hbad, 8, hipMemcpyHostToDevice);
    hipMemcpy(dfirst, &hfirst, 8, hipMemcpyHostToDevice);
    // 2^23 mantissas / 64 per thread / 256 threads = 512 blocks per pair; pairs in slices of
    // 4096 along y
    for (int64_t p0 = 0; p0 < n; p0 += 4096) {
        const int64_t np = n - p0 < 4096 ? n - p0 : 4096;
        hipLaunchKernelGGL(k_proof, dim3(512, (unsigned)np), dim3(256), 0, 0, d + p0, np, dbad,
                           dfirst);
        if (hipDeviceSynchronize() != hipSuccess) return 3;
        fprintf(stderr, "pairs %lld / %lld\n", (long long)(p0 + np), (long long)n);
    }
    hipMemcpy(&hbad, dbad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&hfirst, dfirst, 8, hipMemcpyDeviceToHost);
    printf("{\"pairs\": %lld, \"checks\": %lld, \"mismatches\": %llu, \"first_bad_pair\": %lld}\n",
           (long long)n, (long long)n * ((1ll << 23) + 1), hbad,
           hbad ? (long long)hfirst : -1ll);
    return hbad ? 1 : 0;
}
