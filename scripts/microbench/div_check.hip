// Is x / c (IEEE fp32 division) equal, bit for bit, to the Markstein form
//   q = x * y;  r = fma(-c, q, x);  q' = fma(r, y, q)      (y = RN(1 / c))
// for the Adam step's uniform divisor c = bias_correction2_sqrt(t) = fp32(sqrt(1 - beta2^t))
// and x = sqrt(v) over the exponent range the replays see? Checks every step t in [1, T] with
// N random x per step (exponents uniform in [-64, 64], random mantissas, plus zero), and
// prints the mismatch count (0 = the form may replace the division there).
//   hipcc -O3 --offload-arch=gfx950 scripts/microbench/div_check.hip -o scripts/microbench/div_check
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ uint32_t hash32(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return static_cast<uint32_t>(x);
}

__global__ void k_check(const float *cs, const float *ys, int64_t T, int64_t per,
                        unsigned long long *bad, unsigned long long *first) {
    const int64_t n = T * per;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t t = i / per;
        const float c = cs[t], y = ys[t];
        const uint32_t h = hash32(static_cast<uint64_t>(i) * 0x9E3779B97F4A7C15ull + 1);
        const uint32_t h2 = hash32(static_cast<uint64_t>(i) ^ 0xD1B54A32D192ED03ull);
        // exponent in [-64, 64], mantissa random; 1 in 4096 is zero
        float x = ldexpf(1.0f + (h & 0x7FFFFF) * 0x1p-23f, static_cast<int>(h2 % 129) - 64);
        if ((h2 >> 20) == 0) x = 0.f;
        float qd;
        {
#pragma clang fp contract(off)
            qd = x / c;
        }
        const float q0 = x * y;
        const float r = fmaf(-c, q0, x);
        const float q1 = fmaf(r, y, q0);
        if (__float_as_uint(q1) != __float_as_uint(qd)) {
            atomicAdd(bad, 1ull);
            atomicMin(first, static_cast<unsigned long long>(i));
        }
    }
}

int main(int argc, char **argv) {
    const int64_t T = argc > 1 ? atoll(argv[1]) : 200000;
    const int64_t per = argc > 2 ? atoll(argv[2]) : 65536;
    const double b2 = argc > 3 ? atof(argv[3]) : 0.999;
    float *hc = (float *)malloc(T * 4), *hy = (float *)malloc(T * 4);
    for (int64_t t = 0; t < T; ++t) {
        // the host's scalars (sharding.adam_scalars): float64 math, cast to float32
        hc[t] = static_cast<float>(sqrt(1.0 - pow(b2, static_cast<double>(t + 1))));
        volatile float one = 1.0f;
        hy[t] = one / hc[t];   // RN(1 / c) in fp32
    }
    float *dc, *dy;
    unsigned long long *dbad, *dfirst, hbad = 0, hfirst = ~0ull;
    hipMalloc(&dc, T * 4);
    hipMalloc(&dy, T * 4);
    hipMalloc(&dbad, 8);
    hipMalloc(&dfirst, 8);
    hipMemcpy(dc, hc, T * 4, hipMemcpyHostToDevice);
    hipMemcpy(dy, hy, T * 4, hipMemcpyHostToDevice);
    hipMemcpy(dbad, &hbad, 8, hipMemcpyHostToDevice);
    hipMemcpy(dfirst, &hfirst, 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_check, dim3(8192), dim3(256), 0, 0, dc, dy, T, per, dbad, dfirst);
    hipMemcpy(&hbad, dbad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&hfirst, dfirst, 8, hipMemcpyDeviceToHost);
    printf("beta2 %.6f steps %lld x per step %lld: %llu mismatches", b2, (long long)T,
           (long long)per, hbad);
    if (hbad) printf(" (first at step %llu)", hfirst / per + 1);
    printf("\n");
    return hbad ? 1 : 0;
}
