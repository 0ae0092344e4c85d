// How far is the raw v_sqrt_f32 (__builtin_amdgcn_sqrtf) from the correctly rounded sqrtf over
// the lazy replays' box range (every fp32 x in [2^-96, 2^20], exhaustive, ~9.7e8 values)?
// Counts: raw == sqrtf; sqrtf one ulp below raw; one ulp above; anything else. If one side
// never occurs, dw::sqrt_box needs only the other side's correction.
//   hipcc -O3 --offload-arch=gfx950 scripts/microbench/sqrt_raw_check.hip \
//         -o scripts/microbench/sqrt_raw_check
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

__global__ void k_count(uint32_t lo, uint32_t hi, unsigned long long *cnt, unsigned int *first) {
    const uint64_t n = static_cast<uint64_t>(hi - lo) + 1;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    unsigned long long c[4] = {0, 0, 0, 0};
    for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
         i += stride) {
        const uint32_t b = lo + static_cast<uint32_t>(i);
        const float x = __uint_as_float(b);
        const uint32_t ref = __float_as_uint(sqrtf(x));
        const uint32_t raw = __float_as_uint(__builtin_amdgcn_sqrtf(x));
        const int k = raw == ref ? 0 : ref + 1u == raw ? 1 : ref == raw + 1u ? 2 : 3;
        ++c[k];
        if (k == 3) atomicMin(first, b);
    }
    for (int k = 0; k < 4; ++k)
        if (c[k]) atomicAdd(cnt + k, c[k]);
}

int main() {
    unsigned long long *dc, hc[4] = {0, 0, 0, 0};
    unsigned int *df, hf = ~0u;
    hipMalloc(&dc, sizeof(hc));
    hipMalloc(&df, 4);
    hipMemcpy(dc, hc, sizeof(hc), hipMemcpyHostToDevice);
    hipMemcpy(df, &hf, 4, hipMemcpyHostToDevice);
    const float lo = 0x1p-96f, hi = 0x1p20f;
    uint32_t blo, bhi;
    memcpy(&blo, &lo, 4);
    memcpy(&bhi, &hi, 4);
    hipLaunchKernelGGL(k_count, dim3(8192), dim3(256), 0, 0, blo, bhi, dc, df);
    hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost);
    hipMemcpy(&hf, df, 4, hipMemcpyDeviceToHost);
    printf("raw v_sqrt_f32 over [2^-96, 2^20] (%llu values): exact %llu, one ulp above %llu, "
           "one ulp below %llu, other %llu (first other bits 0x%08x)\n",
           hc[0] + hc[1] + hc[2] + hc[3], hc[0], hc[1], hc[2], hc[3], hf);
    return hc[3] ? 1 : 0;
}
