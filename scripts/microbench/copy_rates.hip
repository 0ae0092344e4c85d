// STREAM-copy variants on one MI355X: which kernel shape measures the HBM copy ceiling that
// bench.py reports as `measured_copy_GBps` (dw_stream_copy).
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/microbench/copy_rates scripts/microbench/copy_rates.hip
//   ./scripts/microbench/copy_rates [MiB]
//
// Prints one JSON line per variant: bytes read + written per second, best of 10 launches.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

// (a) grid-stride, four float4 per lane per trip (the round-3 dw_stream_copy)
__global__ void k_stride4(const float4 *__restrict__ s, float4 *__restrict__ d, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const float4 a = s[i], b = s[i + stride], c = s[i + 2 * stride], e = s[i + 3 * stride];
        d[i] = a;
        d[i + stride] = b;
        d[i + 2 * stride] = c;
        d[i + 3 * stride] = e;
    }
    for (; i < n; i += stride) d[i] = s[i];
}

// (b) one tile of 256 x U float4 per block, a grid over the whole array; NT = nontemporal
template <int U, bool NT>
__global__ void __launch_bounds__(256) k_tile(const float4 *__restrict__ s, float4 *__restrict__ d,
                                              int64_t n) {
    const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
    float4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + u * 256;
        if (i < n) {
            if (NT) {
                r[u].x = __builtin_nontemporal_load(&s[i].x);
                r[u].y = __builtin_nontemporal_load(&s[i].y);
                r[u].z = __builtin_nontemporal_load(&s[i].z);
                r[u].w = __builtin_nontemporal_load(&s[i].w);
            } else {
                r[u] = s[i];
            }
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t i = base + u * 256;
        if (i < n) {
            if (NT) {
                __builtin_nontemporal_store(r[u].x, &d[i].x);
                __builtin_nontemporal_store(r[u].y, &d[i].y);
                __builtin_nontemporal_store(r[u].z, &d[i].z);
                __builtin_nontemporal_store(r[u].w, &d[i].w);
            } else {
                d[i] = r[u];
            }
        }
    }
}

// (c) persistent grid-stride over tiles of 256 x U, NT
template <int U>
__global__ void __launch_bounds__(256) k_tile_stride(const float4 *__restrict__ s,
                                                     float4 *__restrict__ d, int64_t n) {
    const int64_t tiles = (n + 256 * U - 1) / (256 * U);
    for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        const int64_t base = t * 256 * U + threadIdx.x;
        float4 r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + u * 256;
            if (i < n) {
                r[u].x = __builtin_nontemporal_load(&s[i].x);
                r[u].y = __builtin_nontemporal_load(&s[i].y);
                r[u].z = __builtin_nontemporal_load(&s[i].z);
                r[u].w = __builtin_nontemporal_load(&s[i].w);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + u * 256;
            if (i < n) {
                __builtin_nontemporal_store(r[u].x, &d[i].x);
                __builtin_nontemporal_store(r[u].y, &d[i].y);
                __builtin_nontemporal_store(r[u].z, &d[i].z);
                __builtin_nontemporal_store(r[u].w, &d[i].w);
            }
        }
    }
}

template <typename F>
static void run(const char *name, F launch, int64_t bytes) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int r = 0; r < 11; ++r) {
        CHECK(hipEventRecord(e0));
        launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0 && ms < best) best = ms;
    }
    printf("{\"variant\": \"%s\", \"bytes\": %lld, \"ms\": %.4f, \"GBps\": %.1f}\n", name,
           (long long)bytes, best, 2.0 * bytes / (best * 1e-3) / 1e9);
    fflush(stdout);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
}

int main(int argc, char **argv) {
    const int64_t mib = argc > 1 ? atoll(argv[1]) : 2048;
    const int64_t bytes = mib << 20, n = bytes / 16;
    float4 *s, *d;
    CHECK(hipMalloc(&s, bytes));
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMemset(s, 1, bytes));
    CHECK(hipMemset(d, 0, bytes));
    int cu = 256;
    CHECK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
    run("stride4_8pcu", [&] { hipLaunchKernelGGL(k_stride4, dim3(cu * 8), dim3(256), 0, 0, s, d, n); }, bytes);
    run("stride4_32pcu", [&] { hipLaunchKernelGGL(k_stride4, dim3(cu * 32), dim3(256), 0, 0, s, d, n); }, bytes);
    run("tile4", [&] { hipLaunchKernelGGL((k_tile<4, false>), dim3((n + 1023) / 1024), dim3(256), 0, 0, s, d, n); }, bytes);
    run("tile4_nt", [&] { hipLaunchKernelGGL((k_tile<4, true>), dim3((n + 1023) / 1024), dim3(256), 0, 0, s, d, n); }, bytes);
    run("tile8_nt", [&] { hipLaunchKernelGGL((k_tile<8, true>), dim3((n + 2047) / 2048), dim3(256), 0, 0, s, d, n); }, bytes);
    run("tile2_nt", [&] { hipLaunchKernelGGL((k_tile<2, true>), dim3((n + 511) / 512), dim3(256), 0, 0, s, d, n); }, bytes);
    run("tilestride4_nt_8pcu", [&] { hipLaunchKernelGGL((k_tile_stride<4>), dim3(cu * 8), dim3(256), 0, 0, s, d, n); }, bytes);
    run("tilestride4_nt_16pcu", [&] { hipLaunchKernelGGL((k_tile_stride<4>), dim3(cu * 16), dim3(256), 0, 0, s, d, n); }, bytes);
    run("tilestride8_nt_8pcu", [&] { hipLaunchKernelGGL((k_tile_stride<8>), dim3(cu * 8), dim3(256), 0, 0, s, d, n); }, bytes);
    run("hipMemcpyAsync", [&] { CHECK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0)); }, bytes);
    CHECK(hipFree(s));
    CHECK(hipFree(d));
    return 0;
}
