// Random-line roofline for the walkers (profiles/r02_random_lines.json; bench.py reads it).
//
//   hipcc --offload-arch=gfx950 -O3 -o random_lines scripts/microbench/random_lines.hip
//   ./random_lines [table_MiB ...]
//
// A Philox DeepWalk step over the edge-inline CSR is one dependent 16-B load at a random place of
// a 306 MiB table (C3; 8 GiB at C5). Its ceiling is set by how many random lines the chip fetches
// per second, not by HBM bytes. Two shapes over a table of int4 entries:
//   * gather: every lane issues 32 independent 16-B loads at hashed entries (no dependence), a
//     grid far beyond the resident waves — the chip's random-line fetch rate;
//   * chase: 1,048,576 chains, one lane each, 79 dependent steps entry = table[entry.x]
//     (a random functional graph; the walker's access pattern without its Philox arithmetic).
// Prints one JSON line per table size: lines/s of each shape.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

__global__ void k_fill(int4 *t, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t h = mix(static_cast<uint32_t>(i) * 2654435761u + 12345u);
        t[i] = int4{static_cast<int32_t>((uint64_t)h * (uint64_t)n >> 32), 1, 2, 3};
    }
}

constexpr int LOADS = 32;

__global__ void __launch_bounds__(256) k_gather(const int4 *__restrict__ t, int64_t n,
                                                int32_t *sink) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    int32_t acc = 0;
#pragma unroll
    for (int k = 0; k < LOADS; ++k) {
        const uint32_t h = mix(g * LOADS + k);
        acc ^= t[(uint64_t)h * (uint64_t)n >> 32].x;
    }
    if (acc == 0x7fffffff) sink[0] = acc;
}

__global__ void __launch_bounds__(256) k_chase(const int4 *__restrict__ t, int64_t n,
                                               int64_t chains, int steps, int32_t *out) {
    const int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (c >= chains) return;
    int32_t v = static_cast<int32_t>((uint64_t)mix(static_cast<uint32_t>(c)) * (uint64_t)n >> 32);
    for (int s = 0; s < steps; ++s) v = t[v].x;
    out[c] = v;
}

int main(int argc, char **argv) {
    std::vector<int64_t> mibs;
    for (int i = 1; i < argc; ++i) mibs.push_back(atoll(argv[i]));
    if (mibs.empty()) mibs = {306, 1224, 8192};
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    int32_t *sink;
    const int64_t chains = 1 << 20;
    const int steps = 79;
    CHECK(hipMalloc(&sink, chains * sizeof(int32_t)));
    for (int64_t mib : mibs) {
        const int64_t n = mib * (1 << 20) / 16;
        int4 *t;
        CHECK(hipMalloc(&t, n * 16));
        hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, t, n);
        CHECK(hipDeviceSynchronize());
        const int blocks = 256 * 64;   // 4M lanes x 32 loads = 134M random lines
        float best_g = 1e30f, best_c = 1e30f, ms = 0.f;
        for (int rep = 0; rep < 4; ++rep) {
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(k_gather, dim3(blocks), dim3(256), 0, 0, t, n, sink);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            CHECK(hipEventElapsedTime(&ms, a, b));
            if (rep > 0 && ms < best_g) best_g = ms;
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(k_chase, dim3((chains + 255) / 256), dim3(256), 0, 0, t, n, chains,
                               steps, sink);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            CHECK(hipEventElapsedTime(&ms, a, b));
            if (rep > 0 && ms < best_c) best_c = ms;
        }
        const double g_lines = (double)blocks * 256 * LOADS / (best_g * 1e-3);
        const double c_lines = (double)chains * steps / (best_c * 1e-3);
        printf("{\"table_MiB\": %lld, \"gather_lines_per_s\": %.4g, \"gather_ms\": %.4f, "
               "\"chase_chains\": %lld, \"chase_steps\": %d, \"chase_lines_per_s\": %.4g, "
               "\"chase_ms\": %.4f}\n",
               (long long)mib, g_lines, best_g, (long long)chains, steps, c_lines, best_c);
        fflush(stdout);
        CHECK(hipFree(t));
    }
    return 0;
}
