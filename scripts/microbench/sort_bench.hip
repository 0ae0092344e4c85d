// Microbenchmark: device radix sort of SGNS gradient records (key = output row, 20-21 bits;
// value = 64-bit {centre id, coefficient}) — sizing the atomic-free out-table gradient path.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void fill(uint32_t* k, uint64_t* v, int n, uint32_t mask) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { uint32_t x = i * 2654435761u; x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15; k[i] = x & mask; v[i] = i; }
}
__global__ void hist(const uint32_t* k, int n, uint32_t* cnt) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) atomicAdd(cnt + k[i], 1u);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 34406400;
  const int bits = 20;
  uint32_t *k0, *k1, *cnt; uint64_t *v0, *v1; uint32_t *u0, *u1;
  CK(hipMalloc(&k0, n * 4)); CK(hipMalloc(&k1, n * 4)); CK(hipMalloc(&v0, n * 8)); CK(hipMalloc(&v1, n * 8));
  CK(hipMalloc(&u0, n * 4)); CK(hipMalloc(&u1, n * 4)); CK(hipMalloc(&cnt, (1 << bits) * 4));
  hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, 0, k0, v0, n, (1u << bits) - 1);
  size_t tb = 0, tb2 = 0;
  CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k0, k1, v0, v1, n, 0, bits));
  CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, k0, k1, u0, u1, n, 0, bits));
  void* tmp; CK(hipMalloc(&tmp, tb > tb2 ? tb : tb2));
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int variant = 0; variant < 3; ++variant) {
    float best = 1e9;
    for (int it = 0; it < 6; ++it) {
      hipEventRecord(a);
      if (variant == 0) CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, k0, k1, v0, v1, n, 0, bits));
      else if (variant == 1) CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb2, k0, k1, u0, u1, n, 0, bits));
      else { hipMemsetAsync(cnt, 0, (1 << bits) * 4); hipLaunchKernelGGL(hist, dim3((n + 255) / 256), dim3(256), 0, 0, k0, n, cnt); }
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b); if (it > 0 && ms < best) best = ms;
    }
    const char* names[] = {"SortPairs u32 key(20b) + u64 value", "SortPairs u32 key(20b) + u32 value", "atomic histogram u32 (counting-sort pass 1)"};
    printf("%-48s n=%d  %.3f ms  %.2f Gitems/s\n", names[variant], n, best, n / best / 1e6);
  }
  return 0;
}
