// LDS histogram layouts for the count-mode H bins (n = 11: 11 counted groups
// per Q entry, half the lanes Q), same number of entries in every variant:
//  single: H[u][g][x] (rows of 17 words), 11 ds_add_u32 per Q entry,
//          512-thread workgroups, 3 per CU (the fused kernel today);
//  pair:   H2[u][p][x][x'] for 5 group pairs + H[u][11][x], 6 ds_add_u32 per
//          Q entry, one 1024-thread workgroup per CU (83 KB of bins).
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ unsigned nextr(unsigned &x) {
  x = x * 1664525u + 1013904223u;
  return x;
}

template <int BS>
__global__ void __launch_bounds__(BS) k_single(unsigned *out, unsigned seed, int entries) {
  extern __shared__ unsigned h[];
  constexpr int NB = 16 * 12 * 17;
  for (int i = threadIdx.x; i < NB; i += BS) h[i] = 0;
  __syncthreads();
  unsigned x = (threadIdx.x + blockIdx.x * BS) * 2654435761u ^ seed;
  for (int it = 0; it < entries; ++it) {
    const unsigned r = nextr(x), v = r ^ (r >> 7) * 0x9E3779B9u;
    if (r >> 31) {
      const unsigned u = (v >> 28) & 15;
#pragma unroll
      for (int g = 0; g < 11; ++g) atomicAdd(&h[(u * 12 + g) * 17 + ((v >> (2 * g)) & 15)], 1u);
    }
  }
  __syncthreads();
  out[blockIdx.x * BS + threadIdx.x] = h[threadIdx.x % NB];
}

template <int BS>
__global__ void __launch_bounds__(BS) k_pair(unsigned *out, unsigned seed, int entries) {
  extern __shared__ unsigned h[];
  constexpr int NB = 16 * 5 * 256 + 16 * 16;
  for (int i = threadIdx.x; i < NB; i += BS) h[i] = 0;
  __syncthreads();
  unsigned x = (threadIdx.x + blockIdx.x * BS) * 2654435761u ^ seed;
  for (int it = 0; it < entries; ++it) {
    const unsigned r = nextr(x), v = r ^ (r >> 7) * 0x9E3779B9u;
    if (r >> 31) {
      const unsigned u = (v >> 28) & 15;
#pragma unroll
      for (int p = 0; p < 5; ++p) atomicAdd(&h[(u * 5 + p) * 256 + ((v >> (3 * p)) & 255)], 1u);
      atomicAdd(&h[16 * 5 * 256 + u * 16 + ((v >> 20) & 15)], 1u);
    }
  }
  __syncthreads();
  out[blockIdx.x * BS + threadIdx.x] = h[threadIdx.x % NB];
}

template <typename K>
static float timeit(K kern, int grid, int bs, size_t lds, unsigned *out, int entries) {
  (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(bs), lds, 0, out, 7u, entries);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(bs), lds, 0, out, 7u, entries);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  unsigned *out;
  (void)hipMalloc(&out, 256 * 4 * 1024 * 4);
  const double total = 1.25e8;  // entries per launch, like the headline shard
  {
    const int grid = 256 * 3, bs = 512;
    const int e = (int)(total / (grid * bs));
    const float ms = timeit(k_single<512>, grid, bs, 16 * 12 * 17 * 4, out, e);
    printf("single 11 atomics, 3 x 512 per CU:  %.3f ms (%d entries/thread)\n", ms, e);
  }
  {
    const int grid = 256, bs = 1024;
    const int e = (int)(total / (grid * bs));
    const float ms = timeit(k_pair<1024>, grid, bs, (16 * 5 * 256 + 256) * 4, out, e);
    printf("pair    6 atomics, 1 x 1024 per CU: %.3f ms (%d entries/thread)\n", ms, e);
  }
  {
    const int grid = 256 * 2, bs = 512;
    const int e = (int)(total / (grid * bs));
    const float ms = timeit(k_single<512>, grid, bs, 16 * 12 * 17 * 4 + 40000, out, e);
    printf("single 11 atomics, 2 x 512 per CU:  %.3f ms (%d entries/thread)\n", ms, e);
  }
  {
    const int grid = 256, bs = 1024;
    const int e = (int)(total / (grid * bs));
    const float ms = timeit(k_single<1024>, grid, bs, 16 * 12 * 17 * 4 + 90000, out, e);
    printf("single 11 atomics, 1 x 1024 per CU: %.3f ms (%d entries/thread)\n", ms, e);
  }
  return 0;
}
