// Store-pattern microbenchmark: 12 rows x S bytes (the fused kernel's list
// layout), each thread writing 4, 8 or 16 bytes per row per step.
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T>
__global__ void __launch_bounds__(512) k_rows(unsigned char *L, size_t ld, unsigned nvec) {
  for (unsigned q = blockIdx.x * 512 + threadIdx.x; q < nvec; q += gridDim.x * 512) {
#pragma unroll
    for (int g = 0; g < 12; ++g) {
      T v;
      unsigned *pv = reinterpret_cast<unsigned *>(&v);
      for (int i = 0; i < (int)(sizeof(T) / 4); ++i) pv[i] = q * 0x9E3779B9u + g + i;
      reinterpret_cast<T *>(L + g * ld)[q] = v;
    }
  }
}

template <typename T>
static void run(const char *name, unsigned char *L, size_t ld, size_t entries, int grid) {
  const unsigned nvec = (unsigned)(entries / sizeof(T));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k_rows<T>, dim3(grid), dim3(512), 0, 0, L, ld, nvec);
  (void)hipEventRecord(a);
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(k_rows<T>, dim3(grid), dim3(512), 0, 0, L, ld, nvec);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  ms /= 10;
  printf("%-8s grid %5d  %.3f ms  %.2f TB/s\n", name, grid, ms, 12.0 * entries / (ms * 1e-3) / 1e12);
}

int main() {
  const size_t entries = 125000000ull / 64 * 64, ld = entries;
  unsigned char *L;
  if (hipMalloc(&L, 12 * ld) != hipSuccess) return 1;
  for (int grid : {768, 2048, 8192}) {
    run<unsigned>("dword", L, ld, entries, grid);
    run<uint2>("dwordx2", L, ld, entries, grid);
    run<uint4>("dwordx4", L, ld, entries, grid);
  }
  (void)hipFree(L);
  return 0;
}
