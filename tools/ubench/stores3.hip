// Store floor of the fused kernel's exact pattern (768-thread workgroups, 512
// of them, grid-stride over 8-entry thread-steps, 12 rows, one 8-B nontemporal
// store per lane per row) as a function of the row stride ld: rows page
// aligned (Engine.alloc_lists: 1.25e8 rounded up to 4 KiB) plus a pad that
// moves each row's start relative to the DRAM channel / bank interleave.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <typename T>
__global__ void __launch_bounds__(768) k_rows(unsigned char *L, size_t ld, unsigned nunit) {
  const unsigned stride = gridDim.x * 768;
  for (unsigned u = blockIdx.x * 768 + threadIdx.x; u < nunit; u += stride) {
#pragma unroll
    for (int g = 0; g < 12; ++g) {
      T v;
      unsigned *pv = reinterpret_cast<unsigned *>(&v);
      for (int i = 0; i < (int)(sizeof(T) / 4); ++i) pv[i] = u * 0x9E3779B9u + g + i;
      __builtin_nontemporal_store(v, reinterpret_cast<T *>(L + g * ld) + u);
    }
  }
}

template <typename T>
static float run(unsigned char *L, size_t ld, size_t entries, int grid) {
  const unsigned nunit = (unsigned)(entries / sizeof(T));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_rows<T>, dim3(grid), dim3(768), 0, 0, L, ld, nunit);
  (void)hipEventRecord(a);
  for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(k_rows<T>, dim3(grid), dim3(768), 0, 0, L, ld, nunit);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 20;
}

int main() {
  const size_t entries = 125000000ull;
  const size_t base = (entries + 4095) / 4096 * 4096;
  unsigned char *L;
  if (hipMalloc(&L, 12 * (base + (1 << 20))) != hipSuccess) return 1;
  // warm the clock
  for (int r = 0; r < 50; ++r) hipLaunchKernelGGL(k_rows<v2u>, dim3(512), dim3(768), 0, 0, L, base, (unsigned)(entries / 8));
  (void)hipDeviceSynchronize();
  const size_t pads[] = {0, 256, 512, 1024, 2048, 4096, 8192, 12288, 16384, 24576, 32768, 65536, 98304, 131072,
                         262144, 0};
  for (size_t pad : pads) {
    const size_t ld = base + pad;
    const float t2 = run<v2u>(L, ld, entries, 512);
    const float t4 = run<v4u>(L, ld, entries, 512);
    printf("ld = base + %7zu (ld mod 64K = %6zu)  x2 %.3f ms %.2f TB/s   x4 %.3f ms %.2f TB/s\n", pad,
           ld % 65536, t2, 12.0 * entries / (t2 * 1e-3) / 1e12, t4, 12.0 * entries / (t4 * 1e-3) / 1e12);
  }
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  for (int r = 0; r < 20; ++r) (void)hipMemsetAsync(L, r, 12 * entries);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  printf("hipMemset 12 x 1.25e8 B  %.3f ms  %.2f TB/s\n", ms / 20, 12.0 * entries / (ms / 20 * 1e-3) / 1e12);
  (void)hipFree(L);
  return 0;
}
