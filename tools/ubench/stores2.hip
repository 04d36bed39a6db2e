// Write-bandwidth ceiling for the list layout: 12 rows x S bytes.
//  grid-stride (the fused kernel's order) vs workgroup-contiguous column
//  ranges, default vs nontemporal stores, 4/8/16-B vectors, and one
//  contiguous row of the same bytes as the plain-streaming reference.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <typename T, bool NT>
__device__ __forceinline__ void st(T *p, T v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <typename T>
__device__ __forceinline__ T mk(unsigned q, int g) {
  T v;
  unsigned *pv = reinterpret_cast<unsigned *>(&v);
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) pv[i] = q * 0x9E3779B9u + g + i;
  return v;
}

template <typename T, bool NT, int ROWS>
__global__ void __launch_bounds__(512) k_stride(unsigned char *L, size_t ld, unsigned nvec) {
  for (unsigned q = blockIdx.x * 512 + threadIdx.x; q < nvec; q += gridDim.x * 512) {
#pragma unroll
    for (int g = 0; g < ROWS; ++g) st<T, NT>(reinterpret_cast<T *>(L + g * ld) + q, mk<T>(q, g));
  }
}

// 8 B per lane of data, stored as 16 B by one lane of each lane pair (the
// pair's partner row alternates with the row parity): 32 lanes x 16 B per row
template <bool NT, int ROWS>
__global__ void __launch_bounds__(512) k_pairx4(unsigned char *L, size_t ld, unsigned nvec8) {
  for (unsigned q = blockIdx.x * 512 + threadIdx.x; q < nvec8; q += gridDim.x * 512) {
    const unsigned par = threadIdx.x & 1;
#pragma unroll
    for (int g = 0; g < ROWS; ++g) {
      if ((unsigned)(g & 1) == par) {
        v4u v = mk<v4u>(q, g);
        st<v4u, NT>(reinterpret_cast<v4u *>(L + g * ld + (size_t)(q & ~1u) * 8), v);
      }
    }
  }
}

// workgroup b owns vectors [b*per, (b+1)*per) of every row
template <typename T, bool NT, int ROWS>
__global__ void __launch_bounds__(512) k_block(unsigned char *L, size_t ld, unsigned nvec) {
  const unsigned per = (nvec + gridDim.x - 1) / gridDim.x;
  const unsigned q0 = blockIdx.x * per, q1 = q0 + per < nvec ? q0 + per : nvec;
  for (unsigned q = q0 + threadIdx.x; q < q1; q += 512) {
#pragma unroll
    for (int g = 0; g < ROWS; ++g) st<T, NT>(reinterpret_cast<T *>(L + g * ld) + q, mk<T>(q, g));
  }
}

static float timeit(void (*launch)(unsigned char *, size_t, unsigned, int), unsigned char *L, size_t ld,
                    unsigned nvec, int grid) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  launch(L, ld, nvec, grid);
  (void)hipEventRecord(a);
  for (int r = 0; r < 10; ++r) launch(L, ld, nvec, grid);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 10;
}

template <typename T, bool NT, int ROWS, bool BLOCK>
static void go(const char *name, unsigned char *L, size_t bytes_per_row, int grid) {
  const unsigned nvec = (unsigned)(bytes_per_row / sizeof(T));
  auto launch = [](unsigned char *L, size_t ld, unsigned nvec, int grid) {
    if (BLOCK)
      hipLaunchKernelGGL((k_block<T, NT, ROWS>), dim3(grid), dim3(512), 0, 0, L, ld, nvec);
    else
      hipLaunchKernelGGL((k_stride<T, NT, ROWS>), dim3(grid), dim3(512), 0, 0, L, ld, nvec);
  };
  const float ms = timeit(launch, L, bytes_per_row, nvec, grid);
  printf("%-28s grid %5d  %.3f ms  %.2f TB/s\n", name, grid, ms,
         (double)ROWS * bytes_per_row / (ms * 1e-3) / 1e12);
}

template <bool NT>
static void go_pair(const char *name, unsigned char *L, size_t bytes_per_row, int grid) {
  const unsigned nvec8 = (unsigned)(bytes_per_row / 8);
  auto launch = [](unsigned char *L, size_t ld, unsigned nvec, int grid) {
    hipLaunchKernelGGL((k_pairx4<NT, 12>), dim3(grid), dim3(512), 0, 0, L, ld, nvec);
  };
  const float ms = timeit(launch, L, bytes_per_row, nvec8, grid);
  printf("%-28s grid %5d  %.3f ms  %.2f TB/s\n", name, grid, ms, 12.0 * bytes_per_row / (ms * 1e-3) / 1e12);
}

int main() {
  const size_t entries = 125000000ull / 64 * 64;
  unsigned char *L;
  if (hipMalloc(&L, 12 * entries) != hipSuccess) return 1;
  for (int grid : {768, 1024, 4096}) {
    go<v2u, false, 12, false>("12row x2 stride", L, entries, grid);
    go<v2u, true, 12, false>("12row x2 stride nt", L, entries, grid);
    go<v4u, false, 12, false>("12row x4 stride", L, entries, grid);
    go<v4u, true, 12, false>("12row x4 stride nt", L, entries, grid);
    go<v2u, false, 12, true>("12row x2 block", L, entries, grid);
    go<v2u, true, 12, true>("12row x2 block nt", L, entries, grid);
    go<v4u, true, 12, true>("12row x4 block nt", L, entries, grid);
    go<v4u, false, 1, false>("1row x4 stride", L, 12 * entries, grid);
    go<v4u, true, 1, false>("1row x4 stride nt", L, 12 * entries, grid);
    go_pair<true>("12row pair-x4 nt", L, entries, grid);
    go_pair<false>("12row pair-x4", L, entries, grid);
  }
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipMemsetAsync(L, 1, 12 * entries);
  (void)hipEventRecord(a);
  for (int r = 0; r < 10; ++r) (void)hipMemsetAsync(L, r, 12 * entries);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  printf("%-28s             %.3f ms  %.2f TB/s\n", "hipMemset", ms / 10, 12.0 * entries / (ms / 10 * 1e-3) / 1e12);
  (void)hipFree(L);
  return 0;
}
