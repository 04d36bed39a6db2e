// LDS atomic-histogram microbenchmark: cycles per ds_add_u32 wave-instruction
// for the count-mode bin pattern (random (u, x) per lane, fixed group g per
// instruction), half the lanes active, with R lane-interleaved replicas whose
// bank is fixed by lane % R (bank = (x + (lane % R) * 32 / R) mod 32).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int R, bool HALF>
__global__ void __launch_bounds__(512) k_hist(unsigned *out, unsigned seed, int iters) {
  __shared__ unsigned h[R * 3264];
  for (int i = threadIdx.x; i < R * 3264; i += 512) h[i] = 0;
  __syncthreads();
  unsigned x = (threadIdx.x + blockIdx.x * 512) * 2654435761u ^ seed;
  const unsigned lane = threadIdx.x & 63;
  const unsigned rep = lane % R;
  for (int it = 0; it < iters; ++it) {
    x = x * 1664525u + 1013904223u;
    const unsigned u = x >> 28;
    const bool act = !HALF || ((x >> 27) & 1);
    if (act) {
#pragma unroll
      for (int g = 0; g < 11; ++g) {
        const unsigned v = (x >> (2 * g)) & 15;
        // bin (u, g, v): row of 16 bins, replicas interleaved inside a 32-word bank line
        unsigned idx;
        if (R == 1) idx = (u * 12 + g) * 17 + v;
        else idx = ((u * 12 + g) * 16 + v) * R + rep;  // word address: bank = (v*R + rep) % 32
        atomicAdd(&h[idx], 1u);
      }
    }
  }
  __syncthreads();
  out[blockIdx.x * 512 + threadIdx.x] = h[threadIdx.x];
}

template <int R, bool HALF>
static void run(unsigned *out) {
  const int blocks = 256 * 3, iters = 512;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL((k_hist<R, HALF>), dim3(blocks), dim3(512), 0, 0, out, 7u, iters);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL((k_hist<R, HALF>), dim3(blocks), dim3(512), 0, 0, out, 7u, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  // per CU: 3 blocks * 8 waves * iters * 11 instructions
  const double instr = 3.0 * 8 * iters * 11;
  printf("R=%d half=%d  %.3f ms  %.2f LDS cycles per ds_add (at 2.4 GHz, per CU)\n", R, HALF, ms,
         ms * 1e-3 * 2.4e9 / instr);
}

int main() {
  unsigned *out;
  (void)hipMalloc(&out, 256 * 3 * 512 * 4);
  run<1, false>(out);
  run<1, true>(out);
  run<2, true>(out);
  run<4, true>(out);
  run<2, false>(out);
  run<4, false>(out);
  return 0;
}
