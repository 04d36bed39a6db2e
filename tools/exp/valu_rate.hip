// Issue cost of the list kernel's VALU instruction mix on gfx950, one SIMD
// fully occupied (8 waves): cycles (s_memtime) per wave64 instruction for
// independent streams of v_mad_u64_u32 (Philox's multiply), v_mul_lo_u32,
// v_mul_hi_u32, v_add_u32, v_bitop3_b32, v_perm_b32.  The roofline
// in bench.py's roofline.issue prices every VALU instruction at 2 cycles;
// this says what Philox's 64-bit multiplies really cost.
//   hipcc --offload-arch=gfx950 -O3 -o valu_rate tools/exp/valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP 4096  // long enough that dispatch skew does not dilute the 8-way residency
template <int OP>
__global__ __launch_bounds__(512) void k(uint32_t *out, uint32_t seed, uint64_t *cyc) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u;
  uint32_t a4 = a0 + 11u, a5 = a0 + 13u, a6 = a0 + 17u, a7 = a0 + 19u;
  uint64_t m0 = a0, m1 = a1, m2 = a2, m3 = a3, m4 = a4, m5 = a5, m6 = a6, m7 = a7;
  const uint32_t c = 0xD2511F53u ^ seed;
  uint64_t cc;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int r = 0; r < REP; ++r) {
#define MAD(m, a) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(m), "=s"(cc) : "v"(a), "s"(c))  // carry-out SGPR pair reused, as the compiler does
#define V2(op, a, b) asm volatile(op " %0, %0, %1" : "+v"(a) : "v"(b))
#define V3(op, a, b) asm volatile(op " %0, %0, %1, %1" : "+v"(a) : "v"(b))
#define B3(a, b) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a) : "v"(b))
    if constexpr (OP == 0) {
      MAD(m0, a0); MAD(m1, a1); MAD(m2, a2); MAD(m3, a3); MAD(m4, a4); MAD(m5, a5); MAD(m6, a6); MAD(m7, a7);
    } else if constexpr (OP == 1) {
      V2("v_mul_lo_u32", a0, a4); V2("v_mul_lo_u32", a1, a5); V2("v_mul_lo_u32", a2, a6); V2("v_mul_lo_u32", a3, a7);
      V2("v_mul_lo_u32", a4, a0); V2("v_mul_lo_u32", a5, a1); V2("v_mul_lo_u32", a6, a2); V2("v_mul_lo_u32", a7, a3);
    } else if constexpr (OP == 2) {
      V2("v_mul_hi_u32", a0, a4); V2("v_mul_hi_u32", a1, a5); V2("v_mul_hi_u32", a2, a6); V2("v_mul_hi_u32", a3, a7);
      V2("v_mul_hi_u32", a4, a0); V2("v_mul_hi_u32", a5, a1); V2("v_mul_hi_u32", a6, a2); V2("v_mul_hi_u32", a7, a3);
    } else if constexpr (OP == 3) {
      V2("v_add_u32", a0, a4); V2("v_add_u32", a1, a5); V2("v_add_u32", a2, a6); V2("v_add_u32", a3, a7);
      V2("v_add_u32", a4, a0); V2("v_add_u32", a5, a1); V2("v_add_u32", a6, a2); V2("v_add_u32", a7, a3);
    } else if constexpr (OP == 4) {
      B3(a0, a4); B3(a1, a5); B3(a2, a6); B3(a3, a7); B3(a4, a0); B3(a5, a1); B3(a6, a2); B3(a7, a3);
    } else {
      V3("v_perm_b32", a0, a4); V3("v_perm_b32", a1, a5); V3("v_perm_b32", a2, a6); V3("v_perm_b32", a3, a7);
      V3("v_perm_b32", a4, a0); V3("v_perm_b32", a5, a1); V3("v_perm_b32", a6, a2); V3("v_perm_b32", a7, a3);
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  const uint32_t x = (uint32_t)(m0 ^ m1 ^ m2 ^ m3 ^ m4 ^ m5 ^ m6 ^ m7) ^ a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if ((threadIdx.x & 63) == 0) {
    const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    cyc[2 * w] = t1 - t0;      // shader cycles of this wave's loop
    cyc[2 * w + 1] = r1 - r0;  // the same span in 100 MHz ticks
  }
}

int main() {
  const char *names[] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_add_u32", "v_bitop3_b32", "v_perm_b32"};
  void (*ks[])(uint32_t *, uint32_t, uint64_t *) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>};
  uint32_t *out;
  uint64_t *cyc;
  (void)hipMalloc(&out, (size_t)1024 * 512 * 4);
  (void)hipMalloc(&cyc, (size_t)1024 * 8 * 8 * 2);
  static uint64_t h[1024 * 8 * 2];
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  // (grid, block): 8 waves per SIMD (4 x 512 threads per CU), 1 wave per SIMD (1 x 256 per CU)
  const int cfg[2][2] = {{256 * 4, 512}, {256, 256}};
  for (int c = 0; c < 2; ++c) {
    const int grid = cfg[c][0], bs = cfg[c][1], nw = grid * bs / 64;
    const double wps = nw / 1024.0;
    for (int o = 0; o < 6; ++o) {
      for (int it = 0; it < 2; ++it) hipLaunchKernelGGL(ks[o], dim3(grid), dim3(bs), 0, 0, out, 7u + it, cyc);
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL(ks[o], dim3(grid), dim3(bs), 0, 0, out, 9u, cyc);
      (void)hipEventRecord(e1, 0);
      (void)hipDeviceSynchronize();
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      (void)hipMemcpy(h, cyc, nw * 16, hipMemcpyDeviceToHost);
      double s = 0, rt = 0;
      for (int i = 0; i < nw; ++i) s += (double)h[2 * i], rt += (double)h[2 * i + 1];
      const double ghz = s / (rt * 10.0);           // shader cycles per ns
      const double per_wave = s / nw / (8.0 * REP);  // shader cycles per instruction, one wave
      // chip-level: the whole kernel's cycles (events x clock) over the wave-instructions each SIMD issued
      const double simd = ms * 1e6 * ghz / (wps * 8.0 * REP);
      printf("%-14s %6.2f cyc/inst per wave | kernel %.3f ms at %.2f GHz: %5.2f cyc/inst per SIMD (%.0f waves/SIMD)\n",
             names[o], per_wave, ms, ghz, simd, wps);
    }
  }
  return hipGetLastError() != hipSuccess;
}
