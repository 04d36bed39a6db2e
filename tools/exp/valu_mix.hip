// Issue cost of every VALU form the n = 11 list kernel's hot loop uses, on
// gfx950 at 8 waves per SIMD (4 x 512-thread workgroups per CU): cycles per
// wave64 instruction per SIMD for independent streams (8 chains per wave),
// whole-kernel time x the s_memtime clock.  Extends valu_rate.hip (which
// priced v_mad_u64_u32 / v_mul_* / v_perm / v_add / v_bitop3) to the SDWA,
// packed-16-bit, literal-operand, SGPR-writing and 3-input forms.
//   hipcc --offload-arch=gfx950 -O3 -o valu_mix tools/exp/valu_mix.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define REP 2048
#define N_OPS 20
template <int OP>
__global__ __launch_bounds__(512) void k(uint32_t *out, uint32_t seed, uint64_t *cyc) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u;
  uint32_t a4 = a0 + 11u, a5 = a0 + 13u, a6 = a0 + 17u, a7 = a0 + 19u;
  const uint32_t s = 0x3c3c3c3cu ^ seed;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int r = 0; r < REP; ++r) {
#define X8(M) M(a0, a4) M(a1, a5) M(a2, a6) M(a3, a7) M(a4, a0) M(a5, a1) M(a6, a2) M(a7, a3)
#define I2(op) asm volatile(op " %0, %0, %1" : "+v"(x) : "v"(y));
#define A(op) [&](uint32_t &x, uint32_t y) { op }
    if constexpr (OP == 0) {  // VOP2 with a 32-bit literal
#define M(x, y) asm volatile("v_and_b32 %0, 0x3c3c3c3c, %1" : "=v"(x) : "v"(y));
      X8(M)
#undef M
    } else if constexpr (OP == 1) {  // v_add_u32_sdwa, byte select
#define M(x, y) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(x) : "v"(y));
      X8(M)
#undef M
    } else if constexpr (OP == 2) {  // v_pk_lshlrev_b16
#define M(x, y) asm volatile("v_pk_lshlrev_b16 %0, %1, %0" : "+v"(x) : "v"(y));
      X8(M)
#undef M
    } else if constexpr (OP == 3) {  // v_and_or_b32 (VOP3, SGPR operand)
#define M(x, y) asm volatile("v_and_or_b32 %0, %0, %2, %1" : "+v"(x) : "v"(y), "s"(s));
      X8(M)
#undef M
    } else if constexpr (OP == 4) {  // v_lshl_or_b32
#define M(x, y) asm volatile("v_lshl_or_b32 %0, %0, 4, %1" : "+v"(x) : "v"(y));
      X8(M)
#undef M
    } else if constexpr (OP == 5) {  // v_bfe_u32
#define M(x, y) asm volatile("v_bfe_u32 %0, %1, 1, 4" : "=v"(x) : "v"(y));
      X8(M)
#undef M
    } else if constexpr (OP == 6) {  // v_bfe_i32
#define M(x, y) asm volatile("v_bfe_i32 %0, %1, 0, 1" : "=v"(x) : "v"(y));
      X8(M)
#undef M
    } else if constexpr (OP == 7) {  // v_or3_b32
#define M(x, y) asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(x) : "v"(y));
      X8(M)
#undef M
    } else if constexpr (OP == 8) {  // v_bcnt_u32_b32
#define M(x, y) asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(x) : "v"(y));
      X8(M)
#undef M
    } else if constexpr (OP == 9) {  // v_lshl_add_u32
#define M(x, y) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x) : "v"(y));
      X8(M)
#undef M
    } else if constexpr (OP == 10) {  // v_mbcnt_lo_u32_b32 (SGPR mask)
#define M(x, y) asm volatile("v_mbcnt_lo_u32_b32 %0, %2, %1" : "=v"(x) : "v"(y), "s"(s));
      X8(M)
#undef M
    } else if constexpr (OP == 11) {  // v_cmp_ne_u32_sdwa -> SGPR pair (VOPC, byte selects)
      uint64_t m;
#define M(x, y) asm volatile("v_cmp_ne_u32_sdwa %0, %1, %2 src0_sel:BYTE_0 src1_sel:BYTE_1" : "=s"(m) : "v"(x), "v"(y));
      X8(M)
#undef M
    } else if constexpr (OP == 12) {  // v_lshrrev_b32
#define M(x, y) asm volatile("v_lshrrev_b32 %0, 4, %1" : "=v"(x) : "v"(y));
      X8(M)
#undef M
    } else if constexpr (OP == 13) {  // v_or_b32_sdwa, word fold (the distinctness fold)
#define M(x, y) asm volatile("v_or_b32_sdwa %0, %1, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1" : "=v"(x) : "v"(y));
      X8(M)
#undef M
    } else if constexpr (OP == 14) {  // v_bitop3_b32 with an SGPR operand
#define M(x, y) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(y), "s"(s));
      X8(M)
#undef M
    } else if constexpr (OP == 15) {  // v_add_lshl_u32 with an SGPR operand
#define M(x, y) asm volatile("v_add_lshl_u32 %0, %1, %2, 3" : "=v"(x) : "v"(y), "s"(s));
      X8(M)
#undef M
    } else if constexpr (OP == 16) {  // v_perm_b32 with an SGPR selector
#define M(x, y) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(x) : "s"(s));
      X8(M)
#undef M
    } else if constexpr (OP == 17) {  // v_and_b32 VOP2 (register operands)
#define M(x, y) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(y));
      X8(M)
#undef M
    } else if constexpr (OP == 18) {  // v_mul_u32_u24
#define M(x, y) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(y));
      X8(M)
#undef M
    } else {  // v_mov_b32
#define M(x, y) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(y));
      X8(M)
#undef M
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if ((threadIdx.x & 63) == 0) {
    const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    cyc[2 * w] = t1 - t0;
    cyc[2 * w + 1] = r1 - r0;
  }
}

template <int O>
static void run_one(const char *name, uint32_t *out, uint64_t *cyc, uint64_t *h, hipEvent_t e0, hipEvent_t e1) {
  const int grid = 256 * 4, bs = 512, nw = grid * bs / 64;
  const double wps = nw / 1024.0;
  for (int it = 0; it < 2; ++it) hipLaunchKernelGGL(k<O>, dim3(grid), dim3(bs), 0, 0, out, 7u + it, cyc);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k<O>, dim3(grid), dim3(bs), 0, 0, out, 9u, cyc);
  (void)hipEventRecord(e1, 0);
  (void)hipDeviceSynchronize();
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipMemcpy(h, cyc, nw * 16, hipMemcpyDeviceToHost);
  double s = 0, rt = 0;
  for (int i = 0; i < nw; ++i) s += (double)h[2 * i], rt += (double)h[2 * i + 1];
  const double ghz = s / (rt * 10.0);
  const double simd = ms * 1e6 * ghz / (wps * 8.0 * REP);
  printf("%-34s kernel %.3f ms at %.2f GHz: %5.2f cyc/inst per SIMD (8 waves/SIMD)\n", name, ms, ghz, simd);
}

int main() {
  uint32_t *out;
  uint64_t *cyc;
  (void)hipMalloc(&out, (size_t)1024 * 512 * 4);
  (void)hipMalloc(&cyc, (size_t)1024 * 8 * 8 * 2);
  static uint64_t h[1024 * 8 * 2];
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  run_one<0>("v_and_b32 (32-bit literal)", out, cyc, h, e0, e1);
  run_one<1>("v_add_u32_sdwa (byte select)", out, cyc, h, e0, e1);
  run_one<2>("v_pk_lshlrev_b16", out, cyc, h, e0, e1);
  run_one<3>("v_and_or_b32 (SGPR)", out, cyc, h, e0, e1);
  run_one<4>("v_lshl_or_b32", out, cyc, h, e0, e1);
  run_one<5>("v_bfe_u32", out, cyc, h, e0, e1);
  run_one<6>("v_bfe_i32", out, cyc, h, e0, e1);
  run_one<7>("v_or3_b32", out, cyc, h, e0, e1);
  run_one<8>("v_bcnt_u32_b32", out, cyc, h, e0, e1);
  run_one<9>("v_lshl_add_u32", out, cyc, h, e0, e1);
  run_one<10>("v_mbcnt_lo_u32_b32", out, cyc, h, e0, e1);
  run_one<11>("v_cmp_ne_u32_sdwa -> SGPR", out, cyc, h, e0, e1);
  run_one<12>("v_lshrrev_b32", out, cyc, h, e0, e1);
  run_one<13>("v_or_b32_sdwa (word fold)", out, cyc, h, e0, e1);
  run_one<14>("v_bitop3_b32 (SGPR)", out, cyc, h, e0, e1);
  run_one<15>("v_add_lshl_u32 (SGPR)", out, cyc, h, e0, e1);
  run_one<16>("v_perm_b32 (SGPR selector)", out, cyc, h, e0, e1);
  run_one<17>("v_and_b32 (VGPRs)", out, cyc, h, e0, e1);
  run_one<18>("v_mul_u32_u24", out, cyc, h, e0, e1);
  run_one<19>("v_mov_b32", out, cyc, h, e0, e1);
  return hipGetLastError() != hipSuccess;
}
