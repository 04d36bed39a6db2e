// Instruction-rate microbenchmark (gfx950): cycles per wave64 instruction for
// the integer ops the sampler is built from.  8 independent chains per lane,
// 8 waves per SIMD, every CU busy.  Prints ns per instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITER 4096
#define OPS(name, asmstr)                                                           \
  __global__ void __launch_bounds__(256) k_##name(unsigned *out, unsigned seed) {   \
    unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3,         \
             a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed | 1;       \
    for (int i = 0; i < ITER; ++i) {                                                \
      asm volatile(asmstr : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4),       \
                   "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));                          \
    }                                                                               \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;      \
  }
#define X8(ins) ins " %0, %0, %8\n" ins " %1, %1, %8\n" ins " %2, %2, %8\n" ins " %3, %3, %8\n" \
                ins " %4, %4, %8\n" ins " %5, %5, %8\n" ins " %6, %6, %8\n" ins " %7, %7, %8\n"
OPS(add, X8("v_add_u32"))
OPS(xor, X8("v_xor_b32"))
OPS(mullo, X8("v_mul_lo_u32"))
OPS(mulhi, X8("v_mul_hi_u32"))
OPS(mul24, X8("v_mul_u32_u24"))
OPS(lshl, X8("v_lshlrev_b32"))
#define X8_3(ins) ins " %0, %0, %8, %1\n" ins " %1, %1, %8, %2\n" ins " %2, %2, %8, %3\n" ins " %3, %3, %8, %4\n" \
                  ins " %4, %4, %8, %5\n" ins " %5, %5, %8, %6\n" ins " %6, %6, %8, %7\n" ins " %7, %7, %8, %0\n"
#define X8_3B(ins) ins " %0, %0, %8, %1 bitop3:0x96\n" ins " %1, %1, %8, %2 bitop3:0x96\n" ins " %2, %2, %8, %3 bitop3:0x96\n" ins " %3, %3, %8, %4 bitop3:0x96\n" \
                  ins " %4, %4, %8, %5 bitop3:0x96\n" ins " %5, %5, %8, %6 bitop3:0x96\n" ins " %6, %6, %8, %7 bitop3:0x96\n" ins " %7, %7, %8, %0 bitop3:0x96\n"
OPS(bfe, X8_3("v_bfe_u32"))
OPS(lshlor, X8_3("v_lshl_or_b32"))
OPS(lshladd, X8_3("v_lshl_add_u32"))
OPS(alignbit, X8_3("v_alignbit_b32"))
OPS(perm, X8_3("v_perm_b32"))
OPS(xor3, X8_3B("v_bitop3_b32"))
OPS(mad24, X8_3("v_mad_u32_u24"))
OPS(andor, X8_3("v_and_or_b32"))
OPS(add3, X8_3("v_add3_u32"))
OPS(bcnt, X8("v_bcnt_u32_b32"))
OPS(lshr, X8("v_lshrrev_b32"))
OPS(sub, X8("v_sub_u32"))
OPS(min, X8("v_min_u32"))


// 64-bit ops need register pairs: use separate kernels
__global__ void __launch_bounds__(256) k_mad64(unsigned *out, unsigned seed) {
  unsigned long long a[4];
  unsigned x[4];
  for (int j = 0; j < 4; ++j) { a[j] = threadIdx.x + j + seed; x[j] = seed * (j + 3); }
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0\nv_mad_u64_u32 %0, s[0:1], %1, %2, %0"
                   : "+v"(a[j]) : "v"(x[j]), "v"(seed) : "s0", "s1");
  }
  out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a[0] ^ a[1] ^ a[2] ^ a[3]);
}
__global__ void __launch_bounds__(256) k_shr64(unsigned *out, unsigned seed) {
  unsigned long long a[4];
  unsigned s = seed & 31;
  for (int j = 0; j < 4; ++j) a[j] = ((unsigned long long)threadIdx.x << 32) + j + seed;
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      asm volatile("v_lshrrev_b64 %0, %1, %0\nv_lshrrev_b64 %0, %1, %0" : "+v"(a[j]) : "v"(s));
  }
  out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a[0] ^ a[1] ^ a[2] ^ a[3]);
}
__global__ void __launch_bounds__(256) k_dsadd(unsigned *out, unsigned seed) {
  __shared__ unsigned h[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) h[i] = 0;
  __syncthreads();
  unsigned x = threadIdx.x * 2654435761u + seed;
  for (int i = 0; i < ITER / 8; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x = x * 1664525u + 1013904223u;
      atomicAdd(&h[(x >> 20) & 4095], 1u);
    }
  }
  __syncthreads();
  out[blockIdx.x * 256 + threadIdx.x] = h[threadIdx.x];
}

template <typename K>
static void run(const char *name, K kern, int ops_per_iter, unsigned *out) {
  const int blocks = 256 * 8;  // 8 blocks of 256 threads per CU = 8 waves/SIMD
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 7u);
  hipEventRecord(a);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 7u);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  // wave-instructions per SIMD = blocks*4 waves * ITER * ops / (256 CU * 4 SIMD)
  double wi = (double)blocks * 4 * ITER * ops_per_iter / 1024.0;
  printf("%-8s %8.3f ms  %6.3f ns/wave-instr/SIMD  (= %.2f cycles at 2.4 GHz)\n", name, ms,
         ms * 1e6 / wi, ms * 1e6 / wi * 2.4);
}

int main() {
  unsigned *out;
  hipMalloc(&out, 256 * 8 * 256 * 4);
  run("add", k_add, 8, out);
  run("xor", k_xor, 8, out);
  run("lshl", k_lshl, 8, out);
  run("mul24", k_mul24, 8, out);
  run("mullo", k_mullo, 8, out);
  run("mulhi", k_mulhi, 8, out);
  run("mad64", k_mad64, 8, out);
  run("shr64", k_shr64, 8, out);
  run("dsadd", k_dsadd, 8, out);
  run("bfe", k_bfe, 8, out);
  run("lshlor", k_lshlor, 8, out);
  run("lshladd", k_lshladd, 8, out);
  run("alignbit", k_alignbit, 8, out);
  run("perm", k_perm, 8, out);
  run("xor3", k_xor3, 8, out);
  run("mad24", k_mad24, 8, out);
  run("andor", k_andor, 8, out);
  run("add3", k_add3, 8, out);
  run("bcnt", k_bcnt, 8, out);
  run("lshr", k_lshr, 8, out);
  run("sub", k_sub, 8, out);
  run("min", k_min, 8, out);
  // includes 1 LCG mad per atomic
  return 0;
}
