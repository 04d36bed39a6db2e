// Instruction-rate microbenchmark v3 (gfx950): issue cost of one wave64 VALU
// instruction relative to v_add_u32, for the integer ops the list kernel is
// built from.  16 independent chains per lane (no dependency stalls), 8 waves
// per SIMD, every CU busy; each op's kernel is timed right after a v_add_u32
// kernel (same clock regime), min of 5 launches each.  Operand values stay
// random (an xor-shift feeds every chain) so that data-dependent power does
// not favour one op.  Prints cycles per wave-instruction per SIMD, scaled so
// that v_add_u32 = 2 (CDNA4: a wave64 VALU op issues over 2 cycles on a
// 32-wide SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITER 2048
#define C16(m) m(0) m(1) m(2) m(3) m(4) m(5) m(6) m(7) m(8) m(9) m(10) m(11) m(12) m(13) m(14) m(15)

// two-operand form: a_i = op(a_i, b)
#define K2(name, ins)                                                                   \
  __global__ void __launch_bounds__(256) k_##name(unsigned *out, unsigned seed) {       \
    unsigned a[16];                                                                     \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) a[i] = (threadIdx.x + 77 * i) * 2654435761u ^ seed; \
    unsigned b = seed * 2246822519u + threadIdx.x;                                      \
    for (int it = 0; it < ITER; ++it) {                                                 \
      _Pragma("unroll") for (int i = 0; i < 16; ++i) asm volatile(ins " %0, %0, %1" : "+v"(a[i]) : "v"(b) : "vcc"); \
      b ^= b << 13;                                                                     \
    }                                                                                   \
    unsigned r = 0;                                                                     \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) r ^= a[i];                           \
    out[blockIdx.x * 256 + threadIdx.x] = r;                                            \
  }
// three-operand form: a_i = op(a_i, b, c)
#define K3(name, ins)                                                                   \
  __global__ void __launch_bounds__(256) k_##name(unsigned *out, unsigned seed) {       \
    unsigned a[16];                                                                     \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) a[i] = (threadIdx.x + 77 * i) * 2654435761u ^ seed; \
    unsigned b = seed * 2246822519u + threadIdx.x, c = b * 3266489917u;                 \
    for (int it = 0; it < ITER; ++it) {                                                 \
      _Pragma("unroll") for (int i = 0; i < 16; ++i) asm volatile(ins : "+v"(a[i]) : "v"(b), "v"(c) : "vcc"); \
      b ^= b << 13;                                                                     \
    }                                                                                   \
    unsigned r = 0;                                                                     \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) r ^= a[i];                           \
    out[blockIdx.x * 256 + threadIdx.x] = r;                                            \
  }

K2(add, "v_add_u32")
K2(xor, "v_xor_b32")
K2(and, "v_and_b32")
K2(lshlrev, "v_lshlrev_b32")
K2(lshrrev, "v_lshrrev_b32")
K2(mullo, "v_mul_lo_u32")
K2(mulhi, "v_mul_hi_u32")
K2(mul24, "v_mul_u32_u24")
K2(bcnt, "v_bcnt_u32_b32")
K2(min, "v_min_u32")
K2(pklshl, "v_pk_lshlrev_b16")
K2(pkadd, "v_pk_add_u16")
K2(cndmask_vcc, "v_cndmask_b32")  // uses vcc as-is
K3(bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
K3(perm, "v_perm_b32 %0, %0, %1, %2")
K3(bfi, "v_bfi_b32 %0, %0, %1, %2")
K3(bfe, "v_bfe_u32 %0, %0, %1, 4")
K3(andor, "v_and_or_b32 %0, %0, %1, %2")
K3(lshladd, "v_lshl_add_u32 %0, %0, 4, %1")
K3(lshlor, "v_lshl_or_b32 %0, %0, 4, %1")
K3(addlshl, "v_add_lshl_u32 %0, %0, %1, 2")
K3(add3, "v_add3_u32 %0, %0, %1, %2")
K3(or3, "v_or3_b32 %0, %0, %1, %2")
K3(mad24, "v_mad_u32_u24 %0, %0, %1, %2")
K3(alignbit, "v_alignbit_b32 %0, %0, %1, 4")
K3(addsdwa, "v_add_u32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1")
K3(lshlsdwa, "v_lshlrev_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD")
K3(mbcnt, "v_mbcnt_lo_u32_b32 %0, %1, %0")
K3(cmpsdwa, "v_cmp_ne_u32_sdwa vcc, %0, %1 src0_sel:BYTE_1 src1_sel:DWORD\n v_cndmask_b32 %0, %0, %1, vcc")

__global__ void __launch_bounds__(256) k_mad64(unsigned *out, unsigned seed) {
  unsigned long long a[8];
  for (int j = 0; j < 8; ++j) a[j] = (threadIdx.x + j) * 0x9E3779B97F4A7C15ull ^ seed;
  unsigned x = seed * 2246822519u + threadIdx.x;
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, 0\nv_mad_u64_u32 %0, s[0:1], %1, %2, 0"
                   : "+v"(a[j]) : "v"((unsigned)a[j]), "v"(x) : "s0", "s1");
    x ^= x << 13;
  }
  unsigned r = 0;
  for (int j = 0; j < 8; ++j) r ^= (unsigned)(a[j] ^ (a[j] >> 32));
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

typedef void (*KF)(unsigned *, unsigned);
static float time_kern(KF k, unsigned *out) {
  const int blocks = 256 * 8;  // 8 blocks of 256 threads per CU = 8 waves per SIMD
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(a);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 7u + r);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  hipEventDestroy(a);
  hipEventDestroy(b);
  return best;
}

int main() {
  unsigned *out;
  hipMalloc(&out, 256 * 8 * 256 * 4);
  // warm the clock up with 200 ms of adds
  for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_add, dim3(2048), dim3(256), 0, 0, out, 1u);
  hipDeviceSynchronize();
  struct E { const char *n; KF k; int ops; } es[] = {
      {"xor", k_xor, 16},        {"and", k_and, 16},         {"lshlrev", k_lshlrev, 16}, {"lshrrev", k_lshrrev, 16},
      {"mul_lo", k_mullo, 16},   {"mul_hi", k_mulhi, 16},    {"mul_u24", k_mul24, 16},   {"bcnt", k_bcnt, 16},
      {"min", k_min, 16},        {"pk_lshlrev", k_pklshl, 16}, {"pk_add_u16", k_pkadd, 16}, {"cndmask", k_cndmask_vcc, 16},
      {"bitop3", k_bitop3, 16},  {"perm", k_perm, 16},       {"bfi", k_bfi, 16},         {"bfe", k_bfe, 16},
      {"and_or", k_andor, 16},   {"lshl_add", k_lshladd, 16}, {"lshl_or", k_lshlor, 16}, {"add_lshl", k_addlshl, 16},
      {"add3", k_add3, 16},      {"or3", k_or3, 16},         {"mad_u24", k_mad24, 16},   {"alignbit", k_alignbit, 16},
      {"add_sdwa", k_addsdwa, 16}, {"lshl_sdwa", k_lshlsdwa, 16}, {"mbcnt_lo", k_mbcnt, 16},
      {"cmp_sdwa+cnd", k_cmpsdwa, 32}, {"mad_u64", k_mad64, 16}};
  for (const E &e : es) {
    const float ta = time_kern(k_add, out);
    const float tx = time_kern(e.k, out);
    // per kernel: 2048 blocks * 4 waves * ITER * ops wave-instructions over 1024 SIMDs;
    // the add kernel has 16 ops + 1 xorshift (3 instr) per iteration -- same loop overhead
    printf("%-14s %7.3f ms  add %7.3f ms  cycles/wave-instr %5.2f\n", e.n, tx, ta,
           2.0 * tx / ta * 16.0 / e.ops);
  }
  return 0;
}
