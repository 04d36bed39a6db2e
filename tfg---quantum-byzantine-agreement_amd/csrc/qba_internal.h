// qba_internal.h -- shared definitions of libqba (host + gfx950 device code).
//
// Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11) is the counter-based
// generator; the counter is the GLOBAL list-entry index, so a shard computes
// exactly the entries it owns and lists are bit-identical at 1/2/4/8 GPUs.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/qba.h"

// ---------------------------------------------------------------------------
// Experiment builds (tools/exp/build.sh, optionally with the attribution
// probes of tools/exp/probes.patch) define QBA_EXPERIMENT_BUILD; several make
// the results wrong by design.  qba_build_flags() reports it (0 for a shipped
// build; tests/test_oracle_golden.py asserts it).
// ---------------------------------------------------------------------------
#ifdef QBA_EXPERIMENT_BUILD
#define QBA_BUILD_EXPERIMENT_FLAGS 1
#else
#define QBA_BUILD_EXPERIMENT_FLAGS 0
#endif

#define QBA_MAX_FACTORS 16
#define QBA_MAX_TABLE 4096   // uint64 table entries per kind (LDS budget)
#define QBA_BLOCK 256        // threads per workgroup (batched / helper kernels)
#define QBA_LBLOCK 1024      // threads per workgroup of the streaming list kernels (2 per CU at n = 11)
#define QBA_DBLOCK 768       // ... of the deferred-reduction list kernel (small launches)
#define QBA_CHUNK (1ull << 31)  // entries per list-kernel launch (32-bit offsets, u32 bins)
#define QBA_PB_MIN_DEFAULT (1ull << 24)  // entries from which the fused n = 11 kernel counts in pair bins
#define QBA_EPT 4            // entries per thread per step: one dword per list row

// ---------------------------------------------------------------------------
// Philox4x32-10
// ---------------------------------------------------------------------------
struct QbaU4 {
  uint32_t x, y, z, w;
};

// a ^ b ^ k in one VALU op (v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t qba_xor3(uint32_t a, uint32_t b, uint32_t k) {
  return __builtin_amdgcn_bitop3_b32(a, b, k, 0x96);
}

// Keys are wave-uniform (kernel arguments or block-uniform): they stay in SGPRs.
// SK (list-kernel callers with wave-uniform keys): round keys re-derived per
// block on the scalar unit.
template <bool SK = false>
__device__ __forceinline__ QbaU4 qba_philox_k(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = qba_xor3((uint32_t)(p1 >> 32), c1, k0);
    const uint32_t n2 = qba_xor3((uint32_t)(p0 >> 32), c3, k1);
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
    // the round keys re-derived per block on the scalar unit (two s_add per
    // round) instead of 20 loop-invariant SGPRs (register budget of 8 waves)
    if constexpr (SK) asm volatile("" : "+s"(k0), "+s"(k1));
  }
  return QbaU4{c0, c1, c2, c3};
}
__device__ __forceinline__ QbaU4 qba_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                            uint32_t k0, uint32_t k1) {
  return qba_philox_k<false>(c0, c1, c2, c3, k0, k1);
}

// ---------------------------------------------------------------------------
// Compiled resource program (one per circuit kind), see qba_resource.cpp.
//
// Random-bit schedule of one entry e (identical in the CPU twin,
// oracle/sampler_ref.c):
//   block b = philox(ctr = {e_lo, e_hi, b, 0}, key = {seed_lo, seed_hi})
//   block 0 = {x0, x1, x2, x3};  isQ = x0 & 1
//   Q:    F = x2 | x3 << 32 drives the permutation; table words are
//         x1, then block 1 words 0..3, block 2, ...
//   notQ: table words are x1, x2, x3, then block 1 words 0..3, ...
//   Permutation retry a = 1, 2, ...: F = y0 | y1 << 32 of block 0x80000000 + a.
// Each factor takes `bits` column bits at (col_word, col_shift), and when it
// is not uniform a 32-bit u from its own word u_word: outcome pattern
// = (u < thr[col]) ? pat[col] : apat[col].
// ---------------------------------------------------------------------------
struct QbaFactor {
  int32_t bits;
  int32_t uniform;
  int32_t offset;     // into the concatenated table of this program
  int32_t col_word;
  int32_t col_shift;
  int32_t u_word;     // -1 when uniform
};

struct QbaProgram {
  int32_t nfac;
  int32_t table_len;
  int32_t any_nonuniform;
  int32_t valid;
  uint64_t perm_t;  // 2^64 mod n!  (Lemire rejection threshold), Q program only
  QbaFactor fac[QBA_MAX_FACTORS];
};

// Device image of the compiled programs for one n: [prog notq][prog q], the
// closed-form stage tables (16-B words, at QBA_PERM_OFF), then pat[T],
// apat[T], thr[T] (uint64, at tab_off) where T = total table entries (notq
// tables first).
struct QbaProgramSet {
  QbaProgram prog[2];
  int32_t table_total;
  int32_t any_nonuniform;
  int32_t n;
  int32_t canonical;  // both programs have the standard layout of tfg.py's circuits:
                      // not-Q = ceil(n*nQ/8) uniform byte factors over words x1.., tables
                      // of 256 at f*256; Q = one uniform nQ-bit factor on x1.  The
                      // sampler then takes its specialised path (qba_sample_entry_fast).
  // Closed-form sampler (n <= 11 and the programs proven to be exactly the
  // distributions of tfg.py's two circuits, see qba_resource.hip):
  //   not-Q: L0 = L1, L1..Ln independent uniform;  Q: L_g = r ^ pi(g).
  // pi is drawn by forward Fisher-Yates over positions 1..n whose mixed-radix
  // digit string is split into three table indices (stage A: positions 1..3
  // when n >= 8; stages B, C: the 8-byte window that holds the rest) and
  // composed with v_perm_b32.  Random-bit schedule in qba_lists.hip.
  int32_t closed;
  uint32_t t32;             // 2^32 mod n!  (Lemire rejection threshold, 32-bit)
  uint32_t nfact;           // n!
  uint32_t ra, rb, rc;      // stage sizes, ra * rb * rc = n!
  int32_t perm_off;         // byte offset of the stage tables from the image start (QBA_PERM_OFF)
  int32_t perm_words;       // u32 words of stage tables: A [ra][4], B [rb][2], C [rc] (hi only)
  int32_t tab_off;          // byte offset of pat / apat / thr (after the stage tables)
};
// The stage tables sit right after the header, at an offset the list kernels
// know at compile time: their first table loads need no scalar load of the
// header first (one memory round trip less at each workgroup's start).
#define QBA_PERM_OFF ((sizeof(QbaProgramSet) + 15) & ~(size_t)15)

// Closed-form stage tables (host-built, staged to LDS): 4 + 2 + 1 words per
// entry of A, B, C.  Largest: n = 11 -> 990*4 + 1680*2 + 24 = 7344 words.
#define QBA_PERM_MAX_WORDS 7400
#define QBA_CLOSED_MAX_N 11

// ---------------------------------------------------------------------------
// error reporting / context
// ---------------------------------------------------------------------------
int qba_fail(int code, const std::string &msg);
#define QBA_HIP(call)                                                                     \
  do {                                                                                    \
    hipError_t _e = (call);                                                               \
    if (_e != hipSuccess)                                                                 \
      return qba_fail(QBA_EHIP, std::string(#call) + ": " + hipGetErrorString(_e));       \
  } while (0)

// host copy of one compiled program (tables before concatenation)
struct QbaHostProgram {
  QbaProgram p{};
  std::vector<uint64_t> pat, apat, thr;
};

struct qba_ctx {
  int device = 0;
  int num_cus = 256;
  // per-n compiled programs (device image + host copy)
  void *prog_dev[QBA_MAX_PARTIES + 1] = {};
  size_t prog_bytes[QBA_MAX_PARTIES + 1] = {};
  void *prog_host[QBA_MAX_PARTIES + 1] = {};  // QbaProgramSet + tables, host copy
  bool compiled[QBA_MAX_PARTIES + 1][2] = {};
  QbaHostProgram hprog[QBA_MAX_PARTIES + 1][2];
  // scratch
  void *slab = nullptr;
  size_t slab_bytes = 0;
  void *scan = nullptr;  // compaction scratch
  size_t scan_bytes = 0;
  int32_t *flag = nullptr;  // 1-word device flag
  int64_t *count1 = nullptr; // 1-word device counter
  int64_t *stats = nullptr;  // [2]: last counts launch: Q entries with a value >= w, spare
  uint64_t chunk = QBA_CHUNK;  // entries per list-kernel launch (qba_test_set_knobs may lower it)
  // pinned host + device staging of the synchronous *_host entry points
  void *zc = nullptr;     // zero-copy staging: coherent pinned host memory the kernels read / write
  void *zc_d = nullptr;   // its device address
  size_t zc_bytes = 0;
  hipEvent_t zc_ev = nullptr;  // recorded after an asynchronous reader of zc (bits_to_values_host)
  bool zc_pending = false;     // qba_ensure_zc waits for it before zc is rewritten
  void *pin_h = nullptr;
  size_t pin_h_bytes = 0;
  void *pin_d = nullptr;
  size_t pin_d_bytes = 0;
  // the pending deferred reduction (qba_sample_check*_deferred): the slab rows
  // of the last deferred call, reduced by the next one or qba_flush_deferred
  struct {
    int (*flush)(qba_ctx *ctx);  // per-n launcher of its reduction; null: none pending
    const uint32_t *slab;
    int rows, acc, sacc, buf;
    int64_t *H, *C, *P, *stats;
    hipStream_t stream;
  } pend = {};
  hipEvent_t def_ev = nullptr;  // orders a flush on one stream before slab reuse on another
  // RCCL communicator of the GPU-owner ranks (qba_rccl_init), or null
  void *rccl_comm = nullptr;
  int rccl_ranks = 0;
  // test seam (qba_test_set_knobs); the shipped selection otherwise:
  int list_grid = 0;  // > 0: cap on the list kernels' workgroups, pair bins at any size, <= 2^23 entries each
  uint64_t pb_min = QBA_PB_MIN_DEFAULT;  // entries from which the fused n = 11 kernel counts in pair bins
  // graph capture of the pending deferred reduction (pend): 1 when it was
  // recorded inside a capture, with that capture's id
  int pend_captured = 0;
  unsigned long long pend_capture_id = 0;
  // the slab's last user (qba_slab_order / qba_slab_done): its stream's
  // handle as a VALUE only (compared, never passed to HIP: the stream may be
  // destroyed since); a counting launch on another stream synchronises the
  // device first
  unsigned long long slab_last = 0;
  bool slab_set = false;
};
// Capture state of a stream: 1 capturing (its capture id in *id), 0 not.
int qba_capture_of(hipStream_t s, unsigned long long *id);
// Order a counting launch on `stream` after the slab's previous user on
// another stream (waits for the event qba_slab_done recorded), and record
// the event after the launches of a call that used the slab.
int qba_slab_order(qba_ctx *ctx, hipStream_t stream);
int qba_slab_done(qba_ctx *ctx, hipStream_t stream);
void qba_rccl_release(qba_ctx *ctx);

int qba_ensure_slab(qba_ctx *ctx, size_t bytes);
int qba_ensure_scan(qba_ctx *ctx, size_t bytes);
int qba_ensure_staging(qba_ctx *ctx, size_t host_bytes, size_t dev_bytes);
// Small synchronous host-pointer calls (<= QBA_ZC_MAX bytes staged) skip the
// H2D / D2H copies: their kernels read the input from and write the result to
// ctx->zc (through ctx->zc_d) with plain loads and stores -- no atomics on
// host memory.
#define QBA_ZC_MAX (1u << 20)
int qba_ensure_zc(qba_ctx *ctx, size_t bytes);
int qba_set_device(qba_ctx *ctx);

static inline int qba_nq(int n) {  // ceil(log2(n+1)), tfg.py:317
  int q = 0;
  while ((1 << q) < n + 1) ++q;
  return q;
}

static inline int64_t qba_ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
