// qba_exact.hip -- exact-order checks for bit-exact protocol parity, and the
// wire-compatible bit codec.
//
// The reference builds every party's tuple in its own set-iteration order
// (tfg.py:189, 291) and compares tuples position by position (tfg.py:97-98),
// so parity with it needs the host's index orders, not a canonical one.  The
// host keeps the Python sets; these kernels do the per-element work.
#include <string.h>

#include "qba_compact.h"

__global__ void __launch_bounds__(1024)
    qba_k_compact_scan(const int32_t *__restrict__ counts, int64_t ntiles,
                       int64_t *__restrict__ offsets, int64_t *__restrict__ total) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int64_t per = (ntiles + 1023) / 1024;
  const int64_t lo = t * per, hi = lo + per < ntiles ? lo + per : ntiles;
  int64_t s = 0;
  for (int64_t i = lo; i < hi; ++i) s += counts[i];
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
    const int64_t y = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += y;
    __syncthreads();
  }
  int64_t run = part[t] - s;
  for (int64_t i = lo; i < hi; ++i) {
    offsets[i] = run;
    run += counts[i];
  }
  if (t == 1023) *total = part[1023];
}

// Exclusive scan of a large tile-count array in three launches: per-block
// sums of QBA_SC_CH counts (each thread 8 consecutive counts, 16-B loads),
// the single-workgroup scan above over the block sums, then each block's
// scan with its offset added.  The single-workgroup scan alone walks its
// per-thread chunks serially: 8.4 M tile counts (a 35-qubit support) took
// ~15 ms that way.
__device__ __forceinline__ int64_t qba_block_exscan(int64_t v, int64_t *wtot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) wtot[w] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t run = 0;
    for (int k = 0; k < QBA_SC_T / 64; ++k) {
      const int64_t t = wtot[k];
      wtot[k] = run;
      run += t;
    }
    wtot[QBA_SC_T / 64] = run;
  }
  __syncthreads();
  return wtot[w] + incl - v;
}

__device__ __forceinline__ void qba_sc_load(const int32_t *__restrict__ counts, int64_t ntiles, int32_t (&c)[QBA_SC_PER]) {
  const int64_t i0 = (int64_t)blockIdx.x * QBA_SC_CH + (int64_t)threadIdx.x * QBA_SC_PER;
  if (i0 + QBA_SC_PER <= ntiles) {
    const int4 a = reinterpret_cast<const int4 *>(counts + i0)[0], b = reinterpret_cast<const int4 *>(counts + i0)[1];
    c[0] = a.x, c[1] = a.y, c[2] = a.z, c[3] = a.w, c[4] = b.x, c[5] = b.y, c[6] = b.z, c[7] = b.w;
  } else {
#pragma unroll
    for (int k = 0; k < QBA_SC_PER; ++k) c[k] = i0 + k < ntiles ? counts[i0 + k] : 0;
  }
}

__global__ void __launch_bounds__(QBA_SC_T)
    qba_k_scan_reduce(const int32_t *__restrict__ counts, int64_t ntiles, int32_t *__restrict__ bsum) {
  __shared__ int64_t wtot[QBA_SC_T / 64 + 1];
  int32_t c[QBA_SC_PER];
  qba_sc_load(counts, ntiles, c);
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < QBA_SC_PER; ++k) s += c[k];
  qba_block_exscan(s, wtot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = (int32_t)wtot[QBA_SC_T / 64];  // < 2^31: 8192 tiles x 4096 items
}

__global__ void __launch_bounds__(QBA_SC_T)
    qba_k_scan_apply(const int32_t *__restrict__ counts, int64_t ntiles, const int64_t *__restrict__ boff,
                     int64_t *__restrict__ offsets) {
  __shared__ int64_t wtot[QBA_SC_T / 64 + 1];
  int32_t c[QBA_SC_PER];
  qba_sc_load(counts, ntiles, c);
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < QBA_SC_PER; ++k) s += c[k];
  int64_t run = boff[blockIdx.x] + qba_block_exscan(s, wtot);
  const int64_t i0 = (int64_t)blockIdx.x * QBA_SC_CH + (int64_t)threadIdx.x * QBA_SC_PER;
#pragma unroll
  for (int k = 0; k < QBA_SC_PER; ++k) {
    if (i0 + k < ntiles) offsets[i0 + k] = run;
    run += c[k];
  }
}

// --- isQCorrList = {k : Li[k] != Lc[k]}  (tfg.py:327) -------------------------------
struct QbaIsqPred {
  const uint8_t *l0, *l1;
  int64_t *out;
  __device__ bool test(int64_t i) const { return l0[i] != l1[i]; }
  __device__ void emit(int64_t i, int64_t pos) const { out[pos] = i; }
};

extern "C" int qba_isq_indices(qba_ctx *ctx, const uint8_t *li, const uint8_t *lc, uint64_t count,
                               int64_t *idx, int64_t cap, int64_t *count_host, qba_stream stream) {
  if (!ctx || !count_host || (count && (!li || !lc)) || (cap > 0 && !idx) || cap < 0)
    return qba_fail(QBA_EINVAL, "qba_isq_indices: bad arguments");
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  return qba_compact(ctx, QbaIsqPred{li, lc, idx}, (int64_t)count, cap, count_host,
                     (hipStream_t)stream);
}

// --- P = {x in isQCorr : Lc[x] == v}, isQCorr's iteration order kept (tfg.py:182) ------
// An index outside [0, lc_len) is never dereferenced: it flags the call,
// which then fails with QBA_EINVAL (the order comes through the public ABI).
struct QbaSelPred {
  const int64_t *order;
  const uint8_t *lc;
  uint64_t lc_len;
  int64_t v;
  int64_t *out;
  int32_t *bad;
  __device__ bool test(int64_t i) const {
    const int64_t x = order[i];
    if ((uint64_t)x >= lc_len) {
      atomicOr(bad, 1);
      return false;
    }
    return (int64_t)lc[x] == v;
  }
  __device__ void emit(int64_t i, int64_t pos) const { out[pos] = order[i]; }
};

extern "C" int qba_select_eq(qba_ctx *ctx, const int64_t *order, int64_t m, const uint8_t *lc,
                             uint64_t lc_len, int64_t v, int64_t *out, int64_t *count_host,
                             qba_stream stream) {
  if (!ctx || !count_host || m < 0 || (m && (!order || !lc || !out)))
    return qba_fail(QBA_EINVAL, "qba_select_eq: bad arguments");
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  QBA_HIP(hipMemsetAsync(ctx->flag, 0, sizeof(int32_t), s));
  rc = qba_compact(ctx, QbaSelPred{order, lc, lc_len, v, out, ctx->flag}, m, m, count_host, s);
  if (rc) return rc;
  int32_t bad = 0;  // qba_compact has synchronised the stream
  QBA_HIP(hipMemcpy(&bad, ctx->flag, sizeof(int32_t), hipMemcpyDeviceToHost));
  if (bad) return qba_fail(QBA_EINVAL, "qba_select_eq: index outside Lc");
  return QBA_OK;
}

// --- host-pointer forms (the protocol host's calls): small inputs in ONE
// single-workgroup launch through the zero-copy staging, larger ones through
// the device compaction and one D2H ---------------------------------------------------
// the P filter over an order held in host memory: a bad index is a plain
// store of 1 (no atomics on host memory)
struct QbaSelPredZ {
  const int64_t *order;
  const uint8_t *lc;
  uint64_t lc_len;
  int64_t v;
  int64_t *out;
  int64_t *bad;
  __device__ bool test(int64_t i) const {
    const int64_t x = order[i];
    if ((uint64_t)x >= lc_len) {
      *bad = 1;
      return false;
    }
    return (int64_t)lc[x] == v;
  }
  __device__ void emit(int64_t i, int64_t pos) const { out[pos] = order[i]; }
};

extern "C" int qba_isq_indices_host(qba_ctx *ctx, const uint8_t *li, const uint8_t *lc, uint64_t count,
                                    int64_t *idx_host, int64_t cap, int64_t *count_host, qba_stream stream) {
  if (!ctx || !count_host || (count && (!li || !lc)) || (cap > 0 && !idx_host) || cap < 0)
    return qba_fail(QBA_EINVAL, "qba_isq_indices_host: bad arguments");
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const int64_t keep = std::min<int64_t>(cap, (int64_t)count);
  if (count <= QBA_CS_MAX) {
    if ((rc = qba_ensure_zc(ctx, 8 * (size_t)(keep + 1)))) return rc;
    int64_t *z = static_cast<int64_t *>(ctx->zc), *zd = static_cast<int64_t *>(ctx->zc_d);
    z[0] = 0;
    if (count) {
      hipLaunchKernelGGL(qba_k_compact_small<QbaIsqPred>, dim3(1), dim3(QBA_CS_THREADS), 0, s,
                         QbaIsqPred{li, lc, zd + 1}, (int64_t)count, keep, zd);
      QBA_HIP(hipGetLastError());
      QBA_HIP(hipStreamSynchronize(s));
    }
    *count_host = z[0];
    memcpy(idx_host, z + 1, 8 * (size_t)std::min<int64_t>(z[0], keep));
    return QBA_OK;
  }
  if ((rc = qba_ensure_staging(ctx, 8 * (size_t)keep, 8 * (size_t)keep))) return rc;
  int64_t *d = static_cast<int64_t *>(ctx->pin_d);
  if ((rc = qba_compact(ctx, QbaIsqPred{li, lc, d}, (int64_t)count, keep, count_host, s))) return rc;
  const size_t got = (size_t)std::min<int64_t>(*count_host, keep);
  QBA_HIP(hipMemcpyAsync(ctx->pin_h, d, 8 * got, hipMemcpyDeviceToHost, s));
  QBA_HIP(hipStreamSynchronize(s));
  memcpy(idx_host, ctx->pin_h, 8 * got);
  return QBA_OK;
}

extern "C" int qba_select_eq_host(qba_ctx *ctx, const int64_t *order_host, int64_t m, const uint8_t *lc,
                                  uint64_t lc_len, int64_t v, int64_t *out_host, int64_t *count_host,
                                  qba_stream stream) {
  if (!ctx || !count_host || m < 0 || (m && (!order_host || !lc || !out_host)))
    return qba_fail(QBA_EINVAL, "qba_select_eq_host: bad arguments");
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  if (m == 0) {
    *count_host = 0;
    return QBA_OK;
  }
  if (m <= QBA_CS_MAX) {
    // [total | bad | order (m) | out (m)]
    if ((rc = qba_ensure_zc(ctx, 8 * (size_t)(2 + 2 * m)))) return rc;
    int64_t *z = static_cast<int64_t *>(ctx->zc), *zd = static_cast<int64_t *>(ctx->zc_d);
    z[0] = z[1] = 0;
    memcpy(z + 2, order_host, 8 * (size_t)m);
    hipLaunchKernelGGL(qba_k_compact_small<QbaSelPredZ>, dim3(1), dim3(QBA_CS_THREADS), 0, s,
                       QbaSelPredZ{zd + 2, lc, lc_len, v, zd + 2 + m, zd + 1}, m, m, zd);
    QBA_HIP(hipGetLastError());
    QBA_HIP(hipStreamSynchronize(s));
    if (z[1]) return qba_fail(QBA_EINVAL, "qba_select_eq_host: index outside Lc");
    *count_host = z[0];
    memcpy(out_host, z + 2 + m, 8 * (size_t)z[0]);
    return QBA_OK;
  }
  if ((rc = qba_ensure_staging(ctx, 8 * (size_t)m, 16 * (size_t)m))) return rc;
  int64_t *d_order = static_cast<int64_t *>(ctx->pin_d), *d_out = d_order + m;
  memcpy(ctx->pin_h, order_host, 8 * (size_t)m);
  QBA_HIP(hipMemcpyAsync(d_order, ctx->pin_h, 8 * (size_t)m, hipMemcpyHostToDevice, s));
  if ((rc = qba_select_eq(ctx, d_order, m, lc, lc_len, v, d_out, count_host, stream))) return rc;
  QBA_HIP(hipMemcpyAsync(ctx->pin_h, d_out, 8 * (size_t)*count_host, hipMemcpyDeviceToHost, s));
  QBA_HIP(hipStreamSynchronize(s));
  memcpy(out_host, ctx->pin_h, 8 * (size_t)*count_host);
  return QBA_OK;
}

// --- tuple(Li[j] for j in P)  (tfg.py:189, 291) --------------------------------------
__global__ void qba_k_gather(const uint8_t *__restrict__ li, const int64_t *__restrict__ idx,
                             int64_t m, int64_t *__restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = li[idx[i]];
}

// Indices must lie in [0, list_len): verified on the device first so a bad
// packet cannot make the gather read out of bounds.
__global__ void qba_k_bounds(const int64_t *__restrict__ idx, int64_t m, int64_t len,
                             int32_t *__restrict__ bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x)
    if (idx[i] < 0 || idx[i] >= len) atomicOr(bad, 1);
}

extern "C" int qba_gather(qba_ctx *ctx, const uint8_t *li, uint64_t list_len, const int64_t *idx,
                          int64_t m, int64_t *out, qba_stream stream) {
  if (!ctx || m < 0 || (m && (!li || !idx || !out)))
    return qba_fail(QBA_EINVAL, "qba_gather: bad arguments");
  if (m == 0) return QBA_OK;
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const unsigned grid = (unsigned)std::min<int64_t>((m + 255) / 256, 4096);
  QBA_HIP(hipMemsetAsync(ctx->flag, 0, sizeof(int32_t), s));
  hipLaunchKernelGGL(qba_k_bounds, dim3(grid), dim3(256), 0, s, idx, m, (int64_t)list_len, ctx->flag);
  int32_t bad = 0;
  QBA_HIP(hipMemcpyAsync(&bad, ctx->flag, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  QBA_HIP(hipStreamSynchronize(s));
  if (bad) return qba_fail(QBA_EINVAL, "qba_gather: index outside the list");
  hipLaunchKernelGGL(qba_k_gather, dim3(grid), dim3(256), 0, s, li, idx, m, out);
  QBA_HIP(hipGetLastError());
  return QBA_OK;
}

// --- consistent(v, L, w): Cond2 and Cond3 (tfg.py:93-98) ---------------------------
// One thread per position k: every value must satisfy 0 <= x <= w and x != v
// (inclusive w, as the reference), and the m values at k must be pairwise
// distinct.  Any violation clears the flag.
__global__ void qba_k_consistent(const int64_t *__restrict__ t, int64_t m, int64_t len, int64_t v,
                                 int64_t w, int32_t *__restrict__ ok) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < len;
       k += (int64_t)gridDim.x * blockDim.x) {
    bool good = true;
    for (int64_t a = 0; a < m && good; ++a) {
      const int64_t x = t[a * len + k];
      if (x < 0 || x > w || x == v) good = false;
      for (int64_t b = a + 1; b < m && good; ++b)
        if (t[b * len + k] == x) good = false;
    }
    if (!good) atomicAnd(ok, 0);
  }
}

extern "C" int qba_consistent(qba_ctx *ctx, const int64_t *tuples, int64_t m, int64_t len,
                              int64_t v, int64_t w, int32_t *ok_host, qba_stream stream) {
  if (!ctx || !ok_host || m < 1 || len < 0 || (len && !tuples))
    return qba_fail(QBA_EINVAL, "qba_consistent: bad arguments (m >= 1 required)");
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const int32_t one = 1;
  QBA_HIP(hipMemcpyAsync(ctx->flag, &one, sizeof(int32_t), hipMemcpyHostToDevice, s));
  if (len > 0) {
    const unsigned grid = (unsigned)std::min<int64_t>((len + 255) / 256, 4096);
    hipLaunchKernelGGL(qba_k_consistent, dim3(grid), dim3(256), 0, s, tuples, m, len, v, w, ctx->flag);
    QBA_HIP(hipGetLastError());
  }
  QBA_HIP(hipMemcpyAsync(ok_host, ctx->flag, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  QBA_HIP(hipStreamSynchronize(s));
  return QBA_OK;
}

// --- one packet of the exact-order protocol in ONE launch (tfg.py:189-192, 291-294) ---
// The receiving lieutenant gathers its own tuple Li[P] in its set-iteration
// order and evaluates consistent(v, L | {own}) (tfg.py:87-98) over the packet's
// m received tuples.  Cond1 (equal lengths) is the host's; here all tuples
// have length len.  L is a set, so own is dropped from the pairwise test when
// it equals a received tuple: per received tuple a, eq[a] counts positions k
// with t_a[k] == own[k], and a pair (a, own) violates Cond3 iff
// 0 < eq[a] < len.  Output (device, int64): own[0..len), then
// [len] bad index, [len+1] Cond2/3 violation among the received tuples,
// [len+2] Cond2 violation of own, [len+3+a] eq[a].
__global__ void qba_k_check_packet(const uint8_t *__restrict__ li, uint64_t list_len,
                                   const int64_t *__restrict__ stage, int64_t m, int64_t len, int64_t v,
                                   int64_t w, int64_t *__restrict__ out) {
  const int64_t *order = stage, *t = stage + len;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < len;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = order[k];
    int64_t own = -1;
    if ((uint64_t)j >= list_len) {
      atomicOr(reinterpret_cast<unsigned long long *>(&out[len]), 1ull);
    } else {
      own = li[j];
    }
    out[k] = own;
    if (own < 0 || own > w || own == v) atomicOr(reinterpret_cast<unsigned long long *>(&out[len + 2]), 1ull);
    bool good = true;
    for (int64_t a = 0; a < m; ++a) {
      const int64_t x = t[a * len + k];
      if (x < 0 || x > w || x == v) good = false;
      for (int64_t b = a + 1; b < m && good; ++b)
        if (t[b * len + k] == x) good = false;
      if (x == own) atomicAdd(reinterpret_cast<unsigned long long *>(&out[len + 3 + a]), 1ull);
    }
    if (!good) atomicOr(reinterpret_cast<unsigned long long *>(&out[len + 1]), 1ull);
  }
}

extern "C" int qba_check_packet(qba_ctx *ctx, const uint8_t *li, uint64_t list_len, const int64_t *stage,
                                int64_t m, int64_t len, int64_t v, int64_t w, int64_t *out,
                                qba_stream stream) {
  if (!ctx || !out || m < 0 || len < 0 || (len && (!li || !stage)))
    return qba_fail(QBA_EINVAL, "qba_check_packet: bad arguments");
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  QBA_HIP(hipMemsetAsync(out + len, 0, (size_t)(3 + m) * sizeof(int64_t), s));
  if (len > 0) {
    const unsigned grid = (unsigned)std::min<int64_t>((len + 255) / 256, 1024);
    hipLaunchKernelGGL(qba_k_check_packet, dim3(grid), dim3(256), 0, s, li, list_len, stage, m, len, v, w, out);
    QBA_HIP(hipGetLastError());
  }
  return QBA_OK;
}

// --- consistent(v, L, w) over tuples gathered from the device lists (SURVEY.md
// §8(b) qba_check_gather) ---------------------------------------------------------
// T_a[k] = lists[party[a]][idx[a][k]] for m index orders of length len (each
// tuple in its own order, as each lieutenant ships its own set-iteration
// order, tfg.py:189, 291).  L is a set (tfg.py:209, 240, 260), so identical
// tuples collapse: the pair (a, b) violates Cond3 iff 0 < eq(a, b) < len,
// eq = the number of positions where T_a and T_b agree.  cnt (scratch):
// [0] bad index/party, [1] Cond2 violation, [2 + pair] eq per pair a < b,
// each workgroup adding its LDS partial once.
#define QBA_GATHER_MAXM 64
__global__ void __launch_bounds__(256)
    qba_k_check_gather(const uint8_t *__restrict__ lists, uint64_t ld, int rows, uint64_t list_len,
                       const int64_t *__restrict__ idx, const int32_t *__restrict__ party, int64_t m,
                       int64_t len, int64_t v, int64_t w, unsigned long long *__restrict__ cnt) {
  __shared__ unsigned int eq[QBA_GATHER_MAXM * (QBA_GATHER_MAXM - 1) / 2];
  __shared__ unsigned int flags[2];
  const int np = (int)(m * (m - 1) / 2);
  for (int i = threadIdx.x; i < np; i += blockDim.x) eq[i] = 0u;
  if (threadIdx.x < 2) flags[threadIdx.x] = 0u;
  __syncthreads();
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < len;
       k += (int64_t)gridDim.x * blockDim.x) {
    // values re-read per pair (m is small; a runtime-indexed private array
    // would live in scratch)
    auto val = [&](int64_t a) -> int64_t {
      const int64_t j = idx[a * len + k];
      const int32_t r = party[a];
      if (r < 0 || r >= rows || (uint64_t)j >= list_len) return -1;
      return lists[(uint64_t)r * ld + (uint64_t)j];
    };
    int p = 0;
    for (int64_t a = 0; a < m; ++a) {
      const int64_t xa = val(a);
      if (xa < 0) atomicOr(&flags[0], 1u);
      if (xa < 0 || xa > w || xa == v) atomicOr(&flags[1], 1u);
      for (int64_t b = a + 1; b < m; ++b, ++p)
        if (xa == val(b)) atomicAdd(&eq[p], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < np; i += blockDim.x)
    if (eq[i]) atomicAdd(&cnt[2 + i], (unsigned long long)eq[i]);
  if (threadIdx.x < 2 && flags[threadIdx.x]) atomicOr(&cnt[threadIdx.x], 1ull);
}

__global__ void qba_k_check_gather_fin(const unsigned long long *__restrict__ cnt, int64_t m, int64_t len,
                                       int32_t *__restrict__ ok) {
  if (threadIdx.x != 0) return;
  int32_t r = 1;
  if (cnt[0]) {
    r = -1;
  } else if (cnt[1]) {
    r = 0;
  } else {
    const int64_t np = m * (m - 1) / 2;
    for (int64_t p = 0; p < np; ++p)
      if (cnt[2 + p] != 0ull && cnt[2 + p] != (unsigned long long)len) r = 0;
  }
  *ok = r;
}

extern "C" int qba_check_gather(qba_ctx *ctx, const uint8_t *lists, uint64_t ld, int rows, uint64_t list_len,
                                const int64_t *idx, const int32_t *party, int64_t m, int64_t len, int64_t v,
                                int64_t w, int32_t *ok, qba_stream stream) {
  if (!ctx || !ok || m < 1 || m > QBA_GATHER_MAXM || len < 0 || rows < 1 || ld < list_len ||
      (len && (!lists || !idx || !party)))
    return qba_fail(QBA_EINVAL, "qba_check_gather: bad arguments (1 <= m <= 64 tuples required; "
                                "an empty L is the reference's StopIteration, tfg.py:90)");
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  const size_t ncnt = 2 + (size_t)(m * (m - 1) / 2);
  if ((rc = qba_ensure_scan(ctx, ncnt * sizeof(unsigned long long)))) return rc;
  hipStream_t s = (hipStream_t)stream;
  unsigned long long *cnt = static_cast<unsigned long long *>(ctx->scan);
  QBA_HIP(hipMemsetAsync(cnt, 0, ncnt * sizeof(unsigned long long), s));
  if (len > 0) {
    const unsigned grid = (unsigned)std::min<int64_t>((len + 255) / 256, 1024);
    hipLaunchKernelGGL(qba_k_check_gather, dim3(grid), dim3(256), 0, s, lists, ld, rows, list_len, idx, party, m,
                       len, v, w, cnt);
    QBA_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(qba_k_check_gather_fin, dim3(1), dim3(64), 0, s, cnt, m, len, ok);
  QBA_HIP(hipGetLastError());
  return QBA_OK;
}

// The same packet check as ONE workgroup whose stage and output live in the
// zero-copy staging (host memory): its counters are LDS atomics and the
// output is written with plain stores, so nothing but the launch and one sync
// stands between the host and the answer.  m <= QBA_GATHER_MAXM.
__global__ void __launch_bounds__(1024)
    qba_k_check_packet_zc(const uint8_t *__restrict__ li, uint64_t list_len, const int64_t *__restrict__ stage,
                          int64_t m, int64_t len, int64_t v, int64_t w, int64_t *__restrict__ out) {
  __shared__ unsigned int fl[3];
  __shared__ unsigned int eq[QBA_GATHER_MAXM];
  if (threadIdx.x < 3) fl[threadIdx.x] = 0u;
  if (threadIdx.x < QBA_GATHER_MAXM) eq[threadIdx.x] = 0u;
  __syncthreads();
  const int64_t *order = stage, *t = stage + len;
  for (int64_t k = threadIdx.x; k < len; k += blockDim.x) {
    const int64_t j = order[k];
    int64_t own = -1;
    if ((uint64_t)j >= list_len)
      atomicOr(&fl[0], 1u);
    else
      own = li[j];
    out[k] = own;
    if (own < 0 || own > w || own == v) atomicOr(&fl[2], 1u);
    bool good = true;
    for (int64_t a = 0; a < m; ++a) {
      const int64_t x = t[a * len + k];
      if (x < 0 || x > w || x == v) good = false;
      for (int64_t b = a + 1; b < m && good; ++b)
        if (t[b * len + k] == x) good = false;
      if (x == own) atomicAdd(&eq[a], 1u);
    }
    if (!good) atomicOr(&fl[1], 1u);
  }
  __syncthreads();
  if (threadIdx.x < 3) out[len + threadIdx.x] = fl[threadIdx.x];
  if (threadIdx.x < m) out[len + 3 + threadIdx.x] = eq[threadIdx.x];
}

// k packets [order | rows] concatenated in the zero-copy staging (stage_host
// copied in), outputs after them; one launch per packet, one sync.
static int check_packets_zc(qba_ctx *ctx, const uint8_t *li, uint64_t list_len, const int64_t *stage_host,
                            const int64_t *desc, int64_t k, int64_t w, size_t nin, size_t nout,
                            int64_t *out_host, hipStream_t s) {
  int rc = qba_ensure_zc(ctx, 8 * (nin + nout));
  if (rc) return rc;
  int64_t *z = static_cast<int64_t *>(ctx->zc), *zd = static_cast<int64_t *>(ctx->zc_d);
  if (nin) memcpy(z, stage_host, 8 * nin);
  size_t oi = 0, oo = nin;
  for (int64_t i = 0; i < k; ++i) {
    const int64_t m = desc[3 * i], len = desc[3 * i + 1], v = desc[3 * i + 2];
    if (len > 0) {
      hipLaunchKernelGGL(qba_k_check_packet_zc, dim3(1), dim3(1024), 0, s, li, list_len, zd + oi, m, len, v, w,
                         zd + oo);
      QBA_HIP(hipGetLastError());
    } else {
      for (int64_t q = 0; q < 3 + m; ++q) z[oo + q] = 0;
    }
    oi += (size_t)len * (size_t)(m + 1);
    oo += (size_t)(len + 3 + m);
  }
  QBA_HIP(hipStreamSynchronize(s));
  memcpy(out_host, z + nin, 8 * nout);
  return QBA_OK;
}

// Synchronous host-pointer form (the protocol host's per-packet call): a
// small packet (m <= 64 tuples, <= QBA_ZC_MAX bytes) is checked by one
// workgroup straight from and into the zero-copy staging; a larger one goes
// through the ctx's pinned staging: one H2D, one launch, one D2H, one sync.
extern "C" int qba_check_packet_host(qba_ctx *ctx, const uint8_t *li, uint64_t list_len,
                                     const int64_t *stage_host, int64_t m, int64_t len, int64_t v,
                                     int64_t w, int64_t *out_host, qba_stream stream) {
  if (!ctx || !out_host || m < 0 || len < 0 || (len && (!li || !stage_host)))
    return qba_fail(QBA_EINVAL, "qba_check_packet_host: bad arguments");
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  const size_t nin = (size_t)len * (size_t)(m + 1), nout = (size_t)(len + 3 + m);
  hipStream_t s = (hipStream_t)stream;
  if (m <= QBA_GATHER_MAXM && 8 * (nin + nout) <= QBA_ZC_MAX) {
    const int64_t desc[3] = {m, len, v};
    return check_packets_zc(ctx, li, list_len, stage_host, desc, 1, w, nin, nout, out_host, s);
  }
  if ((rc = qba_ensure_staging(ctx, 8 * (nin > nout ? nin : nout), 8 * (nin + nout)))) return rc;
  int64_t *pin = static_cast<int64_t *>(ctx->pin_h), *d_in = static_cast<int64_t *>(ctx->pin_d),
          *d_out = d_in + nin;
  if (nin) {
    memcpy(pin, stage_host, 8 * nin);
    QBA_HIP(hipMemcpyAsync(d_in, pin, 8 * nin, hipMemcpyHostToDevice, s));
  }
  if ((rc = qba_check_packet(ctx, li, list_len, d_in, m, len, v, w, d_out, stream))) return rc;
  QBA_HIP(hipMemcpyAsync(pin, d_out, 8 * nout, hipMemcpyDeviceToHost, s));
  QBA_HIP(hipStreamSynchronize(s));
  memcpy(out_host, pin, 8 * nout);
  return QBA_OK;
}

// A round's packets (tfg.py:337-348 -> 289-294) in one host round trip: the
// k stages concatenated (packet i: [order | rows] of len_i * (m_i + 1)
// int64, desc[i] = {m_i, len_i, v_i}), ONE H2D through the pinned staging, one
// qba_check_packet launch per packet, ONE D2H of the concatenated outputs
// (packet i: len_i + 3 + m_i int64, as qba_check_packet) and one sync.
extern "C" int qba_check_packets_host(qba_ctx *ctx, const uint8_t *li, uint64_t list_len,
                                      const int64_t *stage_host, const int64_t *desc, int64_t k, int64_t w,
                                      int64_t *out_host, qba_stream stream) {
  if (!ctx || !desc || !out_host || k < 1 || !stage_host)
    return qba_fail(QBA_EINVAL, "qba_check_packets_host: bad arguments");
  size_t nin = 0, nout = 0;
  bool small = true;
  for (int64_t i = 0; i < k; ++i) {
    const int64_t m = desc[3 * i], len = desc[3 * i + 1];
    if (m < 0 || len < 0 || (len && !li))
      return qba_fail(QBA_EINVAL, "qba_check_packets_host: bad packet descriptor");
    nin += (size_t)len * (size_t)(m + 1);
    nout += (size_t)(len + 3 + m);
    small = small && m <= QBA_GATHER_MAXM;
  }
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  if (small && 8 * (nin + nout) <= QBA_ZC_MAX)
    return check_packets_zc(ctx, li, list_len, stage_host, desc, k, w, nin, nout, out_host, s);
  if ((rc = qba_ensure_staging(ctx, 8 * (nin > nout ? nin : nout), 8 * (nin + nout)))) return rc;
  int64_t *pin = static_cast<int64_t *>(ctx->pin_h), *d_in = static_cast<int64_t *>(ctx->pin_d),
          *d_out = d_in + nin;
  if (nin) {
    memcpy(pin, stage_host, 8 * nin);
    QBA_HIP(hipMemcpyAsync(d_in, pin, 8 * nin, hipMemcpyHostToDevice, s));
  }
  size_t oi = 0, oo = 0;
  for (int64_t i = 0; i < k; ++i) {
    const int64_t m = desc[3 * i], len = desc[3 * i + 1], v = desc[3 * i + 2];
    if ((rc = qba_check_packet(ctx, li, list_len, d_in + oi, m, len, v, w, d_out + oo, stream))) return rc;
    oi += (size_t)len * (size_t)(m + 1);
    oo += (size_t)(len + 3 + m);
  }
  QBA_HIP(hipMemcpyAsync(pin, d_out, 8 * nout, hipMemcpyDeviceToHost, s));
  QBA_HIP(hipStreamSynchronize(s));
  memcpy(out_host, pin, 8 * nout);
  return QBA_OK;
}

// --- wire codec: rawS bits (one int64 per measured bit, MSB first) <-> values ---------
__global__ void qba_k_bits_to_values(const int64_t *__restrict__ raw, uint64_t count, int nq,
                                     uint8_t *__restrict__ vals) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < count;
       k += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t v = 0;
    for (int j = 0; j < nq; ++j) v = (v << 1) | (uint32_t)(raw[k * nq + j] & 1);
    vals[k] = (uint8_t)v;
  }
}

__global__ void qba_k_values_to_bits(const uint8_t *__restrict__ vals, uint64_t count, int nq,
                                     int64_t *__restrict__ raw) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count * nq;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = i / nq;
    const int j = (int)(i - k * nq);
    raw[i] = (vals[k] >> (nq - 1 - j)) & 1;
  }
}

extern "C" int qba_bits_to_values(qba_ctx *ctx, const int64_t *raw, uint64_t count, int nq,
                                  uint8_t *vals, qba_stream stream) {
  if (!ctx || nq < 1 || nq > 8 || (count && (!raw || !vals)))
    return qba_fail(QBA_EINVAL, "qba_bits_to_values: bad arguments (1 <= nq <= 8)");
  if (count == 0) return QBA_OK;
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  const unsigned grid = (unsigned)std::min<uint64_t>((count + 255) / 256, 8192);
  hipLaunchKernelGGL(qba_k_bits_to_values, dim3(grid), dim3(256), 0, (hipStream_t)stream, raw,
                     count, nq, vals);
  QBA_HIP(hipGetLastError());
  return QBA_OK;
}

// rawS of a whole run (tfg.py:81-84): rows [0, rows) of a lists matrix (row
// stride ld) encoded and copied to raw_host[rows][count * nq]; synchronous.
extern "C" int qba_lists_to_bits_host(qba_ctx *ctx, const uint8_t *lists, uint64_t ld, int rows,
                                      uint64_t count, int nq, int64_t *raw_host, qba_stream stream) {
  if (!ctx || rows < 0 || nq < 1 || nq > 8 || (rows && count && (!lists || !raw_host)))
    return qba_fail(QBA_EINVAL, "qba_lists_to_bits_host: bad arguments");
  const size_t n = (size_t)rows * count * nq;
  if (n == 0) return QBA_OK;
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const bool zc = 8 * n <= QBA_ZC_MAX;  // small: the kernels write the host staging directly
  if ((rc = zc ? qba_ensure_zc(ctx, 8 * n) : qba_ensure_staging(ctx, 8 * n, 8 * n))) return rc;
  int64_t *d = static_cast<int64_t *>(zc ? ctx->zc_d : ctx->pin_d);
  const unsigned grid = (unsigned)std::min<uint64_t>((count * nq + 255) / 256, 8192);
  for (int g = 0; g < rows; ++g)
    hipLaunchKernelGGL(qba_k_values_to_bits, dim3(grid), dim3(256), 0, s, lists + (uint64_t)g * ld, count, nq,
                       d + (size_t)g * count * nq);
  QBA_HIP(hipGetLastError());
  if (!zc) QBA_HIP(hipMemcpyAsync(ctx->pin_h, d, 8 * n, hipMemcpyDeviceToHost, s));
  QBA_HIP(hipStreamSynchronize(s));
  memcpy(raw_host, zc ? ctx->zc : ctx->pin_h, 8 * n);
  return QBA_OK;
}

// measure_to_ints of a received rawS row (tfg.py:158, 161) from host memory:
// one H2D through the pinned staging, the decode kernel; synchronous.
extern "C" int qba_bits_to_values_host(qba_ctx *ctx, const int64_t *raw_host, uint64_t count, int nq,
                                       uint8_t *vals, qba_stream stream) {
  if (!ctx || nq < 1 || nq > 8 || (count && (!raw_host || !vals)))
    return qba_fail(QBA_EINVAL, "qba_bits_to_values_host: bad arguments (1 <= nq <= 8)");
  if (count == 0) return QBA_OK;
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  const size_t n = count * (size_t)nq;
  hipStream_t s = (hipStream_t)stream;
  const bool zc = 8 * n <= QBA_ZC_MAX;  // small: the kernel reads the host staging directly
  const int64_t *src;
  if (zc) {
    if ((rc = qba_ensure_zc(ctx, 8 * n))) return rc;
    memcpy(ctx->zc, raw_host, 8 * n);
    src = static_cast<const int64_t *>(ctx->zc_d);
  } else {
    if ((rc = qba_ensure_staging(ctx, 8 * n, 8 * n))) return rc;
    memcpy(ctx->pin_h, raw_host, 8 * n);
    QBA_HIP(hipMemcpyAsync(ctx->pin_d, ctx->pin_h, 8 * n, hipMemcpyHostToDevice, s));
    src = static_cast<const int64_t *>(ctx->pin_d);
  }
  const unsigned grid = (unsigned)std::min<uint64_t>((count + 255) / 256, 8192);
  hipLaunchKernelGGL(qba_k_bits_to_values, dim3(grid), dim3(256), 0, s, src, count, nq, vals);
  if (zc) {  // no wait: the next user of the staging waits for this event instead
    QBA_HIP(hipGetLastError());
    if (!ctx->zc_ev) QBA_HIP(hipEventCreateWithFlags(&ctx->zc_ev, hipEventDisableTiming));
    QBA_HIP(hipEventRecord(ctx->zc_ev, s));
    ctx->zc_pending = true;
    return QBA_OK;
  }
  QBA_HIP(hipGetLastError());
  QBA_HIP(hipStreamSynchronize(s));
  return QBA_OK;
}

extern "C" int qba_values_to_bits(qba_ctx *ctx, const uint8_t *vals, uint64_t count, int nq,
                                  int64_t *raw, qba_stream stream) {
  if (!ctx || nq < 1 || nq > 8 || (count && (!raw || !vals)))
    return qba_fail(QBA_EINVAL, "qba_values_to_bits: bad arguments (1 <= nq <= 8)");
  if (count == 0) return QBA_OK;
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  const unsigned grid = (unsigned)std::min<uint64_t>((count * nq + 255) / 256, 8192);
  hipLaunchKernelGGL(qba_k_values_to_bits, dim3(grid), dim3(256), 0, (hipStream_t)stream, vals,
                     count, nq, raw);
  QBA_HIP(hipGetLastError());
  return QBA_OK;
}
