// qba_compact.h -- order-preserving stream compaction (count / scan / emit).
//
// Used where the reference builds an ordered selection: the ascending
// isQCorrList (tfg.py:327), the P filter that keeps isQCorr's iteration order
// (tfg.py:182) and the support of a statevector (resource compilation).
// Three launches: per-tile counts, a single-workgroup exclusive scan of the
// tile counts, and an emit pass that re-evaluates the predicate and writes
// each selected item at its global rank.  A tile is 256 threads x 16 items.
// The predicate is evaluated coalesced (round r: thread t tests item
// r * 256 + t of the tile, so a wave reads 64 consecutive items); the emit
// pass stages the flags in LDS and ranks them with each thread owning 16
// consecutive items.
#pragma once

#include "qba_internal.h"

#define QBA_CT_THREADS 256
#define QBA_CT_ITEMS 16
#define QBA_CT_TILE (QBA_CT_THREADS * QBA_CT_ITEMS)

template <class Pred>
__global__ void __launch_bounds__(QBA_CT_THREADS)
    qba_k_compact_count(Pred p, int64_t n, int32_t *__restrict__ tile_counts) {
  __shared__ int32_t wsum[QBA_CT_THREADS / 64];
  const int64_t tbase = (int64_t)blockIdx.x * QBA_CT_TILE;
  int32_t c = 0;
#pragma unroll
  for (int r = 0; r < QBA_CT_ITEMS; ++r) {
    const int64_t i = tbase + r * QBA_CT_THREADS + threadIdx.x;
    if (i < n && p.test(i)) ++c;
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t s = 0;
    for (int w = 0; w < QBA_CT_THREADS / 64; ++w) s += wsum[w];
    tile_counts[blockIdx.x] = s;
  }
}

// exclusive scan of ntiles int32 counts -> int64 offsets, total in *total
__global__ void __launch_bounds__(1024)
    qba_k_compact_scan(const int32_t *__restrict__ counts, int64_t ntiles,
                       int64_t *__restrict__ offsets, int64_t *__restrict__ total);

// multi-block scan of large tile-count arrays (qba_exact.hip)
#define QBA_SC_T 1024
#define QBA_SC_PER 8
#define QBA_SC_CH (QBA_SC_T * QBA_SC_PER)
__global__ void __launch_bounds__(QBA_SC_T)
    qba_k_scan_reduce(const int32_t *__restrict__ counts, int64_t ntiles, int32_t *__restrict__ bsum);
__global__ void __launch_bounds__(QBA_SC_T)
    qba_k_scan_apply(const int32_t *__restrict__ counts, int64_t ntiles, const int64_t *__restrict__ boff,
                     int64_t *__restrict__ offsets);

template <class Pred>
__global__ void __launch_bounds__(QBA_CT_THREADS)
    qba_k_compact_emit(Pred p, int64_t n, const int64_t *__restrict__ offsets, int64_t cap) {
  __shared__ int32_t wsum[QBA_CT_THREADS / 64];
  __shared__ uint32_t flags[QBA_CT_TILE / 4];  // one byte per item of the tile
  const int64_t tile = blockIdx.x;
  const int64_t tbase = tile * QBA_CT_TILE;
  uint8_t *f8 = reinterpret_cast<uint8_t *>(flags);
#pragma unroll
  for (int r = 0; r < QBA_CT_ITEMS; ++r) {
    const int64_t i = tbase + r * QBA_CT_THREADS + threadIdx.x;
    f8[r * QBA_CT_THREADS + threadIdx.x] = (i < n && p.test(i)) ? 1 : 0;
  }
  __syncthreads();
  // this thread's 16 consecutive items: 4 flag words, 0/1 bytes -> 4 bits each
  const int64_t base = tbase + (int64_t)threadIdx.x * QBA_CT_ITEMS;
  uint32_t bits = 0;
#pragma unroll
  for (int q = 0; q < QBA_CT_ITEMS / 4; ++q)
    bits |= ((flags[threadIdx.x * (QBA_CT_ITEMS / 4) + q] * 0x01020408u) >> 24) << (4 * q);
  const int32_t c = __popc(bits);
  // inclusive scan over the wave
  int32_t incl = c;
  const int lane = threadIdx.x & 63;
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) wsum[threadIdx.x >> 6] = incl;
  __syncthreads();
  int32_t wbase = 0;
  for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) wbase += wsum[w];
  int64_t pos = offsets[tile] + wbase + incl - c;
  while (bits) {
    const int k = __ffs(bits) - 1;
    bits &= bits - 1;
    if (pos < cap) p.emit(base + k, pos);
    ++pos;
  }
}

// Inputs of at most QBA_CS_MAX items in ONE launch of one workgroup (the
// exact-order protocol's small calls, e.g. configs[0]'s sizeL = 1000): the
// predicate evaluated coalesced into LDS flags, 16 consecutive items ranked
// per thread, the total written to *total by the last thread.  total and
// whatever emit writes may be host memory (the zero-copy staging).
#define QBA_CS_THREADS 1024
#define QBA_CS_MAX (QBA_CS_THREADS * QBA_CT_ITEMS)
template <class Pred>
__global__ void __launch_bounds__(QBA_CS_THREADS)
    qba_k_compact_small(Pred p, int64_t n, int64_t cap, int64_t *__restrict__ total) {
  __shared__ int32_t wsum[QBA_CS_THREADS / 64];
  __shared__ uint32_t flags[QBA_CS_MAX / 4];
  uint8_t *f8 = reinterpret_cast<uint8_t *>(flags);
  for (int r = 0; r < QBA_CT_ITEMS; ++r) {
    const int64_t i = (int64_t)r * QBA_CS_THREADS + threadIdx.x;
    f8[i] = (i < n && p.test(i)) ? 1 : 0;
  }
  __syncthreads();
  const int64_t base = (int64_t)threadIdx.x * QBA_CT_ITEMS;
  uint32_t bits = 0;
#pragma unroll
  for (int q = 0; q < QBA_CT_ITEMS / 4; ++q)
    bits |= ((flags[threadIdx.x * (QBA_CT_ITEMS / 4) + q] * 0x01020408u) >> 24) << (4 * q);
  const int32_t c = __popc(bits);
  int32_t incl = c;
  const int lane = threadIdx.x & 63;
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) wsum[threadIdx.x >> 6] = incl;
  __syncthreads();
  int32_t wbase = 0;
  for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) wbase += wsum[w];
  int64_t pos = wbase + incl - c;
  if (threadIdx.x == QBA_CS_THREADS - 1) *total = pos + c;
  while (bits) {
    const int k = __ffs(bits) - 1;
    bits &= bits - 1;
    if (pos < cap) p.emit(base + k, pos);
    ++pos;
  }
}

// Runs the three passes on `stream`, then waits and returns the total in *count_host.
template <class Pred>
static int qba_compact(qba_ctx *ctx, Pred p, int64_t n, int64_t cap, int64_t *count_host,
                       hipStream_t stream) {
  if (n <= 0) {
    *count_host = 0;
    return QBA_OK;
  }
  const int64_t ntiles = (n + QBA_CT_TILE - 1) / QBA_CT_TILE;
  const int64_t nb = (ntiles + QBA_SC_CH - 1) / QBA_SC_CH;  // scan blocks (large inputs)
  // [offsets int64 ntiles | block offsets int64 nb | counts int32 ntiles (16-B aligned) | block sums int32 nb]
  const int64_t n64 = (ntiles + nb + 1) & ~(int64_t)1;  // counts start 16-B aligned (int4 loads)
  const size_t need = n64 * sizeof(int64_t) + ((ntiles + 3) & ~3) * sizeof(int32_t) + nb * sizeof(int32_t) + 64;
  int rc = qba_ensure_scan(ctx, need);
  if (rc) return rc;
  int64_t *offsets = reinterpret_cast<int64_t *>(ctx->scan);
  int64_t *boff = offsets + ntiles;
  int32_t *counts = reinterpret_cast<int32_t *>(offsets + n64);
  int32_t *bsum = counts + ((ntiles + 3) & ~3);
  if (ntiles > 0x7fffffffLL) return qba_fail(QBA_EUNSUPPORTED, "compaction: input too large");
  hipLaunchKernelGGL(qba_k_compact_count<Pred>, dim3((unsigned)ntiles), dim3(QBA_CT_THREADS), 0,
                     stream, p, n, counts);
  QBA_HIP(hipGetLastError());
  if (nb <= 1) {
    hipLaunchKernelGGL(qba_k_compact_scan, dim3(1), dim3(1024), 0, stream, counts, ntiles, offsets,
                       ctx->count1);
  } else {
    hipLaunchKernelGGL(qba_k_scan_reduce, dim3((unsigned)nb), dim3(QBA_SC_T), 0, stream, counts, ntiles, bsum);
    hipLaunchKernelGGL(qba_k_compact_scan, dim3(1), dim3(1024), 0, stream, bsum, nb, boff, ctx->count1);
    hipLaunchKernelGGL(qba_k_scan_apply, dim3((unsigned)nb), dim3(QBA_SC_T), 0, stream, counts, ntiles, boff,
                       offsets);
  }
  QBA_HIP(hipGetLastError());
  hipLaunchKernelGGL(qba_k_compact_emit<Pred>, dim3((unsigned)ntiles), dim3(QBA_CT_THREADS), 0,
                     stream, p, n, offsets, cap);
  QBA_HIP(hipGetLastError());
  QBA_HIP(hipMemcpyAsync(count_host, ctx->count1, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
  QBA_HIP(hipStreamSynchronize(stream));
  return QBA_OK;
}
