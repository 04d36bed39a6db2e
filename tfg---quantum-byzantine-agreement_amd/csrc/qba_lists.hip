// qba_lists.hip -- C ABI of the list kernels: argument checks, 2^31-entry
// launch chunks and dispatch to the per-n instantiations (qba_lists_inst.hip).
#include "qba_lists.h"

// Experiment builds only (tools/exp): restrict instantiation to one n.
#ifndef QBA_ONLY_N
#define QBA_ONLY_N 0
#endif

// 0 for a shipped build: no experiment switch in this object or in any
// per-n list-kernel object linked with it (qba_internal.h)
extern "C" int qba_build_flags(void) {
  int f = QBA_BUILD_EXPERIMENT_FLAGS;
#define QBA_FLAG(k) \
  if constexpr (QBA_ONLY_N == 0 || k == QBA_ONLY_N) f |= qba_lists_build_flags<k>();
  QBA_FLAG(1) QBA_FLAG(2) QBA_FLAG(3) QBA_FLAG(4) QBA_FLAG(5) QBA_FLAG(6) QBA_FLAG(7) QBA_FLAG(8)
  QBA_FLAG(9) QBA_FLAG(10) QBA_FLAG(11) QBA_FLAG(12) QBA_FLAG(13) QBA_FLAG(14) QBA_FLAG(15)
#undef QBA_FLAG
  return f;
}

static int nbins_of(int n) {  // QCfg<n>::NBP
  const int g = n + 1, q = qba_nq(n), w = 1 << q;
  return (w * g * (w + 1) + w * g * (g - 1) / 2 + 2 + 3) & ~3;
}

// packed: nibble rows, ld >= ceil(count / 2) bytes
static int check_common(qba_ctx *ctx, int n, const uint8_t *lists, uint64_t count, uint64_t ld,
                        const char *who, bool packed = false) {
  if (!ctx) return qba_fail(QBA_EINVAL, std::string(who) + ": ctx is NULL");
  if (n < 1 || n > QBA_MAX_PARTIES)
    return qba_fail(QBA_EUNSUPPORTED, std::string(who) + ": n_parties must be in [1, 15]");
  if (count == 0) return QBA_OK;
  if (!lists) return qba_fail(QBA_EINVAL, std::string(who) + ": lists is NULL");
  const uint64_t need = packed ? (count + 1) / 2 : count;
  if (ld < need || (ld & 3) || (reinterpret_cast<uintptr_t>(lists) & 3))
    return qba_fail(QBA_EINVAL, std::string(who) + (packed ? ": need ld >= (count + 1) / 2" : ": need ld >= count") +
                                    ", ld % 4 == 0 and a 4-byte aligned base");
  return qba_set_device(ctx);
}

static int need_program(qba_ctx *ctx, int n, const char *who) {
  if (!ctx->compiled[n][0] || !ctx->compiled[n][1])
    return qba_fail(QBA_ESTATE, std::string(who) + ": no resource program compiled for n=" +
                                    std::to_string(n) + " (call qba_resource_compile for both kinds)");
  return QBA_OK;
}

static int batched(qba_ctx *ctx, int n, uint64_t seed_base, int64_t n_inst, uint64_t count, uint8_t *lists,
                   uint64_t ld, uint64_t inst_stride, int64_t *H, int64_t *C, int64_t *P, qba_stream stream,
                   bool packed, const char *who) {
  int rc = check_common(ctx, n, lists, count, ld, who, packed);
  if (rc) return rc;
  if (n_inst < 0 || !H || !C || !P || (n_inst > 1 && inst_stride < (uint64_t)(n + 1) * ld) ||
      (inst_stride & 3) || count >= (1ull << 31))
    return qba_fail(QBA_EINVAL, std::string(who) + ": bad arguments (inst_stride >= (n+1)*ld, "
                                "multiple of 4; count < 2^31)");
  if (n_inst == 0 || count == 0) return QBA_OK;
  if ((rc = need_program(ctx, n, who))) return rc;
  QbaBatch B{n, (const QbaProgramSet *)ctx->prog_dev[n], seed_base, n_inst, count, lists, ld,
             inst_stride, H, C, P, (hipStream_t)stream, packed ? 1 : 0};
  switch (n) {
#define QBA_CASE(k)                                                                     \
  case k:                                                                               \
    if constexpr (QBA_ONLY_N == 0 || k == QBA_ONLY_N) return qba_launch_batched<k>(ctx, B); \
    return qba_fail(QBA_EUNSUPPORTED, "experiment build");
    QBA_CASE(1) QBA_CASE(2) QBA_CASE(3) QBA_CASE(4) QBA_CASE(5) QBA_CASE(6) QBA_CASE(7)
    QBA_CASE(8) QBA_CASE(9) QBA_CASE(10) QBA_CASE(11) QBA_CASE(12) QBA_CASE(13) QBA_CASE(14)
    QBA_CASE(15)
#undef QBA_CASE
    default:
      return qba_fail(QBA_EUNSUPPORTED, "n_parties must be in [1, 15]");
  }
}

extern "C" int qba_sample_check_batched(qba_ctx *ctx, int n, uint64_t seed_base, int64_t n_inst,
                                        uint64_t count, uint8_t *lists, uint64_t ld,
                                        uint64_t inst_stride, int64_t *H, int64_t *C, int64_t *P,
                                        qba_stream stream) {
  return batched(ctx, n, seed_base, n_inst, count, lists, ld, inst_stride, H, C, P, stream, false,
                 "qba_sample_check_batched");
}

extern "C" int qba_sample_check_batched_packed(qba_ctx *ctx, int n, uint64_t seed_base, int64_t n_inst,
                                               uint64_t count, uint8_t *packed, uint64_t ld,
                                               uint64_t inst_stride, int64_t *H, int64_t *C, int64_t *P,
                                               qba_stream stream) {
  return batched(ctx, n, seed_base, n_inst, count, packed, ld, inst_stride, H, C, P, stream, true,
                 "qba_sample_check_batched_packed");
}

static int dispatch_one(qba_ctx *ctx, const QbaLaunch &L) {
  switch (L.n) {
#define QBA_CASE(k)                                                                   \
  case k:                                                                             \
    if constexpr (QBA_ONLY_N == 0 || k == QBA_ONLY_N) return qba_launch_lists<k>(ctx, L); \
    return qba_fail(QBA_EUNSUPPORTED, "experiment build");
    QBA_CASE(1) QBA_CASE(2) QBA_CASE(3) QBA_CASE(4) QBA_CASE(5) QBA_CASE(6) QBA_CASE(7)
    QBA_CASE(8) QBA_CASE(9) QBA_CASE(10) QBA_CASE(11) QBA_CASE(12) QBA_CASE(13) QBA_CASE(14)
    QBA_CASE(15)
#undef QBA_CASE
    default:
      return qba_fail(QBA_EUNSUPPORTED, "n_parties must be in [1, 15]");
  }
}

// Launches of at most QBA_CHUNK entries (32-bit in-kernel offsets, u32 bins)
// that never cross a multiple of 2^33 entries (inside a launch the high word
// of the Philox pair counter e >> 1 is constant: qba_sample_quad keeps it in
// an SGPR); chunks after the first accumulate into the caller's counts.
//
// Nibble rows: every chunk boundary is an even column (whole bytes: chunk
// sizes are multiples of 4, and an even first makes the 2^33 split even; an
// odd first never takes the pair fast path, so it needs no split), so no
// byte is shared by two launches.
static int dispatch(qba_ctx *ctx, const QbaLaunch &L0) {
  QbaLaunch L = L0;
  uint64_t done = 0;
  int rc = QBA_OK;
  constexpr uint64_t PHI_SPAN = 1ull << 33;
  const bool pk = L0.packed != 0;
  const uintptr_t VA = pk ? 3 : 7;  // the wide step's row-vector alignment - 1
  do {
    L.count = L0.count - done < ctx->chunk ? L0.count - done : ctx->chunk;
    if (!pk || !((L0.first + done) & 1)) {
      const uint64_t to_span = PHI_SPAN - ((L0.first + done) & (PHI_SPAN - 1));
      if (L.count > to_span) L.count = to_span;
    }
    // A chunk that starts off the wide kernels' row alignment (8 B; 4 B for
    // nibble rows) -- the caller's first column, or the 2^33 split above --
    // is cut to the next aligned column, so that every later chunk of the
    // call runs the wide kernel (qba_launch_lists picks the narrow one for
    // unaligned rows); rows must be aligned to begin with (ld % 8 == 0).
    uint8_t *const at = L0.lists + (pk ? done >> 1 : done);
    const uintptr_t mis = reinterpret_cast<uintptr_t>(at) & VA;
    const uint64_t cut = pk ? 2 * (4 - mis) : 8 - mis;
    if (mis && !(L0.ld & VA) && L.count > cut) L.count = cut;
    L.first = L0.first + done;
    L.lists = at;
    L.accumulate = done ? 1 : L0.accumulate;
    L.stats_accumulate = done ? 1 : 0;
    rc = dispatch_one(ctx, L);
    done += L.count;
  } while (!rc && done < L0.count);
  return rc;
}

int qba_capture_of(hipStream_t s, unsigned long long *id) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long cid = 0;
  if (hipStreamGetCaptureInfo(s, &st, &cid) != hipSuccess) st = hipStreamCaptureStatusNone;
  *id = st == hipStreamCaptureStatusActive ? cid : 0ull;
  return st == hipStreamCaptureStatusActive ? 1 : 0;
}

// A pending deferred reduction may only be launched in the capture state it
// was recorded in: an eager one into an eager stream, a captured one into the
// same capture.  Otherwise the reduction would become a graph node that
// re-reduces an overwritten slab on every replay, or an eager launch would
// reduce the slab of a graph that has not run (include/qba.h).
static int pend_capture_ok(qba_ctx *ctx, hipStream_t s) {
  unsigned long long id = 0;
  const int cap = qba_capture_of(s, &id);
  if (cap == ctx->pend_captured && (!cap || id == ctx->pend_capture_id)) return QBA_OK;
  return qba_fail(QBA_ESTATE, ctx->pend_captured
                                  ? "a deferred reduction recorded inside a graph capture is still pending outside "
                                    "it: call qba_flush_deferred before ending the capture"
                                  : "a deferred reduction is pending from before a graph capture: call "
                                    "qba_flush_deferred before beginning the capture");
}

// Only eager streams are ordered here: inside a capture the graph's own
// dependencies order its nodes, and across a capture boundary the caller
// synchronises (include/qba.h).  The previous user's stream is never touched
// (it may be destroyed since): a counting launch on another stream than the
// previous one synchronises the device, which completes that stream's work.
// A stream switch is rare; an event recorded after every counting launch
// instead put a ~6 us marker between each launch and the next on the same
// stream (profiles/r5/slab_event).
//
// Streams are told apart by their handle values (hipStreamGetId, which would
// survive a handle's reuse, is a HIP 7.1 symbol that the HIP runtime PyTorch
// ships here lacks), so a stream must be synchronised before it is destroyed
// if this ctx counted on it (include/qba.h; PyTorch pools its streams and
// never destroys them).  The device synchronisation runs in relaxed capture
// mode, so a graph that another thread captures in global mode is neither
// invalidated nor waited for (a capture has no executing work).
static unsigned long long stream_key(hipStream_t s) { return reinterpret_cast<uintptr_t>(s) | (1ull << 63); }

int qba_slab_order(qba_ctx *ctx, hipStream_t stream) {
  unsigned long long id = 0;
  if (ctx->slab_set && ctx->slab_last != stream_key(stream) && !qba_capture_of(stream, &id)) {
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    QBA_HIP(hipThreadExchangeStreamCaptureMode(&mode));
    const hipError_t e = hipDeviceSynchronize();
    (void)hipThreadExchangeStreamCaptureMode(&mode);  // restore this thread's mode
    QBA_HIP(e);
    ctx->slab_set = false;
  }
  return QBA_OK;
}

int qba_slab_done(qba_ctx *ctx, hipStream_t stream) {
  unsigned long long id = 0;
  ctx->slab_set = !qba_capture_of(stream, &id);
  ctx->slab_last = stream_key(stream);
  return QBA_OK;
}

int qba_flush_pending(qba_ctx *ctx, hipStream_t next) {
  auto &pd = ctx->pend;
  if (!pd.flush) return QBA_OK;
  if (int rc = pend_capture_ok(ctx, pd.stream)) return rc;
  if (next != pd.stream)
    if (int rc = pend_capture_ok(ctx, next)) return rc;
  int (*f)(qba_ctx *) = pd.flush;
  int rc = f(ctx);
  pd.flush = nullptr;
  if (rc || (rc = qba_slab_done(ctx, pd.stream))) return rc;  // the reduction read the slab
  if (next != pd.stream) {  // the slab may be rewritten on `next`: after this reduction
    if (!ctx->def_ev) QBA_HIP(hipEventCreateWithFlags(&ctx->def_ev, hipEventDisableTiming));
    QBA_HIP(hipEventRecord(ctx->def_ev, pd.stream));
    QBA_HIP(hipStreamWaitEvent(next, ctx->def_ev, 0));
  }
  return QBA_OK;
}

extern "C" int qba_flush_deferred(qba_ctx *ctx) {
  if (!ctx) return qba_fail(QBA_EINVAL, "qba_flush_deferred: ctx is required");
  if (!ctx->pend.flush) return QBA_OK;
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  if ((rc = pend_capture_ok(ctx, ctx->pend.stream))) {
    // a captured reduction outside its capture cannot be launched any more:
    // it is dropped (that call's counts stay incomplete) and the ctx is usable
    if (ctx->pend_captured) ctx->pend.flush = nullptr;
    return rc;
  }
  return qba_flush_pending(ctx, ctx->pend.stream);
}

static int zero_counts(qba_ctx *ctx, int n, int64_t *H, int64_t *C, int64_t *P, hipStream_t s) {
  if (int rc = qba_flush_pending(ctx, s)) return rc;  // a pending reduction may target the same outputs
  const int g = n + 1, w = 1 << qba_nq(n);
  QBA_HIP(hipMemsetAsync(H, 0, sizeof(int64_t) * w * g * w, s));
  QBA_HIP(hipMemsetAsync(C, 0, sizeof(int64_t) * w * g * g, s));
  QBA_HIP(hipMemsetAsync(P, 0, sizeof(int64_t) * w, s));
  return QBA_OK;
}

extern "C" int qba_sample(qba_ctx *ctx, int n, uint64_t seed, uint64_t first, uint64_t count,
                          uint8_t *lists, uint64_t ld, qba_stream stream) {
  int rc = check_common(ctx, n, lists, count, ld, "qba_sample");
  if (rc || count == 0) return rc;
  if ((rc = need_program(ctx, n, "qba_sample"))) return rc;
  QbaLaunch L{n, 0, (const QbaProgramSet *)ctx->prog_dev[n], seed, first, count, lists, ld,
              nullptr, nullptr, nullptr, nullptr, 0, (hipStream_t)stream};
  return dispatch(ctx, L);
}

extern "C" int qba_sample_check(qba_ctx *ctx, int n, uint64_t seed, uint64_t first,
                                uint64_t count, uint8_t *lists, uint64_t ld, int64_t *H,
                                int64_t *C, int64_t *P, int accumulate, qba_stream stream) {
  int rc = check_common(ctx, n, lists, count, ld, "qba_sample_check");
  if (rc) return rc;
  if (!H || !C || !P) return qba_fail(QBA_EINVAL, "qba_sample_check: H, C and P are required");
  if (count == 0)
    return accumulate ? qba_flush_pending(ctx, (hipStream_t)stream) : zero_counts(ctx, n, H, C, P, (hipStream_t)stream);
  if ((rc = need_program(ctx, n, "qba_sample_check"))) return rc;
  QbaLaunch L{n, 1, (const QbaProgramSet *)ctx->prog_dev[n], seed, first, count, lists, ld,
              H, C, P, ctx->stats, accumulate, (hipStream_t)stream};
  return dispatch(ctx, L);
}

extern "C" int qba_sample_check_deferred(qba_ctx *ctx, int n, uint64_t seed, uint64_t first,
                                         uint64_t count, uint8_t *lists, uint64_t ld, int64_t *H,
                                         int64_t *C, int64_t *P, int accumulate, qba_stream stream) {
  int rc = check_common(ctx, n, lists, count, ld, "qba_sample_check_deferred");
  if (rc) return rc;
  if (!H || !C || !P) return qba_fail(QBA_EINVAL, "qba_sample_check_deferred: H, C and P are required");
  if (count == 0)
    return accumulate ? qba_flush_pending(ctx, (hipStream_t)stream) : zero_counts(ctx, n, H, C, P, (hipStream_t)stream);
  if ((rc = need_program(ctx, n, "qba_sample_check_deferred"))) return rc;
  QbaLaunch L{n, 1, (const QbaProgramSet *)ctx->prog_dev[n], seed, first, count, lists, ld,
              H, C, P, ctx->stats, accumulate, (hipStream_t)stream, 0, 0, 1};
  return dispatch(ctx, L);
}

extern "C" int qba_check_counts(qba_ctx *ctx, int n, const uint8_t *lists, uint64_t count,
                                uint64_t ld, int64_t *H, int64_t *C, int64_t *P, int accumulate,
                                qba_stream stream) {
  int rc = check_common(ctx, n, lists, count, ld, "qba_check_counts");
  if (rc) return rc;
  if (!H || !C || !P) return qba_fail(QBA_EINVAL, "qba_check_counts: H, C and P are required");
  if (count == 0)
    return accumulate ? qba_flush_pending(ctx, (hipStream_t)stream) : zero_counts(ctx, n, H, C, P, (hipStream_t)stream);
  QbaLaunch L{n, 2, nullptr, 0, 0, count, const_cast<uint8_t *>(lists), ld,
              H, C, P, ctx->stats, accumulate, (hipStream_t)stream};
  return dispatch(ctx, L);
}

// ---- nibble rows ("packed lists", qba.h) ----------------------------------------
extern "C" int qba_sample_packed(qba_ctx *ctx, int n, uint64_t seed, uint64_t first, uint64_t count,
                                 uint8_t *packed, uint64_t ldp, qba_stream stream) {
  int rc = check_common(ctx, n, packed, count, ldp, "qba_sample_packed", true);
  if (rc || count == 0) return rc;
  if ((rc = need_program(ctx, n, "qba_sample_packed"))) return rc;
  QbaLaunch L{n, 0, (const QbaProgramSet *)ctx->prog_dev[n], seed, first, count, packed, ldp,
              nullptr, nullptr, nullptr, nullptr, 0, (hipStream_t)stream, 0, 1};
  return dispatch(ctx, L);
}

extern "C" int qba_sample_check_packed(qba_ctx *ctx, int n, uint64_t seed, uint64_t first,
                                       uint64_t count, uint8_t *packed, uint64_t ldp, int64_t *H,
                                       int64_t *C, int64_t *P, int accumulate, qba_stream stream) {
  int rc = check_common(ctx, n, packed, count, ldp, "qba_sample_check_packed", true);
  if (rc) return rc;
  if (!H || !C || !P) return qba_fail(QBA_EINVAL, "qba_sample_check_packed: H, C and P are required");
  if (count == 0)
    return accumulate ? qba_flush_pending(ctx, (hipStream_t)stream) : zero_counts(ctx, n, H, C, P, (hipStream_t)stream);
  if ((rc = need_program(ctx, n, "qba_sample_check_packed"))) return rc;
  QbaLaunch L{n, 1, (const QbaProgramSet *)ctx->prog_dev[n], seed, first, count, packed, ldp,
              H, C, P, ctx->stats, accumulate, (hipStream_t)stream, 0, 1};
  return dispatch(ctx, L);
}

extern "C" int qba_sample_check_packed_deferred(qba_ctx *ctx, int n, uint64_t seed, uint64_t first,
                                                uint64_t count, uint8_t *packed, uint64_t ldp, int64_t *H,
                                                int64_t *C, int64_t *P, int accumulate, qba_stream stream) {
  int rc = check_common(ctx, n, packed, count, ldp, "qba_sample_check_packed_deferred", true);
  if (rc) return rc;
  if (!H || !C || !P) return qba_fail(QBA_EINVAL, "qba_sample_check_packed_deferred: H, C and P are required");
  if (count == 0)
    return accumulate ? qba_flush_pending(ctx, (hipStream_t)stream) : zero_counts(ctx, n, H, C, P, (hipStream_t)stream);
  if ((rc = need_program(ctx, n, "qba_sample_check_packed_deferred"))) return rc;
  QbaLaunch L{n, 1, (const QbaProgramSet *)ctx->prog_dev[n], seed, first, count, packed, ldp,
              H, C, P, ctx->stats, accumulate, (hipStream_t)stream, 0, 1, 1};
  return dispatch(ctx, L);
}

extern "C" int qba_check_counts_packed(qba_ctx *ctx, int n, const uint8_t *packed, uint64_t count,
                                       uint64_t ldp, int64_t *H, int64_t *C, int64_t *P, int accumulate,
                                       qba_stream stream) {
  int rc = check_common(ctx, n, packed, count, ldp, "qba_check_counts_packed", true);
  if (rc) return rc;
  if (!H || !C || !P) return qba_fail(QBA_EINVAL, "qba_check_counts_packed: H, C and P are required");
  if (count == 0)
    return accumulate ? qba_flush_pending(ctx, (hipStream_t)stream) : zero_counts(ctx, n, H, C, P, (hipStream_t)stream);
  QbaLaunch L{n, 2, nullptr, 0, 0, count, const_cast<uint8_t *>(packed), ldp,
              H, C, P, ctx->stats, accumulate, (hipStream_t)stream, 0, 1};
  return dispatch(ctx, L);
}

// Byte rows <-> nibble rows, one packed byte per thread (conversion helpers,
// not on the hot path).  bad counts values > 15 (not representable; their
// nibble is stored as value & 15).
__global__ void qba_k_pack(const uint8_t *__restrict__ lists, uint64_t ld, uint64_t count, uint64_t nbytes,
                           uint64_t total, uint8_t *__restrict__ packed, uint64_t ldp,
                           unsigned long long *__restrict__ bad) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t g = t / nbytes, b = t - g * nbytes, c = 2 * b;
    const uint8_t *r = lists + g * ld;
    const uint32_t lo = r[c], hi = c + 1 < count ? r[c + 1] : 0u;
    if (bad && (lo > 15u || hi > 15u)) atomicAdd(bad, (unsigned long long)((lo > 15u) + (hi > 15u)));
    packed[g * ldp + b] = (uint8_t)((lo & 15u) | ((hi & 15u) << 4));
  }
}

__global__ void qba_k_unpack(const uint8_t *__restrict__ packed, uint64_t ldp, uint64_t count, uint64_t nbytes,
                             uint64_t total, uint8_t *__restrict__ lists, uint64_t ld) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t g = t / nbytes, b = t - g * nbytes, c = 2 * b;
    const uint32_t v = packed[g * ldp + b];
    uint8_t *r = lists + g * ld;
    r[c] = (uint8_t)(v & 15u);
    if (c + 1 < count) r[c + 1] = (uint8_t)(v >> 4);
  }
}

static int convert_args(qba_ctx *ctx, const void *a, const void *b, int rows, uint64_t count, uint64_t ld,
                        uint64_t ldp, const char *who) {
  if (!ctx || rows < 0 || (rows && count && (!a || !b)) || (rows && count && (ld < count || ldp < (count + 1) / 2)))
    return qba_fail(QBA_EINVAL, std::string(who) + ": bad arguments (ld >= count, ldp >= (count + 1) / 2)");
  return qba_set_device(ctx);
}

static dim3 convert_grid(uint64_t total) {
  const uint64_t b = (total + 255) / 256;
  return dim3((unsigned)(b < 65536 ? (b ? b : 1) : 65536));
}

extern "C" int qba_lists_pack(qba_ctx *ctx, const uint8_t *lists, uint64_t ld, int rows, uint64_t count,
                              uint8_t *packed, uint64_t ldp, int64_t *bad_dev, qba_stream stream) {
  int rc = convert_args(ctx, lists, packed, rows, count, ld, ldp, "qba_lists_pack");
  if (rc) return rc;
  if (bad_dev) QBA_HIP(hipMemsetAsync(bad_dev, 0, sizeof(int64_t), (hipStream_t)stream));
  const uint64_t nbytes = (count + 1) / 2, total = (uint64_t)rows * nbytes;
  if (total == 0) return QBA_OK;
  hipLaunchKernelGGL(qba_k_pack, convert_grid(total), dim3(256), 0, (hipStream_t)stream, lists, ld, count, nbytes,
                     total, packed, ldp, reinterpret_cast<unsigned long long *>(bad_dev));
  QBA_HIP(hipGetLastError());
  return QBA_OK;
}

extern "C" int qba_lists_unpack(qba_ctx *ctx, const uint8_t *packed, uint64_t ldp, int rows, uint64_t count,
                                uint8_t *lists, uint64_t ld, qba_stream stream) {
  int rc = convert_args(ctx, packed, lists, rows, count, ld, ldp, "qba_lists_unpack");
  if (rc) return rc;
  const uint64_t nbytes = (count + 1) / 2, total = (uint64_t)rows * nbytes;
  if (total == 0) return QBA_OK;
  hipLaunchKernelGGL(qba_k_unpack, convert_grid(total), dim3(256), 0, (hipStream_t)stream, packed, ldp, count,
                     nbytes, total, lists, ld);
  QBA_HIP(hipGetLastError());
  return QBA_OK;
}

extern "C" int qba_reserve(qba_ctx *ctx, int n, int64_t max_blocks) {
  if (!ctx || n < 1 || n > QBA_MAX_PARTIES || max_blocks < 1)
    return qba_fail(QBA_EINVAL, "qba_reserve: bad arguments");
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  if (ctx->pend.flush && (rc = qba_flush_pending(ctx, ctx->pend.stream))) return rc;  // before a reallocation
  return qba_ensure_slab(ctx, (size_t)max_blocks * nbins_of(n) * sizeof(uint32_t));
}

// ---------------------------------------------------------------------------
// Philox KAT helper
// ---------------------------------------------------------------------------
__global__ void qba_k_philox(const uint32_t *__restrict__ ctr, int64_t n, uint32_t k0, uint32_t k1,
                             uint32_t *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const QbaU4 r = qba_philox(ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3], k0, k1);
  out[4 * i] = r.x;
  out[4 * i + 1] = r.y;
  out[4 * i + 2] = r.z;
  out[4 * i + 3] = r.w;
}

extern "C" int qba_philox_dev(qba_ctx *ctx, const uint32_t *ctr, int64_t n, uint64_t key,
                              uint32_t *out, qba_stream stream) {
  if (!ctx || n < 0 || (n && (!ctr || !out))) return qba_fail(QBA_EINVAL, "qba_philox_dev: bad arguments");
  if (n == 0) return QBA_OK;
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  hipLaunchKernelGGL(qba_k_philox, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, ctr, n, (uint32_t)key, (uint32_t)(key >> 32), out);
  QBA_HIP(hipGetLastError());
  return QBA_OK;
}
