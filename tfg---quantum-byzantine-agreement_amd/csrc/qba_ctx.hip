// qba_ctx.hip -- library context, error channel and scratch management.
#include <stdio.h>
#include <stdlib.h>

#include <string>

#include "qba_internal.h"

static thread_local std::string g_last_error;

int qba_fail(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}

extern "C" const char *qba_last_error(void) { return g_last_error.c_str(); }

extern "C" int qba_version(void) { return 100; /* 0.1.0 */ }

int qba_set_device(qba_ctx *ctx) {
  int cur = -1;
  QBA_HIP(hipGetDevice(&cur));
  if (cur != ctx->device) QBA_HIP(hipSetDevice(ctx->device));
  return QBA_OK;
}

extern "C" int qba_init(int device, qba_ctx **out) {
  if (!out) return qba_fail(QBA_EINVAL, "qba_init: out is NULL");
  *out = nullptr;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0)
    return qba_fail(QBA_EHIP, "qba_init: no HIP device visible (" +
                                  std::string(hipGetErrorString(e)) + ")");
  if (device < 0 || device >= ndev)
    return qba_fail(QBA_EINVAL, "qba_init: device " + std::to_string(device) + " out of range");
  QBA_HIP(hipSetDevice(device));
  hipDeviceProp_t prop;
  QBA_HIP(hipGetDeviceProperties(&prop, device));
  std::string arch = prop.gcnArchName;
  if (arch.rfind("gfx950", 0) != 0)
    return qba_fail(QBA_EUNSUPPORTED, "qba_init: built for gfx950 (MI355X), found " + arch);
  qba_ctx *ctx = new qba_ctx();
  ctx->device = device;
  ctx->num_cus = prop.multiProcessorCount;
  if (hipMalloc(&ctx->flag, 64) != hipSuccess || hipMalloc(&ctx->count1, 64) != hipSuccess ||
      hipMalloc(&ctx->stats, 64) != hipSuccess || hipMemset(ctx->stats, 0, 64) != hipSuccess) {
    qba_destroy(ctx);
    return qba_fail(QBA_ENOMEM, "qba_init: device scratch allocation failed");
  }
  *out = ctx;
  return QBA_OK;
}

// qba_lists.hip; absent from the host-only sanitizer build (no list kernels)
extern "C" __attribute__((weak)) int qba_flush_deferred(qba_ctx *ctx);

// Test seam (include/qba.h): the launch-shape knobs the GPU tests use to
// drive chunk splits, pair bins on small launches and pair-bin wraps.  The
// library never reads them from the environment; a ctx nobody calls this on
// runs the shipped selection.
extern "C" int qba_test_set_knobs(qba_ctx *ctx, uint64_t chunk_entries, int64_t pb_min_entries, int list_grid) {
  if (!ctx || chunk_entries > QBA_CHUNK || (chunk_entries && chunk_entries < 4) || list_grid < 0 ||
      list_grid >= (1 << 20))
    return qba_fail(QBA_EINVAL, "qba_test_set_knobs: bad arguments");
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  // a pending deferred reduction was recorded under the old launch shape
  if (ctx->pend.flush && qba_flush_deferred && (rc = qba_flush_deferred(ctx))) return rc;
  ctx->chunk = chunk_entries ? (chunk_entries & ~3ull) : QBA_CHUNK;
  ctx->pb_min = pb_min_entries < 0 ? QBA_PB_MIN_DEFAULT : (uint64_t)pb_min_entries;
  ctx->list_grid = list_grid;
  return QBA_OK;
}

extern "C" int qba_destroy(qba_ctx *ctx) {
  if (!ctx) return QBA_OK;
  (void)hipSetDevice(ctx->device);
  // a pending deferred reduction completes its call's counts before the slab goes
  if (ctx->pend.flush && qba_flush_deferred && qba_flush_deferred(ctx) == QBA_OK) (void)hipDeviceSynchronize();
  qba_rccl_release(ctx);
  for (int n = 0; n <= QBA_MAX_PARTIES; ++n) {
    if (ctx->prog_dev[n]) (void)hipFree(ctx->prog_dev[n]);
    free(ctx->prog_host[n]);
  }
  if (ctx->slab) (void)hipFree(ctx->slab);
  if (ctx->scan) (void)hipFree(ctx->scan);
  if (ctx->flag) (void)hipFree(ctx->flag);
  if (ctx->count1) (void)hipFree(ctx->count1);
  if (ctx->stats) (void)hipFree(ctx->stats);
  if (ctx->zc_pending) (void)hipEventSynchronize(ctx->zc_ev);
  if (ctx->zc_ev) (void)hipEventDestroy(ctx->zc_ev);
  if (ctx->def_ev) (void)hipEventDestroy(ctx->def_ev);
  if (ctx->zc) (void)hipHostFree(ctx->zc);
  if (ctx->pin_h) (void)hipHostFree(ctx->pin_h);
  if (ctx->pin_d) (void)hipFree(ctx->pin_d);
  delete ctx;
  return QBA_OK;
}

static int ensure(void *&ptr, size_t &have, size_t want, const char *what) {
  if (have >= want) return QBA_OK;
  if (ptr) {
    QBA_HIP(hipDeviceSynchronize());
    QBA_HIP(hipFree(ptr));
    ptr = nullptr;
    have = 0;
  }
  size_t sz = want + want / 4 + 4096;
  if (hipMalloc(&ptr, sz) != hipSuccess)
    return qba_fail(QBA_ENOMEM, std::string("scratch allocation failed: ") + what);
  have = sz;
  return QBA_OK;
}

int qba_ensure_slab(qba_ctx *ctx, size_t bytes) { return ensure(ctx->slab, ctx->slab_bytes, bytes, "slab"); }
int qba_ensure_scan(qba_ctx *ctx, size_t bytes) { return ensure(ctx->scan, ctx->scan_bytes, bytes, "scan"); }

// pinned host staging (hipHostMalloc) + device staging for the synchronous
// host-pointer entry points: one H2D, the kernel(s), one D2H, one sync.
int qba_ensure_staging(qba_ctx *ctx, size_t host_bytes, size_t dev_bytes) {
  if (ctx->pin_h_bytes < host_bytes) {
    if (ctx->pin_h) QBA_HIP(hipHostFree(ctx->pin_h));
    ctx->pin_h = nullptr;
    ctx->pin_h_bytes = 0;
    const size_t sz = host_bytes + host_bytes / 4 + 65536;
    if (hipHostMalloc(&ctx->pin_h, sz, hipHostMallocDefault) != hipSuccess)
      return qba_fail(QBA_ENOMEM, "pinned staging allocation failed");
    ctx->pin_h_bytes = sz;
  }
  return ensure(ctx->pin_d, ctx->pin_d_bytes, dev_bytes, "device staging");
}

int qba_ensure_zc(qba_ctx *ctx, size_t bytes) {
  if (ctx->zc_pending) {  // an asynchronous kernel may still read the staging
    QBA_HIP(hipEventSynchronize(ctx->zc_ev));
    ctx->zc_pending = false;
  }
  if (ctx->zc_bytes >= bytes) return QBA_OK;
  if (ctx->zc) QBA_HIP(hipHostFree(ctx->zc));
  ctx->zc = ctx->zc_d = nullptr;
  ctx->zc_bytes = 0;
  const size_t sz = bytes < 65536 ? 65536 : bytes + bytes / 4;
  if (hipHostMalloc(&ctx->zc, sz, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
    return qba_fail(QBA_ENOMEM, "zero-copy staging allocation failed");
  if (hipHostGetDevicePointer(&ctx->zc_d, ctx->zc, 0) != hipSuccess) {
    (void)hipHostFree(ctx->zc);
    ctx->zc = nullptr;
    return qba_fail(QBA_EHIP, "zero-copy staging: no device address");
  }
  ctx->zc_bytes = sz;
  return QBA_OK;
}

extern "C" int qba_last_stats(qba_ctx *ctx, int64_t *out2) {
  if (!ctx || !out2) return qba_fail(QBA_EINVAL, "qba_last_stats: bad arguments");
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  if (qba_flush_deferred && (rc = qba_flush_deferred(ctx))) return rc;  // the last call's stats follow its reduction
  QBA_HIP(hipDeviceSynchronize());
  QBA_HIP(hipMemcpy(out2, ctx->stats, 2 * sizeof(int64_t), hipMemcpyDeviceToHost));
  return QBA_OK;
}
