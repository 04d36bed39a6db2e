// qba_rccl.hip -- the one collective of the multi-GPU path:
// a sum all-reduce of the int64 count buffer [H | C | P] over the GPU-owner
// ranks, RCCL over xGMI.  For C-ABI callers that do not use torch.distributed
// (an mpiexec launch of the tfg.py host: the unique id travels over MPI).
//
// librccl is opened on first use (dlopen), so libqba loads and runs its
// single-GPU paths without it.
#include <dlfcn.h>
#include <string.h>

#include <rccl/rccl.h>

#include "qba_internal.h"

namespace {
struct Rccl {
  void *h = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  const char *(*error_string)(ncclResult_t) = nullptr;
};

int rccl(Rccl *&out) {
  static Rccl r;
  static bool tried = false;
  if (!tried) {
    tried = true;
    for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      r.h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
      if (r.h) break;
    }
    if (r.h) {
      r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(r.h, "ncclGetUniqueId"));
      r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(r.h, "ncclCommInitRank"));
      r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(r.h, "ncclAllReduce"));
      r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(r.h, "ncclCommDestroy"));
      r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(r.h, "ncclGetErrorString"));
    }
  }
  if (!r.get_unique_id || !r.comm_init_rank || !r.all_reduce || !r.comm_destroy || !r.error_string)
    return qba_fail(QBA_EUNSUPPORTED, "RCCL (librccl.so) is not available");
  out = &r;
  return QBA_OK;
}

int rccl_fail(Rccl *r, ncclResult_t e, const char *what) {
  return qba_fail(QBA_EHIP, std::string(what) + ": " + r->error_string(e));
}
}  // namespace

extern "C" int qba_rccl_unique_id(uint8_t *id_host) {
  if (!id_host) return qba_fail(QBA_EINVAL, "qba_rccl_unique_id: id is NULL");
  Rccl *r;
  if (int rc = rccl(r)) return rc;
  ncclUniqueId id;
  if (ncclResult_t e = r->get_unique_id(&id)) return rccl_fail(r, e, "ncclGetUniqueId");
  memcpy(id_host, id.internal, NCCL_UNIQUE_ID_BYTES);
  return QBA_OK;
}

extern "C" int qba_rccl_init(qba_ctx *ctx, const uint8_t *id_host, int nranks, int rank) {
  if (!ctx || !id_host || nranks < 1 || rank < 0 || rank >= nranks)
    return qba_fail(QBA_EINVAL, "qba_rccl_init: bad arguments");
  Rccl *r;
  if (int rc = rccl(r)) return rc;
  if (int rc = qba_set_device(ctx)) return rc;
  if (ctx->rccl_comm) {
    r->comm_destroy(reinterpret_cast<ncclComm_t>(ctx->rccl_comm));
    ctx->rccl_comm = nullptr;
  }
  ncclUniqueId id;
  memcpy(id.internal, id_host, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t comm;
  if (ncclResult_t e = r->comm_init_rank(&comm, nranks, id, rank)) return rccl_fail(r, e, "ncclCommInitRank");
  ctx->rccl_comm = comm;
  ctx->rccl_ranks = nranks;
  return QBA_OK;
}

extern "C" int qba_allreduce_i64(qba_ctx *ctx, int64_t *buf_dev, int64_t count, qba_stream stream) {
  if (!ctx || (!buf_dev && count) || count < 0) return qba_fail(QBA_EINVAL, "qba_allreduce_i64: bad arguments");
  if (!ctx->rccl_comm) return qba_fail(QBA_ESTATE, "qba_allreduce_i64: no communicator (qba_rccl_init)");
  if (!count) return QBA_OK;
  Rccl *r;
  if (int rc = rccl(r)) return rc;
  if (int rc = qba_set_device(ctx)) return rc;
  if (ncclResult_t e = r->all_reduce(buf_dev, buf_dev, (size_t)count, ncclInt64, ncclSum,
                                     reinterpret_cast<ncclComm_t>(ctx->rccl_comm),
                                     reinterpret_cast<hipStream_t>(stream)))
    return rccl_fail(r, e, "ncclAllReduce");
  return QBA_OK;
}

// called by qba_destroy
void qba_rccl_release(qba_ctx *ctx) {
  if (!ctx->rccl_comm) return;
  Rccl *r;
  if (rccl(r) == QBA_OK) r->comm_destroy(reinterpret_cast<ncclComm_t>(ctx->rccl_comm));
  ctx->rccl_comm = nullptr;
}
