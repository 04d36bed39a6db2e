// qba_lists.h -- interface between the list-kernel dispatch (qba_lists.hip)
// and the per-n kernel instantiations (qba_lists_inst.hip, one object per n:
// the templates in qba_lists_kern.h are compiled 15 times in parallel).
#pragma once

#include "qba_internal.h"

struct QbaLaunch {
  int n;
  int mode;
  const QbaProgramSet *ps;
  uint64_t seed, first, count;
  uint8_t *lists;
  uint64_t ld;
  int64_t *H, *C, *P, *stats;
  int accumulate;
  hipStream_t stream;
  int stats_accumulate;
  int packed;  // nibble rows (qba.h "packed lists"): ld is the packed row stride in bytes
  int defer;   // MODE 1: reduction deferred to the next deferred call / qba_flush_deferred
};

struct QbaBatch {
  int n;
  const QbaProgramSet *ps;
  uint64_t seed_base;
  int64_t n_inst;
  uint64_t count;
  uint8_t *lists;
  uint64_t ld, inst_stride;
  int64_t *H, *C, *P;
  hipStream_t stream;
  int packed;  // nibble rows: ld / inst_stride in bytes of packed rows
};

template <int NP>
int qba_launch_lists(qba_ctx *ctx, const QbaLaunch &L);
// Launch the pending deferred reduction (if any) on its stream; a later launch
// on stream `next` that reuses the slab then waits for it.
int qba_flush_pending(qba_ctx *ctx, hipStream_t next);
template <int NP>
int qba_launch_batched(qba_ctx *ctx, const QbaBatch &B);
// QBA_BUILD_EXPERIMENT_FLAGS of the per-n object (qba_build_flags ORs them)
template <int NP>
int qba_lists_build_flags();
