// qba_lists_inst.hip -- one n's list kernels and launchers; built once per
// n = 1..15 with -DQBA_INST_N=n (csrc/Makefile), in parallel.
#include "qba_lists_kern.h"

#ifndef QBA_INST_N
#error "build with -DQBA_INST_N=<n>"
#endif

template int qba_launch_lists<QBA_INST_N>(qba_ctx *ctx, const QbaLaunch &L);
template int qba_launch_batched<QBA_INST_N>(qba_ctx *ctx, const QbaBatch &B);
template <> int qba_lists_build_flags<QBA_INST_N>() { return QBA_BUILD_EXPERIMENT_FLAGS; }
