#!/bin/bash
# Experiment builds of libqba (one n: N=<n>, default 11) for A/B timing on the GPU box.
# Usage: tools/exp/build.sh name [-DFLAG ...]
#   SRC=<dir>  build the list kernels from another copy of csrc/ (e.g. a
#              `git show <rev>:...` export) instead of the working tree.
#   PROBES=1   apply tools/exp/probes.patch to a copy first: the attribution
#              probes (-DQBA_EXP_NOSTORE, _NOATOMIC, _NOCOND3, _CHEAPRNG, _TIMING,
#              ...) and the switches of the rejected variants, as of round 5.
set -e
here="$(cd "$(dirname "$0")/../../tfg---quantum-byzantine-agreement_amd/csrc" && pwd)"
src=${SRC:-$here}
if [ -n "$PROBES" ]; then
  tmp=$(mktemp -d); mkdir -p $tmp/csrc; cp $src/* $tmp/csrc/ 2>/dev/null || true
  pp="$(cd "$(dirname "$0")" && pwd)/probes.patch"; (cd $tmp && patch -s -p1 < "$pp")
  src=$tmp/csrc
fi
name=$1; shift
N=${N:-11}
out=${EXPOUT:-$here/../_build/exp}; mkdir -p $out
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -fvisibility=hidden -munsafe-fp-atomics -I$here -I$here/../../include -DQBA_EXPERIMENT_BUILD"
/opt/rocm/bin/hipcc $F -DQBA_ONLY_N=$N "$@" -c $src/qba_lists.hip -o $out/$name.o
# the shipped list kernels take their arguments preloaded (csrc/Makefile PRELOAD)
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-kernarg-preload-count=16 -DQBA_INST_N=$N "$@" -c $src/qba_lists_inst.hip -o $out/${name}_n$N.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/$name.so $out/$name.o $out/${name}_n$N.o \
  $here/../_build/qba_ctx.o $here/../_build/qba_exact.o $here/../_build/qba_sv.o $here/../_build/qba_resource.o \
  $here/../_build/qba_rccl.o $here/../_build/qba_plan.o $here/../_build/qba_host.o -ldl
rm -f $out/$name.o $out/${name}_n$N.o
