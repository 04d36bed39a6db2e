#!/bin/bash
# Experiment builds of libqba (n = 11 only) with cost knobs switched off, to
# attribute the fused kernel's time.  Usage: tools/exp/build.sh name [-DFLAG ...]
set -e
cd "$(dirname "$0")/../../tfg---quantum-byzantine-agreement_amd/csrc"
name=$1; shift
out=../_build/exp; mkdir -p $out
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -fvisibility=hidden -munsafe-fp-atomics"
/opt/rocm/bin/hipcc $F -DQBA_ONLY_N=11 "$@" -c qba_lists.hip -o $out/$name.o
/opt/rocm/bin/hipcc $F -DQBA_INST_N=11 "$@" -c qba_lists_inst.hip -o $out/${name}_n11.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/$name.so $out/$name.o $out/${name}_n11.o \
  ../_build/qba_ctx.o ../_build/qba_exact.o ../_build/qba_sv.o ../_build/qba_resource.o
