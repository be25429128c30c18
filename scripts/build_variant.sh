#!/bin/bash
# Build an A/B variant of libqlx.so into abvar/<name>/libqlx.so: qnet32.hip recompiled with extra flags (e.g.
# -DQLX_Q32_NO_SWZ), every other object taken from the main build.  Use with QLX_LIB_PATH=abvar/<name>/libqlx.so.
# VARIANT_SRC=qnet rebuilds qnet.hip (the bf16 Q-net) instead; VARIANT_SCHED replaces the scheduler flags.
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p abvar/$name
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-result -I include -I q-learning_amd/csrc -munsafe-fp-atomics -ffp-contract=off ${VARIANT_SCHED--mllvm --amdgpu-sched-strategy=max-ilp} ${VARIANT_VFORM--mllvm -amdgpu-mfma-vgpr-form=1}"
src=${VARIANT_SRC:-qnet32}
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -c q-learning_amd/csrc/$src.hip -o abvar/$name/$src.o
objs=$(ls q-learning_amd/lib/obj/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 $objs abvar/$name/$src.o -shared -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib -o abvar/$name/libqlx.so
echo abvar/$name/libqlx.so
