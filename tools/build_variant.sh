#!/bin/bash
# Build an A/B variant of libmox.so with extra -D flags into build/var_NAME/
# (bench.py / tests load it with MOX_LIB=build/var_NAME/libmox.so, or
# mox.Engine(lib_path=...)).
# Usage: bash tools/build_variant.sh NAME "-DFLAG ..."
# SRC=DIR builds DIR's sources instead of map-oxidize_amd/csrc (e.g. an older
# commit's, exported with tools/export_src.sh).
set -e
NAME=$1; shift
FLAGS="-DMOX_EXPERIMENT_BUILD $*"  # experiment builds only (mox_internal.h: ablation switches)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build/var_$NAME
mkdir -p $OUT
H="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result"
K=${KFLAGS:-"-mllvm -amdgpu-sched-strategy=max-memory-clause"}  # KFLAGS: another kernel scheduler for an A/B
C=${SRC:-$ROOT/map-oxidize_amd/csrc}
rm -f $OUT/*.o $OUT/libmox.so
$H $K $FLAGS -c $C/mox_kernels.hip -o $OUT/k.o & P1=$!
$H $FLAGS -c $C/mox_engine.hip -o $OUT/e.o & P2=$!
$H $FLAGS -c $C/mox_multi.hip -o $OUT/m.o & P3=$!
$H $K $FLAGS -c $C/mox_bsort.hip -o $OUT/b.o & P4=$!
g++ -O3 -std=c++17 -fPIC -c $C/mox_table.cpp -o $OUT/t.o & P5=$!
wait $P1 && wait $P2 && wait $P3 && wait $P4 && wait $P5
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/libmox.so $OUT/k.o $OUT/e.o $OUT/m.o $OUT/b.o $OUT/t.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built $OUT/libmox.so"
