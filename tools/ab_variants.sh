#!/bin/bash
# Timing-only builds of libomg.so with -D<macro>=<n> (n = 1..N) into
# octree-mg_amd/_variants/, for kernel A/B under OMG_LIB.  Results of these
# builds are wrong by design; nothing but tools/ loads them.
#   tools/ab_variants.sh OMG_PS_VARIANT 3
set -e
cd "$(dirname "$0")/../octree-mg_amd/csrc"
M=$1; N=$2
mkdir -p ../_variants
for n in $(seq 1 "$N"); do
  d=/tmp/omg_var_$n; mkdir -p $d
  for f in omg_kernels omg_sweep omg_tiles; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I/opt/rocm/include \
      -D$M=$n -c -o $d/$f.o $f.hip &
  done
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I/opt/rocm/include \
    -D$M=$n -x hip -c -o $d/omg_api.o omg_api.cpp &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -o ../_variants/libomg_v$n.so $d/*.o -shared -L/opt/rocm/lib -lrccl \
    -Wl,-rpath,/opt/rocm/lib
done
ls -la ../_variants
