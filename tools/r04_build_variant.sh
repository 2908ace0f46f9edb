#!/bin/bash
# one timing-only build of libomg.so with extra compile flags, for A/B under
# OMG_LIB:  tools/r04_build_variant.sh name "<flags>"  ->  octree-mg_amd/_variants/libomg_<name>.so
set -e
cd "$(dirname "$0")/../octree-mg_amd/csrc"
mkdir -p ../_variants
name=$1; flags=$2
d=/tmp/omg_var_$name; mkdir -p $d
for f in omg_kernels omg_sweep omg_tiles omg_free; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I/opt/rocm/include \
    $flags -c -o $d/$f.o $f.hip &
done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I/opt/rocm/include \
  $flags -x hip -c -o $d/omg_api.o omg_api.cpp &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -o ../_variants/libomg_$name.so $d/*.o -shared -L/opt/rocm/lib -lrccl -lhipfft \
  -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
ls -la ../_variants/libomg_$name.so
