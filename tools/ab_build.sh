#!/bin/bash
# Timing-only builds of libomg.so with extra compile flags, for kernel A/B
# under OMG_LIB (tools/ab_run.sh).  Each argument is name:flags, e.g.
#   tools/ab_build.sh lpw16:-DOMG_SUMS_LPW=16 pre:-DOMG_PS_PRE=1
# -> octree-mg_amd/_variants/libomg_<name>.so.  Nothing but tools/ loads them.
set -e
cd "$(dirname "$0")/../octree-mg_amd/csrc"
mkdir -p ../_variants
rm -f ../_variants/libomg_*.so
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  d=/tmp/omg_var_$name; mkdir -p $d
  for f in omg_kernels omg_sweep omg_tiles omg_free; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I/opt/rocm/include \
      $flags -c -o $d/$f.o $f.hip &
  done
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I/opt/rocm/include \
    $flags -x hip -c -o $d/omg_api.o omg_api.cpp &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -o ../_variants/libomg_$name.so $d/*.o -shared -L/opt/rocm/lib -lrccl -lhipfft -lrocprofiler-sdk-roctx \
    -Wl,-rpath,/opt/rocm/lib
done
ls -la ../_variants
