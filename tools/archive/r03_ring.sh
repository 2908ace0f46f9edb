#!/bin/bash
# Kernel-trace the lexicographic sweep (tools/sweep_bench.py smooth_gs, 512^3)
# for the default library and each timing build in octree-mg_amd/_variants
# (tools/ab_build.sh); prints the average duration of the sweep kernel.
#   tools/r03_ring.sh <tag> [variant ...]
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r03/$1; shift
mkdir -p $O
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib=$R/octree-mg_amd/_variants/libomg_$v.so
  (cd /tmp && OMG_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv \
     -- python3 $R/tools/sweep_bench.py 10 512 smooth_gs) > $O/$v.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/$v.log; exit 1; }
  f=$(find $O/$v -name "*kernel_trace.csv" | head -1)
  echo "== $v: $(grep smooth_gs $O/$v.log)"
  python3 $R/tools/trace_by_grid.py $f "gs_lex|rhs_|fill" | head -6
done
