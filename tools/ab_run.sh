#!/bin/bash
# Kernel traces of tools/sweep_bench.py <op> for the default library and each
# octree-mg_amd/_variants/libomg_v*.so (see tools/ab_variants.sh).
#   tools/ab_run.sh [op] [reps]  -> gpurun_out/ab/<name>/run_kernel_trace.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OP=${1:-vcycle}; REPS=${2:-5}
R=$PWD
for lib in default $(ls $R/octree-mg_amd/_variants/libomg_*.so 2>/dev/null); do
  name=$(basename "$lib" .so)
  if [ "$lib" = default ]; then unset OMG_LIB; else export OMG_LIB=$lib; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/ab/$name" -o run --output-format csv \
     -- python3 "$R/tools/sweep_bench.py" $REPS 512 $OP) > "$R/gpurun_out/ab_$name.log" 2>&1 || exit $?
done
