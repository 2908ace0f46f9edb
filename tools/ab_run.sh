#!/bin/bash
# Kernel traces of tools/sweep_bench.py <op> for the default library and each
# octree-mg_amd/_variants/libomg_v*.so (see tools/ab_variants.sh).
#   tools/ab_run.sh [op] [reps] [rounds]  -> gpurun_out/ab/<name>[_r<round>]/run_kernel_trace.csv
# (rounds > 1 interleaves the libraries, for box-to-box and run-to-run noise)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OP=${1:-vcycle}; REPS=${2:-5}; ROUNDS=${3:-1}
R=$PWD
for round in $(seq 1 "$ROUNDS"); do
for lib in default $(ls $R/octree-mg_amd/_variants/libomg_*.so 2>/dev/null); do
  name=$(basename "$lib" .so)
  [ "$ROUNDS" -gt 1 ] && name=${name}_r$round
  if [ "$lib" = default ]; then unset OMG_LIB; else export OMG_LIB=$lib; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/ab/$name" -o run --output-format csv \
     -- python3 "$R/tools/sweep_bench.py" $REPS 512 $OP) > "$R/gpurun_out/ab_$name.log" 2>&1 || exit $?
done
done
