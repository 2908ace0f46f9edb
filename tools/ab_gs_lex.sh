#!/bin/bash
# Lexicographic GS at 512^3 (tools/sweep_bench.py smooth_gs): the one-wave
# kernel (default), the 4-wave workgroup kernel (OMG_GS_LEX_WG) and any
# timing variants in octree-mg_amd/_variants (tools/ab_variants.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$PWD
run() {
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/gs_$1" -o run --output-format csv \
     -- python3 "$R/tools/sweep_bench.py" 3 512 smooth_gs) > "$R/gpurun_out/gs_$1.log" 2>&1
}
run wave || exit $?
OMG_GS_LEX_WG=1 run wg || exit $?
for lib in $(ls $R/octree-mg_amd/_variants/libomg_*.so 2>/dev/null); do
  OMG_LIB=$lib run $(basename $lib .so) || exit $?
done
