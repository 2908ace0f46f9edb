#!/bin/bash
# two loopback ranks in one process (bench.py's weak set-up, 256^3 per rank)
# under --kernel-trace --memory-copy-trace: does the halo exchange (the
# comm stream's copies and unpacks) overlap the interior substeps?
#   tools/r04_loop_trace.sh <outdir>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=$PWD/${1:-gpurun_out/r04/loop_trace}
mkdir -p "$OUT"
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/t" -o lt \
   --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/loopback_bench.py" 2 256 5) > "$OUT/run.log" 2>&1 || exit $?
python3 tools/overlap_summary.py "$OUT/t" > "$OUT/overlap.txt" || exit $?
exit 0
