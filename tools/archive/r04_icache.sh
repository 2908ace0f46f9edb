#!/bin/bash
# instruction-cache counters per kernel on C4 (one pass, two SQ counters)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r04/s24_icache
mkdir -p "$OUT"
(cd /tmp && timeout -k 10 -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d "$OUT" -o pmc --output-format csv -- \
   python3 "$GRAFT_REPO_ROOT/tools/configs_bench.py" --no-cpu --only C4) > "$OUT/run.log" 2>&1
rc=$?
tail -5 "$OUT/run.log"
exit $rc
