#!/bin/bash
# final bench line + rocprof summary + C4 trace on the last tree
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
R=$PWD
mkdir -p $O
timeout -k 10 400 python bench.py > $O/s25_bench.json 2> $O/s25_bench.err || exit 1
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/s25_prof -o run --output-format csv \
   -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline) > $O/s25_prof.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/s25_trace_C4 -o run --output-format csv \
   -- python3 $R/tools/configs_bench.py --no-cpu --only C4) > $O/s25_trace_C4.log 2>&1 || exit 1
f=$(find $O/s25_trace_C4 -name "*kernel_trace.csv" | head -1)
python3 tools/trace_by_grid.py $f > $O/s25_trace_C4_by_grid.txt || exit 1
python3 tools/cycle_seq.py $f 90 > $O/s25_trace_C4_cycle.txt || exit 1
