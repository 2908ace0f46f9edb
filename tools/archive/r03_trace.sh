#!/bin/bash
# kernel traces of C4 and C3 (configs_bench, no CPU): per-kernel, per-grid averages
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r03
mkdir -p $O
for c in C4 C3 C2; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$c -o run --output-format csv \
     -- python3 $R/tools/configs_bench.py --no-cpu --only $c) > $O/trace_$c.log 2>&1 || { echo "trace $c rc=$?"; tail -20 $O/trace_$c.log; exit 1; }
  f=$(find $O/trace_$c -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_by_grid.py $f > $O/trace_${c}_by_grid.txt
  head -40 $O/trace_${c}_by_grid.txt
done
