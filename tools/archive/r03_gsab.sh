#!/bin/bash
# lexicographic GS kernel decomposition at 512^3: default vs timing-only builds
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
bash $R/tools/ab_gs_lex.sh || exit $?
for d in $R/gpurun_out/gs_*; do
  [ -d $d ] || continue
  f=$(find $d -name "*kernel_trace.csv" | head -1)
  echo "== $(basename $d)"; python3 $R/tools/trace_by_grid.py $f gs_lex | head -4
done
