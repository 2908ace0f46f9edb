#!/bin/bash
# C4 diagnostics: kernel trace by grid, coarse-tail phase times (C4, C3, C1),
# and the tail's HBM<->LDS rounds A/B (libomg_io24: all loads in one round)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r03
mkdir -p $O
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/diag_trace_C4 -o run --output-format csv \
   -- python3 $R/tools/configs_bench.py --no-cpu --only C4) > $O/diag_trace_C4.log 2>&1 || { echo "trace rc=$?"; tail -20 $O/diag_trace_C4.log; exit 1; }
f=$(find $O/diag_trace_C4 -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_by_grid.py $f > $O/diag_trace_C4_by_grid.txt
head -45 $O/diag_trace_C4_by_grid.txt
cd $R
bash tools/r03_tailtime.sh "C4 C3 C1" diag_tail || exit 1
bash tools/r03_abn.sh "c1_ or c4 or per or ref or u32 or helm32" "C4 C3 C1" diag_ab OMG_LIB=octree-mg_amd/_variants/libomg_io24.so OMG_LIB=octree-mg_amd/_variants/libomg_head.so || exit 1
