#!/bin/bash
# PMC traffic of the fused level-1 kernels (k_smooth_resid, k_prolong_smooth)
# over 512^3 V-cycles, plus a fresh C4 kernel trace by grid
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r03
mkdir -p $O
cd $R
timeout -k 10 600 bash tools/pmc.sh "k_smooth_resid|k_prolong_smooth" vcycle 3 > $O/pmc_fused.log 2>&1 || { echo "pmc rc=$?"; tail -20 $O/pmc_fused.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc_vcycle > $O/pmc_fused.json 2>&1 || true
head -60 $O/pmc_fused.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace2_C4 -o run --output-format csv \
   -- python3 $R/tools/configs_bench.py --no-cpu --only C4) > $O/trace2_C4.log 2>&1 || { echo "trace rc=$?"; tail -20 $O/trace2_C4.log; exit 1; }
f=$(find $O/trace2_C4 -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_by_grid.py $f > $O/trace2_C4_by_grid.txt
head -30 $O/trace2_C4_by_grid.txt
