# round 5 step 8: rocprofv3 kernel trace + stats of the bench (C3 line,
# c4_refined, gs_lex), the C3 cycle's launch gaps, and the PMC passes of the
# level-1 red-black substep (profiles/r05/pmc_smoother.json)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05
mkdir -p $O
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/s8_prof -o s8 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline) > $O/s8_rocprof.log 2>&1 || exit 1
ST=$(find $O/s8_prof -name "*kernel_stats.csv" | head -1); KT=$(find $O/s8_prof -name "*kernel_trace.csv" | head -1)
cp "$ST" $O/s8_rocprof_kernel_stats.csv && python3 tools/trace_by_grid.py "$KT" "gsrb_tile|smooth_resid|prolong_smooth|box_sums|seq_sum|gs_lex_reg|face_gc" > $O/s8_trace_by_grid.txt
python3 tools/trace_gaps.py "$KT" k_coarse_tail 8 > $O/s8_trace_gaps.txt
head -40 $O/s8_trace_by_grid.txt
timeout -k 10 900 bash tools/pmc.sh k_gsrb_tile smooth 5 > $O/s8_pmc.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_smooth > $O/s8_pmc_smooth.json
tail -20 $O/s8_pmc_smooth.json
