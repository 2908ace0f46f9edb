#!/bin/bash
# bench line + its rocprof summary, C4 and perf-gs kernel traces, GS sweep
# PMC bytes, C4 coarse-tail phases
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
R=$PWD
mkdir -p $O
timeout -k 10 400 python bench.py > $O/s7_bench.json 2> $O/s7_bench.err || exit 1
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/s7_prof -o run --output-format csv \
   -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline) > $O/s7_prof.log 2>&1 || exit 1
for cfg in C4 perf-gs C2-gs; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/s7_trace_$cfg -o run --output-format csv \
     -- python3 $R/tools/configs_bench.py --no-cpu --only $cfg) > $O/s7_trace_$cfg.log 2>&1 || exit 1
  f=$(find $O/s7_trace_$cfg -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_by_grid.py $f > $O/s7_trace_${cfg}_by_grid.txt || exit 1
done
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex "gs_lex_reg|phys_gc|fill_tile" \
     -d $R/$O/s7_pmc_gs/p$i -o pmc --output-format csv -- python3 $R/tools/configs_bench.py --no-cpu --only perf-gs) \
     > $O/s7_pmc_gs_p$i.log 2>&1 || exit 1
done
python3 tools/pmc_occupancy.py $O/s7_pmc_gs > $O/s7_pmc_gs.txt || exit 1
OMG_TAIL_TIMING=1 timeout -k 10 120 python -u tools/configs_bench.py --no-cpu --only C4 C1 > $O/s7_tail_phases.txt 2>&1 || exit 1
