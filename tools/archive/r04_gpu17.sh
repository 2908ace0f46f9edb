#!/bin/bash
# end-of-round state: the whole GPU suite, the bench line and its rocprof
# summary, the C4 trace and PMC occupancy, C4 / C2-gs tail phases
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
R=$PWD
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/s21_pytest_gpu.log 2>&1 || { tail -30 $O/s21_pytest_gpu.log; exit 1; }
tail -1 $O/s21_pytest_gpu.log
timeout -k 10 400 python bench.py > $O/s21_bench.json 2> $O/s21_bench.err || exit 1
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/s21_prof -o run --output-format csv \
   -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline) > $O/s21_prof.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/s21_trace_C4 -o run --output-format csv \
   -- python3 $R/tools/configs_bench.py --no-cpu --only C4) > $O/s21_trace_C4.log 2>&1 || exit 1
f=$(find $O/s21_trace_C4 -name "*kernel_trace.csv" | head -1)
python3 tools/trace_by_grid.py $f > $O/s21_trace_C4_by_grid.txt || exit 1
python3 tools/cycle_seq.py $f 90 > $O/s21_trace_C4_cycle.txt || exit 1
bash tools/r04_c4_pmc.sh gpurun_out/r04/s21_pmc_c4 || exit 1
OMG_TAIL_TIMING=1 timeout -k 10 120 python -u tools/configs_bench.py --no-cpu --only C4 C2-gs > $O/s21_tail_phases.txt 2>&1 || exit 1
