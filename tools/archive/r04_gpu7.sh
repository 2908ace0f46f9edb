#!/bin/bash
# mid kernel at its default cap (8 boxes) against none and 64; A/B against
# round 3; C4 PMC; loopback trace; level-1 y/z PMC; bench line + rocprof;
# C4 / perf-gs / C2-gs traces; C4 coarse-tail phases
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
R=$PWD
mkdir -p $O
for round in 1 2; do
  timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 C1 C1-gsrb C2 C3 > $O/s8_mid_A$round.txt 2>&1 || exit 1
  OMG_NO_MID=1 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 C1 C1-gsrb C2 C3 > $O/s8_mid_B$round.txt 2>&1 || exit 1
done
bash tools/r04_ab.sh s8 "C4 C2-gs perf-gs C3 C2 C1-gsrb" octree-mg_amd/_variants/libomg_r03.so > $O/s8_ab.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/s8_bench.json 2> $O/s8_bench.err || exit 1
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/s8_prof -o run --output-format csv \
   -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline) > $O/s8_prof.log 2>&1 || exit 1
for cfg in C4 perf-gs C2-gs; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/s8_trace_$cfg -o run --output-format csv \
     -- python3 $R/tools/configs_bench.py --no-cpu --only $cfg) > $O/s8_trace_$cfg.log 2>&1 || exit 1
  f=$(find $O/s8_trace_$cfg -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_by_grid.py $f > $O/s8_trace_${cfg}_by_grid.txt || exit 1
done
OMG_TAIL_TIMING=1 timeout -k 10 120 python -u tools/configs_bench.py --no-cpu --only C4 C1 > $O/s8_tail_phases.txt 2>&1 || exit 1
bash tools/r04_c4_pmc.sh gpurun_out/r04/s8_pmc_c4 || exit 1
bash tools/r04_loop_trace.sh gpurun_out/r04/s8_loop_trace || exit 1
bash tools/r04_pmc_yz.sh > $O/s8_pmc_yz.txt 2>&1 || exit 1
