#!/bin/bash
# lexicographic GS: the register ring on smaller 16^3 levels (OMG_GS_RING_MIN)
# A/B, the GS coarse-tail phases, the sweep's PMC; the loopback overlap trace
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
R=$PWD
mkdir -p $O
for round in 1 2; do
  for m in 2048 512 64; do
    OMG_GS_RING_MIN=$m timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C2-gs perf-gs > $O/s10_ring${m}_$round.txt 2>&1 || exit 1
  done
done
OMG_TAIL_TIMING=1 timeout -k 10 120 python -u tools/configs_bench.py --no-cpu --only C2-gs C1 > $O/s10_tail_phases_gs.txt 2>&1 || exit 1
bash tools/r04_loop_trace.sh gpurun_out/r04/s10_loop_trace || exit 1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex "gs_lex_reg|phys_gc" \
     -d $R/$O/s10_pmc_gs/p$i -o pmc --output-format csv -- python3 $R/tools/configs_bench.py --no-cpu --only perf-gs) \
     > $O/s10_pmc_gs_p$i.log 2>&1 || exit 1
done
python3 tools/pmc_occupancy.py $O/s10_pmc_gs > $O/s10_pmc_gs.txt || exit 1
