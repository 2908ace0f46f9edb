#!/bin/bash
# C4 (one-level-refined tree) under PMC: waves, busy and wave cycles per
# kernel and level (grid size), HBM bytes; one counter group per run.
#   tools/r04_c4_pmc.sh <outdir>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=$PWD/${1:-gpurun_out/r04/pmc_c4}
mkdir -p "$OUT"
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc $grp -d "$OUT/p$i" -o pmc --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/tools/configs_bench.py" --no-cpu --only C4) > "$OUT/p$i.log" 2>&1 || exit $?
done
python3 tools/pmc_occupancy.py "$OUT" > "$OUT/summary.txt" || exit $?
exit 0
