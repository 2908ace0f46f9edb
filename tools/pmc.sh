#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, nothing else traced) for a
# kernel regex over tools/sweep_bench.py.   tools/pmc.sh <regex> <op> [reps]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
RE=${1:-k_gsrb_tile}; OP=${2:-smooth}; REPS=${3:-5}
OUT=$PWD/gpurun_out/pmc_$OP
mkdir -p "$OUT"
timeout -k 10 300 python3 tools/sweep_bench.py 20 512 $OP > "$OUT/time.log" 2>&1 || exit $?
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$RE" -d "$OUT/p$i" -o pmc --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/sweep_bench.py" $REPS 512 $OP) > "$OUT/p$i.log" 2>&1 || exit $?
done
exit 0
