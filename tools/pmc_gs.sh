#!/bin/bash
# One SQ counter pass over the lexicographic GS sweep (tools/sweep_bench.py
# smooth_gs): where the waves of k_gs_lex_wave spend their cycles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc_gs
mkdir -p "$OUT"
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
   SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex "gs_lex" \
   -d "$OUT/p1" -o pmc --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/sweep_bench.py" 2 512 smooth_gs) \
   > "$OUT/p1.log" 2>&1 || exit $?
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES \
   GRBM_GUI_ACTIVE --kernel-include-regex "gs_lex" \
   -d "$OUT/p2" -o pmc --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/sweep_bench.py" 2 512 smooth_gs) \
   > "$OUT/p2.log" 2>&1 || exit $?
