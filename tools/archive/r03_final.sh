#!/bin/bash
# End of round 3 on one GPU: smoke, the default bench line, its rocprofv3
# kernel stats, and the level-1 smoother's PMC passes (tools/pmc.sh).
# Outputs in gpurun_out/r03/final_* (copied into profiles/r03/ afterwards).
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
O=$R/gpurun_out/r03
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/final_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/final_smoke.log; exit 1; }
tail -1 $O/final_smoke.log
timeout -k 10 600 python -u bench.py > $O/final_bench.json 2> $O/final_bench.err || { echo "bench rc=$?"; tail -20 $O/final_bench.err; exit 1; }
tail -c 600 $O/final_bench.json
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/final_prof" -o run --output-format csv \
   -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-extra) > $O/final_prof.log 2>&1 || { echo "rocprof rc=$?"; tail -20 $O/final_prof.log; exit 1; }
timeout -k 10 600 bash tools/pmc.sh k_gsrb_tile smooth 5 > $O/final_pmc.log 2>&1 || { echo "pmc rc=$?"; tail -20 $O/final_pmc.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc_smooth > $O/final_pmc_smoother.json 2>&1 || true
cat $O/final_pmc_smoother.json | head -30
