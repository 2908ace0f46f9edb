#!/bin/bash
# End-of-round measurement on one GPU: bench.py (N=1, the BASELINE workload),
# its rocprofv3 kernel stats, and the smoother's PMC passes (tools/pmc.sh) —
# outputs under gpurun_out/ (copy the ones to keep into profiles/rNN/).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv \
   -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline) > gpurun_out/prof.log 2>&1 || exit 1
timeout -k 10 900 bash tools/pmc.sh k_gsrb_tile smooth 5 || exit 1
python tools/pmc_summary.py gpurun_out/pmc_smooth > gpurun_out/pmc_smoother.json 2>&1 || true
