#!/bin/bash
# the whole GPU suite, then the bench line and its rocprof summary
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
R=$PWD
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/s9_pytest_gpu.log 2>&1 || { tail -30 $O/s9_pytest_gpu.log; exit 1; }
tail -1 $O/s9_pytest_gpu.log
timeout -k 10 400 python bench.py > $O/s9_bench.json 2> $O/s9_bench.err || exit 1
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/s9_prof -o run --output-format csv \
   -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline) > $O/s9_prof.log 2>&1 || exit 1
