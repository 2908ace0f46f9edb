#!/bin/bash
# round 4: the new tests first, then the whole GPU suite, then the bench
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_multirank.py tests/test_gpu_failures.py tests/test_gpu_parity.py tests/test_fortran_dropin.py \
  -k "c4_refined or c2_gs_ring or host_wait or another_rank or rolls_back or c4_ref2 or ahelm_smoother" \
  > $O/new_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
R=$PWD
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace_C4 -o run --output-format csv \
   -- python3 $R/tools/configs_bench.py --no-cpu --only C4) > $O/trace_C4.log 2>&1 || exit 1
f=$(find $O/trace_C4 -name "*kernel_trace.csv" | head -1)
python3 tools/trace_by_grid.py $f > $O/trace_C4_by_grid.txt
