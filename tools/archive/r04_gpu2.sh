#!/bin/bash
# round 4: GS ghost-set tests + the touched kernels' parity, then A/B against the round-3 build
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_fortran_dropin.py tests/test_gpu_multirank.py -k "_rb or refinement_bnd" > $O/s2_rb.log 2>&1 || { tail -30 $O/s2_rb.log; exit 1; }
tail -1 $O/s2_rb.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_smoothers.py \
  tests/test_gpu_parity.py tests/test_gpu_multirank.py -k "not c3_512" > $O/s2_tests.log 2>&1 || { tail -30 $O/s2_tests.log; exit 1; }
tail -1 $O/s2_tests.log
bash tools/r04_ab.sh s2 "C4 C2-gs perf-gs C3 C2" octree-mg_amd/_variants/libomg_r03.so
R=$PWD
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$O/lat -o run --output-format csv -- $R/tools/lat_probe) > $O/lat.log 2>&1 || exit 1
python3 tools/trace_by_grid.py $(find $O/lat -name "*kernel_trace.csv" | head -1) > $O/lat_by_grid.txt
