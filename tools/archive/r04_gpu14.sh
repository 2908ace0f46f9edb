#!/bin/bash
# rhs chain at the use points: periodic parity, then C3 A/B
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multirank.py \
  -k "per or c3_per512 or fused_down or diff_" > $O/s15_tests.log 2>&1 || { tail -30 $O/s15_tests.log; exit 1; }
tail -1 $O/s15_tests.log
for round in 1 2 3; do
  timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C3 > $O/s15_A$round.txt 2>&1 || exit 1
  OMG_NO_RHS_CHAIN=1 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C3 > $O/s15_B$round.txt 2>&1 || exit 1
done
