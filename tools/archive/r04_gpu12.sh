#!/bin/bash
# the rhs chain: parity (goldens incl. periodic multi-rank and diffusion,
# failures, drop-in), then A/B against OMG_NO_RHS_CHAIN on the periodic configs
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_multirank.py tests/test_gpu_failures.py tests/test_fortran_dropin.py > $O/s13_tests.log 2>&1 || { tail -30 $O/s13_tests.log; exit 1; }
tail -1 $O/s13_tests.log
for round in 1 2; do
  timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C3 C4 > $O/s13_A$round.txt 2>&1 || exit 1
  OMG_NO_RHS_CHAIN=1 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C3 > $O/s13_B$round.txt 2>&1 || exit 1
done
timeout -k 10 400 python bench.py > $O/s13_bench.json 2> $O/s13_bench.err || exit 1
