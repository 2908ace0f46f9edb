#!/bin/bash
# k_fill_crhs: parity (one-rank goldens, per-operation and fused tests,
# multi-rank goldens), then A/B against OMG_NO_FILL_CRHS and OMG_NO_RBGV
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_multirank.py tests/test_gpu_smoothers.py -k "not c3_512" > $O/s12_tests.log 2>&1 || { tail -30 $O/s12_tests.log; exit 1; }
tail -1 $O/s12_tests.log
for round in 1 2; do
  timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 C2 C3 C1-gsrb C2-gs > $O/s12_A$round.txt 2>&1 || exit 1
  OMG_NO_FILL_CRHS=1 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 C2 C3 C1-gsrb C2-gs > $O/s12_B$round.txt 2>&1 || exit 1
  OMG_NO_RBGV=1 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 > $O/s12_C$round.txt 2>&1 || exit 1
done
