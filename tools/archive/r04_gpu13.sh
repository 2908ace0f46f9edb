#!/bin/bash
# the whole GPU suite, then A/B of the rhs chain, the fused fill + coarse rhs
# and the stored rb coarse parts, then the bench line
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/s14_pytest_gpu.log 2>&1 || { tail -30 $O/s14_pytest_gpu.log; exit 1; }
tail -1 $O/s14_pytest_gpu.log
for round in 1 2; do
  timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C3 C4 C2 C1-gsrb C2-gs > $O/s14_A$round.txt 2>&1 || exit 1
  OMG_NO_RHS_CHAIN=1 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C3 > $O/s14_nochain$round.txt 2>&1 || exit 1
  OMG_NO_FILL_CRHS=1 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C3 C4 C2 C1-gsrb C2-gs > $O/s14_nofc$round.txt 2>&1 || exit 1
  OMG_NO_RBGV=1 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 > $O/s14_norbgv$round.txt 2>&1 || exit 1
done
timeout -k 10 400 python bench.py > $O/s14_bench.json 2> $O/s14_bench.err || exit 1
