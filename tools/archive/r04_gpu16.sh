#!/bin/bash
# the tail forming its top level's fill + coarse rhs: the whole GPU suite,
# then A/B against OMG_NO_TAIL_CRHS=1, then the tail phases
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/s20_pytest_gpu.log 2>&1 || { tail -30 $O/s20_pytest_gpu.log; exit 1; }
tail -1 $O/s20_pytest_gpu.log
for round in 1 2 3; do
  timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 C1-gsrb C2 C2-gs C3 > $O/s20_A$round.txt 2>&1 || exit 1
  OMG_NO_TAIL_CRHS=1 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 C1-gsrb C2 C2-gs C3 > $O/s20_B$round.txt 2>&1 || exit 1
done
OMG_TAIL_TIMING=1 timeout -k 10 120 python -u tools/configs_bench.py --no-cpu --only C4 C2-gs > $O/s20_tail_phases.txt 2>&1 || exit 1
