#!/bin/bash
# parity subset, then configs_bench A/B: default vs an environment switch
#   tools/r03_ab.sh "<pytest -k expr>" "<configs>" "VAR=1" [tag]
set -o pipefail
O=gpurun_out/r03
mkdir -p $O
K="$1"; CFG="$2"; ENVB="$3"; TAG="${4:-ab}"
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_failures.py tests/test_fortran_dropin.py -k "$K" > $O/${TAG}_parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/${TAG}_parity.log; exit 1; }
  tail -1 $O/${TAG}_parity.log
fi
for round in 1 2; do
  timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only $CFG > $O/${TAG}_A$round.txt 2>&1 || { echo "A rc=$?"; tail $O/${TAG}_A$round.txt; exit 1; }
  env $ENVB timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only $CFG > $O/${TAG}_B$round.txt 2>&1 || { echo "B rc=$?"; tail $O/${TAG}_B$round.txt; exit 1; }
  echo "A$round (default)"; grep -v "^{" $O/${TAG}_A$round.txt | tail -n +2
  echo "B$round ($ENVB)"; grep -v "^{" $O/${TAG}_B$round.txt | tail -n +2
done
