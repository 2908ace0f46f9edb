#!/bin/bash
# parity subset, then configs_bench: default against several environment
# switches, interleaved, two rounds
#   tools/r03_abn.sh "<pytest -k expr>" "<configs>" tag "VAR=1" ["VAR2=1" ...]
set -o pipefail
O=gpurun_out/r03
mkdir -p $O
K="$1"; CFG="$2"; TAG="$3"; shift 3
if [ -n "$K" ]; then
  timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_failures.py tests/test_gpu_smoothers.py tests/test_fortran_dropin.py -k "$K" > $O/${TAG}_parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/${TAG}_parity.log; exit 1; }
  tail -1 $O/${TAG}_parity.log
fi
for round in 1 2; do
  timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only $CFG > $O/${TAG}_A$round.txt 2>&1 || { echo "A rc=$?"; tail $O/${TAG}_A$round.txt; exit 1; }
  echo "A$round (default)"; grep -v "^{" $O/${TAG}_A$round.txt | tail -n +2
  i=0
  for ENVB in "$@"; do
    i=$((i+1))
    env $ENVB timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only $CFG > $O/${TAG}_B${i}_$round.txt 2>&1 || { echo "B$i rc=$?"; tail $O/${TAG}_B${i}_$round.txt; exit 1; }
    echo "B$i $round ($ENVB)"; grep -v "^{" $O/${TAG}_B${i}_$round.txt | tail -n +2
  done
done
