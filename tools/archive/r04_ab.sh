#!/bin/bash
# configs_bench: this tree's libomg.so (A) against another build (B, OMG_LIB),
# interleaved, two rounds:  tools/r04_ab.sh tag "<configs>" <lib.so>
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
TAG="$1"; CFG="$2"; LIBB="$3"
for round in 1 2; do
  timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only $CFG > $O/${TAG}_A$round.txt 2>&1 || { echo "A rc=$?"; tail $O/${TAG}_A$round.txt; exit 1; }
  echo "A$round"; grep -v "^{" $O/${TAG}_A$round.txt | tail -n +2
  OMG_LIB=$LIBB timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only $CFG > $O/${TAG}_B$round.txt 2>&1 || { echo "B rc=$?"; tail $O/${TAG}_B$round.txt; exit 1; }
  echo "B$round ($LIBB)"; grep -v "^{" $O/${TAG}_B$round.txt | tail -n +2
done
