#!/bin/bash
# coarse-tail phase times (OMG_TAIL_TIMING=1: wall clock of thread 0 per phase)
# for the given configs; the last lines per config
set -o pipefail
O=gpurun_out/r03
mkdir -p $O
TAG="${2:-tail}"
for cfg in $1; do
  OMG_TAIL_TIMING=1 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only $cfg > $O/${TAG}_$cfg.txt 2> $O/${TAG}_$cfg.err || { echo "rc=$? $cfg"; tail $O/${TAG}_$cfg.err; exit 1; }
  echo "== $cfg"; grep "tail us" $O/${TAG}_$cfg.err | tail -4
done
