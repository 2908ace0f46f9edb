#!/bin/bash
# round 3, first GPU pass: new failure-detection tests, the 256^3 / 512^3
# goldens (1 rank and 2/4/8-rank loopback), then the bench line.
set -o pipefail
O=gpurun_out/r03
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_failures.py > $O/g1_failures.log 2>&1 || { echo "failures tests rc=$?"; tail -30 $O/g1_failures.log; exit 1; }
timeout -k 10 600 $PYT tests/test_gpu_parity.py -k "c2_256 or c5_helm256 or c3_per512" > $O/g1_parity_big.log 2>&1 || { echo "parity big rc=$?"; tail -30 $O/g1_parity_big.log; exit 1; }
timeout -k 10 900 $PYT tests/test_gpu_multirank.py -k "c3_512" > $O/g1_multirank_c3.log 2>&1 || { echo "multirank c3 rc=$?"; tail -30 $O/g1_multirank_c3.log; exit 1; }
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/g1_bench.json 2> $O/g1_bench.err || { echo "bench rc=$?"; tail -30 $O/g1_bench.err; exit 1; }
tail -c 3000 $O/g1_bench.json
