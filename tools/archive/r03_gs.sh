#!/bin/bash
# lexicographic GS row-pipeline kernel: parity on every GS golden, then
# timing against the round-2 LDS wavefront kernel (OMG_GS_LEX=wave)
set -o pipefail
O=gpurun_out/r03
mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 600 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_gpu_multirank.py -k "gs and not gsrb" > $O/gs_parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/gs_parity.log; exit 1; }
tail -2 $O/gs_parity.log
timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C1 C2-gs perf-gs > $O/gs_rows.txt 2>&1 || { echo "bench rc=$?"; tail -20 $O/gs_rows.txt; exit 1; }
OMG_GS_LEX=wave timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C1 C2-gs perf-gs > $O/gs_wave.txt 2>&1 || { echo "bench2 rc=$?"; tail -20 $O/gs_wave.txt; exit 1; }
echo ROWS; tail -4 $O/gs_rows.txt; echo WAVE; tail -4 $O/gs_wave.txt
