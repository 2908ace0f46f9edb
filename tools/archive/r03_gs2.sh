#!/bin/bash
# lex GS: parity of every GS golden, then 512^3 sweep timing (default vs variants)
set -o pipefail
O=gpurun_out/r03
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multirank.py -k "gs and not gsrb" > $O/gs2_parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/gs2_parity.log; exit 1; }
tail -1 $O/gs2_parity.log
bash tools/r03_gsab.sh
timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C1 C2-gs perf-gs > $O/gs2_configs.txt 2>&1 || { echo "cfg rc=$?"; tail $O/gs2_configs.txt; exit 1; }
tail -4 $O/gs2_configs.txt
