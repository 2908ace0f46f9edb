#!/bin/bash
# GPU tests, every config on one GPU and the coarse-tail phase times (a
# quick check after a kernel change; outputs under gpurun_out/)
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo rc=$? >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/configs_bench.py --no-cpu > gpurun_out/configs.log 2>&1 || exit 1
for c in C1-gsrb C3; do
  OMG_TAIL_TIMING=1 timeout -k 10 200 python tools/configs_bench.py --no-cpu --only $c > gpurun_out/tail_$c.log 2>&1 || exit 1
done
