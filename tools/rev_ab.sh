#!/bin/bash
# A/B of the alternating pass direction (LevelView::rev): bench.py and every
# config with OMG_NO_REV=1 (all passes forwards) against the default, twice
# each, interleaved; then the GPU tests on the default build.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/rev_ab
mkdir -p $O
for i in 1 2; do
  OMG_NO_REV=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/fwd_$i.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/rev_$i.log 2>&1 || exit 1
done
OMG_NO_REV=1 timeout -k 10 300 python tools/configs_bench.py --no-cpu > $O/configs_fwd.log 2>&1 || exit 1
timeout -k 10 300 python tools/configs_bench.py --no-cpu > $O/configs_rev.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo rc=$? >> $O/pytest_gpu.log
