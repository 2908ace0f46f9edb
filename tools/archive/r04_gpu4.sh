#!/bin/bash
# probes + c0 diagnosis, then the round-4 tests (c0 ghost-set case aside), then A/B against round 3
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 120 ./tools/xcd_probe > $O/xcd_probe.txt 2>&1; echo "xcd rc=$?" >> $O/xcd_probe.txt
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_smoothers.py \
  tests/test_gpu_parity.py tests/test_gpu_multirank.py -k "not c3_512" > $O/s4_tests.log 2>&1 || { tail -30 $O/s4_tests.log; exit 1; }
tail -1 $O/s4_tests.log
bash tools/r04_ab.sh s4 "C4 C2-gs perf-gs C3 C2" octree-mg_amd/_variants/libomg_r03.so
bash tools/r04_pmc_yz.sh > gpurun_out/r04/pmc_yz.txt 2>&1 || exit 1
for round in 1 2; do
  timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 C1 C1-gsrb C2 C3 > gpurun_out/r04/s4_mid_A$round.txt 2>&1 || exit 1
  OMG_NO_MID=1 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 C1 C1-gsrb C2 C3 > gpurun_out/r04/s4_mid_B$round.txt 2>&1 || exit 1
  OMG_NO_FUSE_DOWN_BC=1 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 C2 > gpurun_out/r04/s4_bc_B$round.txt 2>&1 || exit 1
done
