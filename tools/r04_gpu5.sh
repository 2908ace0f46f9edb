#!/bin/bash
# barrier probe, the round-4 GPU tests, A/B against round 3, mid / fused-bc
# A/B, then the C4 PMC passes and the two-rank loopback trace
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 120 ./tools/xcd_probe > $O/xcd_probe7.txt 2>&1; echo "xcd rc=$?" >> $O/xcd_probe7.txt
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_smoothers.py tests/test_gpu_multirank.py -k "not c3_512" > $O/s7_tests.log 2>&1 || { tail -30 $O/s7_tests.log; exit 1; }
tail -1 $O/s7_tests.log
for round in 1 2; do
  timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 C1 C1-gsrb C2 > gpurun_out/r04/s7_mid_A$round.txt 2>&1 || exit 1
  OMG_NO_MID=1 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 C1 C1-gsrb C2 > gpurun_out/r04/s7_mid_B$round.txt 2>&1 || exit 1
  OMG_MID_MAX_BOXES=64 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 C1 C1-gsrb C2 > gpurun_out/r04/s7_mid_C$round.txt 2>&1 || exit 1
  OMG_NO_FUSE_DOWN_BC=1 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 C2 > gpurun_out/r04/s7_bc_B$round.txt 2>&1 || exit 1
done
bash tools/r04_ab.sh s7 "C4 C2-gs perf-gs C3 C2" octree-mg_amd/_variants/libomg_r03.so || exit 1
bash tools/r04_c4_pmc.sh gpurun_out/r04/pmc_c4 || exit 1
bash tools/r04_loop_trace.sh gpurun_out/r04/loop_trace || exit 1
bash tools/r04_pmc_yz.sh > gpurun_out/r04/pmc_yz.txt 2>&1 || exit 1
