#!/bin/bash
# round-4 switches A/B with the mid kernel off (its default): the fused
# physical / refinement-boundary down-step, the GS ghost sets
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
for round in 1 2; do
  timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 C2 C5-helm C2-gs perf-gs > $O/s11_A$round.txt 2>&1 || exit 1
  OMG_NO_FUSE_DOWN_BC=1 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C4 C2 C5-helm > $O/s11_nobc$round.txt 2>&1 || exit 1
  OMG_NO_GS_DBL=1 timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C2-gs perf-gs > $O/s11_nodbl$round.txt 2>&1 || exit 1
done
# the two-context loopback trace with a hardware queue per stream (the box
# default GPU_MAX_HW_QUEUES=4 puts 7 streams on 4 in-order queues)
GPU_MAX_HW_QUEUES=8 bash tools/r04_loop_trace.sh gpurun_out/r04/s11_loop_trace_hwq8 || exit 1
python3 tools/overlap_pairs.py gpurun_out/r04/s11_loop_trace_hwq8/t > gpurun_out/r04/s11_loop_trace_hwq8/pairs.txt || exit 1
