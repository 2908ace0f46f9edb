#!/bin/bash
# Loopback multi-rank cycle times with and without the fused down substep
# (OMG_NO_FUSE_DOWN), interleaved: tools/ab_loop.sh -> gpurun_out/ab_loop.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for i in 1 2; do
  for cfg in "8 128 5" "2 256 5"; do
    OMG_NO_FUSE_DOWN=1 timeout -k 10 300 python tools/loopback_bench.py $cfg 0 | sed 's/^/off /' || exit $?
    timeout -k 10 300 python tools/loopback_bench.py $cfg 0 | sed 's/^/on  /' || exit $?
  done
done > gpurun_out/ab_loop.log 2>&1
