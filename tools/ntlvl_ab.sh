#!/bin/bash
# A/B of the smoother's cache policy on levels that nearly fit the Infinity
# Cache: OMG_GS_NT_BYTES=0 (non-temporal everywhere) against the default
# bound, interleaved twice, over the configs with 256^3 levels and C3.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/ntlvl_ab; mkdir -p $O
for i in 1 2; do
  OMG_GS_NT_BYTES=0 timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C2 C3 C4 C5-helm C5-vlpl C5-ahelm > $O/nt_$i.log 2>&1 || exit 1
  timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C2 C3 C4 C5-helm C5-vlpl C5-ahelm > $O/cached_$i.log 2>&1 || exit 1
done
