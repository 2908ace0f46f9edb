#!/bin/bash
# FETCH_SIZE / WRITE_SIZE against known bytes (tools/fetch_probe.hip), one
# counter per rocprofv3 pass -> gpurun_out/r06/fetch_calib/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r06/fetch_calib; mkdir -p $O
for k in rd8 rd16 wr8 wr8nt cp8; do
  timeout -k 10 60 ./tools/fetch_probe $k 5 > $O/$k.time 2>&1 || exit 1
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 60 rocprofv3 --pmc $c -d $O/${k}_$c -o pmc --output-format csv -- $R/tools/fetch_probe $k 3) \
      > $O/${k}_$c.log 2>&1 || exit 1
  done
done
exit 0
