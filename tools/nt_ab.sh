#!/bin/bash
# bench.py for the default library and the _variants (tools/ab_build.sh), each
# with the alternating pass direction and with OMG_NO_REV=1, interleaved over
# rounds:  tools/nt_ab.sh [rounds]  -> gpurun_out/nt_ab/<lib>_<dir>_<round>.log
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD; O=gpurun_out/nt_ab; mkdir -p $O
for round in $(seq 1 "${1:-2}"); do
  for lib in default $(ls $R/octree-mg_amd/_variants/libomg_*.so 2>/dev/null); do
    name=$(basename "$lib" .so)
    if [ "$lib" = default ]; then unset OMG_LIB; else export OMG_LIB=$lib; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/${name}_rev_$round.log 2>&1 || exit 1
    OMG_NO_REV=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/${name}_fwd_$round.log 2>&1 || exit 1
  done
done
