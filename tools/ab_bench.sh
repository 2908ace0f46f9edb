#!/bin/bash
# Interleaved A/B of bench.py's C3 cycle (no extras, no parity, no profile
# pass) for the default library and every octree-mg_amd/_variants/libomg_*.so,
# then one rocprofv3 kernel trace of each:
#   tools/ab_bench.sh <tag> [rounds] [extra env for all, e.g. OMG_NO_DEEP=1]
# -> gpurun_out/r06/<tag>_ab/<lib>_<round>.json, <lib>_trace/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$PWD; O=gpurun_out/r06/${1:-ab}_ab; mkdir -p $O
for round in $(seq 1 "${2:-3}"); do
  for lib in default $(ls $R/octree-mg_amd/_variants/libomg_*.so 2>/dev/null); do
    name=$(basename "$lib" .so)
    if [ "$lib" = default ]; then unset OMG_LIB; else export OMG_LIB=$lib; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra --no-parity \
      --no-profile-pass > $O/${name}_$round.json 2> $O/${name}_$round.err || exit 1
    echo "$name $round $(python3 -c "import json,sys; print(json.load(open('$O/${name}_$round.json'))['ms_per_step'])")"
  done
done
for lib in default $(ls $R/octree-mg_amd/_variants/libomg_*.so 2>/dev/null); do
  name=$(basename "$lib" .so)
  if [ "$lib" = default ]; then unset OMG_LIB; else export OMG_LIB=$lib; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/$O/${name}_trace" -o run --output-format csv \
     -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-extra --no-parity --no-profile-pass) \
     > $O/${name}_trace.log 2>&1 || exit 1
done
exit 0
