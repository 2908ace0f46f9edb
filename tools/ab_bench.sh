#!/bin/bash
# Interleaved A/B of bench.py's C3 cycle (no extras, no parity, no profile
# pass) for the default library, every octree-mg_amd/_variants/libomg_*.so and
# every environment setting in $AB_ENVS (space-separated VAR=value, e.g.
# "OMG_NO_BLOCK4P=1"), then one rocprofv3 kernel trace of each:
#   [AB_ENVS=...] tools/ab_bench.sh <tag> [rounds]
# -> gpurun_out/r06/<tag>_ab/<config>_<round>.json, <config>_trace/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$PWD; O=gpurun_out/r06/${1:-ab}_ab; mkdir -p $O
CONFIGS="default $(ls $R/octree-mg_amd/_variants/libomg_*.so 2>/dev/null) ${AB_ENVS:-}"
setup() {   # -> $name; exports OMG_LIB / the env setting of config $1
  unset OMG_LIB
  for e in ${AB_ENVS:-}; do unset "${e%%=*}"; done
  case $1 in
    default) name=default ;;
    *.so) name=$(basename "$1" .so); export OMG_LIB=$1 ;;
    *=*) name=env_${1%%=*}; export "$1" ;;
  esac
}
for round in $(seq 1 "${2:-3}"); do
  for cfg in $CONFIGS; do
    setup $cfg
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra --no-parity \
      --no-profile-pass > $O/${name}_$round.json 2> $O/${name}_$round.err || exit 1
    echo "$name $round $(python3 -c "import json,sys; print(json.load(open('$O/${name}_$round.json'))['ms_per_step'])")"
  done
done
for cfg in $CONFIGS; do
  setup $cfg
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/$O/${name}_trace" -o run --output-format csv \
     -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-extra --no-parity --no-profile-pass) \
     > $O/${name}_trace.log 2>&1 || exit 1
done
exit 0
