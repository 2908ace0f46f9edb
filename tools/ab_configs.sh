#!/bin/bash
# tools/configs_bench.py (GPU only) for the default library and each
# octree-mg_amd/_variants/libomg_*.so: ms per cycle of the named configs.
#   tools/ab_configs.sh C1 C1-gsrb ...  -> gpurun_out/abcfg_<name>.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
for lib in default $(ls $R/octree-mg_amd/_variants/libomg_*.so 2>/dev/null); do
  name=$(basename "$lib" .so)
  if [ "$lib" = default ]; then unset OMG_LIB; else export OMG_LIB=$lib; fi
  timeout -k 10 300 python3 "$R/tools/configs_bench.py" --no-cpu --only "$@" > "$R/gpurun_out/abcfg_$name.log" 2>&1 || exit $?
done
