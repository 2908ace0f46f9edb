#!/bin/bash
# DESIGN §8.4 measured: the level-1 red-black substep at 512^3 without its
# y/z ghost pushes (yz1) and also without its y/z ghost loads (yz3) -- the
# upper bound of what reading the y/z neighbours' boundary rows instead would
# save -- against the product build: HBM bytes per launch (PMC, one counter
# group per pass), duration (kernel trace), and the C3 cycle (configs_bench).
# The variants' results are wrong by construction (timing only).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/r04/pmc_yz
mkdir -p $O
for v in base yz1 yz3; do
  if [ $v = base ]; then unset OMG_LIB; else export OMG_LIB=$R/octree-mg_amd/_variants/libomg_$v.so; fi
  for grp in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex k_gsrb_tile -d $O/${v}_$grp -o pmc \
       --output-format csv -- python3 $R/tools/sweep_bench.py 5 512 smooth) > $O/${v}_$grp.log 2>&1 || { echo "$v $grp failed"; exit 1; }
  done
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/${v}_trace -o run --output-format csv \
     -- python3 $R/tools/sweep_bench.py 20 512 smooth) > $O/${v}_trace.log 2>&1 || { echo "$v trace failed"; exit 1; }
done
unset OMG_LIB
for round in 1 2; do
  for v in base yz1 yz3; do
    if [ $v = base ]; then unset OMG_LIB; else export OMG_LIB=$R/octree-mg_amd/_variants/libomg_$v.so; fi
    timeout -k 10 300 python -u tools/configs_bench.py --no-cpu --only C3 > $O/cfg_${v}_$round.txt 2>&1 || exit 1
    echo "$v $round: $(grep -v '^{' $O/cfg_${v}_$round.txt | tail -1)"
  done
done
