# round 5 step 17: k_gsrb3 planes in flight 3 (main) / 4 / 5 / 6 / 8 on C3,
# then HBM and L2 counters of the main build's launches (one group per pass)
O=gpurun_out/r05/s17
mkdir -p $O
V=$PWD/octree-mg_amd/_variants
for round in 1 2; do
  for v in main a4 a5 a6 a8; do
    echo "== round $round $v" >> $O/ab.txt
    case $v in
      main) timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1 ;;
      *) OMG_LIB=$V/libomg_b3_$v.so timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1 ;;
    esac
  done
done
grep -E "^==|^C3 " $O/ab.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 120 rocprofv3 --pmc $grp --kernel-include-regex "k_gsrb3|k_gsrb_tile" -d $GRAFT_REPO_ROOT/$O/p$i -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/configs_bench.py --no-cpu --only C3) > $O/p$i.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py $O > $O/pmc.json && python3 -c "
import json; d=json.load(open('$O/pmc.json'))
for k,v in d.items(): print(k, v.get('dispatches'), {c: round(x/1e6,1) for c,x in v['counters_avg'].items()})"
