# round 5 step 52: PMC of k_gsrb4 and k_gsrb3 (the bench roofline now names the
# level's longest pass), kernel trace of the bench, smoke, the bench line (the
# GPU suite ran on this library in s51: 520 passed)
O=gpurun_out/r05/s52
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 120 rocprofv3 --pmc $grp --kernel-include-regex "k_gsrb[34]" -d $GRAFT_REPO_ROOT/$O/p$i -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/configs_bench.py --no-cpu --only C3) > $O/p$i.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py $O > $O/pmc_block3.json && cp $O/pmc_block3.json profiles/r05/pmc_block3.json && echo pmc ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 1
python tools/trace_by_grid.py $O/prof/run_kernel_trace.csv > $O/by_grid.txt; head -12 $O/by_grid.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['value'], json.dumps(d['roofline']))
print(json.dumps(d['kernels_one_cycle']))
print('c4', d['c4_refined']['ms_per_step'], 'gs', d['gs_lex']['ms_per_step'])"
