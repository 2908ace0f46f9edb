# round 5 step 23: smoke, then the bench line (N=1 default run)
O=gpurun_out/r05/s23
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['value'], json.dumps(d['roofline']))
print('c4', d['c4_refined']['ms_per_step'], 'gs', d['gs_lex']['ms_per_step'])"
