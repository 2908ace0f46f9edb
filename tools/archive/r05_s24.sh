# round 5 step 24: HBM counters of the 512^3 lexicographic GS sweep
# (k_gs_lex_reg with the 16-B pair pushes), one counter group per pass
O=gpurun_out/r05/s24
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "gs_lex" -d $GRAFT_REPO_ROOT/$O/p$i -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/sweep_bench.py 5 512 smooth_gs) > $O/p$i.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, collections, glob
per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/r05/s24/p*/pmc_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]; wg = int(r["Grid_Size"]) // int(r["Workgroup_Size"])
        per[(k, wg)][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open("gpurun_out/r05/s24/pmc_gs.txt", "w") as o:
    for key, cs in sorted(per.items()):
        a = {c: sum(v) / len(v) for c, v in cs.items()}
        line = f"{key[0]} workgroups={key[1]} n={max(len(v) for v in cs.values())} " + " ".join(f"{c}={x:.1f}" for c, x in a.items())
        if "FETCH_SIZE" in a and "WRITE_SIZE" in a:
            line += f"  raw GB: read {a['FETCH_SIZE']*1024/1e9:.3f} write {a['WRITE_SIZE']*1024/1e9:.3f} total {(a['FETCH_SIZE']+a['WRITE_SIZE'])*1024/1e9:.3f}"
        o.write(line + "\n"); print(line)
PY
