# round 5 step 7: bench line, then interleaved A/B of the round-4 library
# against this one on C3 / C2-gs / C4 (ms per cycle), then a kernel trace
mkdir -p gpurun_out/r05
timeout -k 10 400 python bench.py > gpurun_out/r05/s7_bench.json 2> gpurun_out/r05/s7_bench.err || exit 1
tail -c 400 gpurun_out/r05/s7_bench.json
for round in 1 2; do
  for lib in before after; do
    if [ $lib = before ]; then L=$PWD/octree-mg_amd/_variants/libomg_r05_before.so; else L=$PWD/octree-mg_amd/libomg.so; fi
    echo "== round $round lib $lib" >> gpurun_out/r05/s7_ab.txt
    OMG_LIB=$L timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 C2-gs C4 >> gpurun_out/r05/s7_ab.txt 2>&1 || exit 1
  done
done
grep -E "^==|^C3 |^C2-gs |^C4 " gpurun_out/r05/s7_ab.txt | head -40
