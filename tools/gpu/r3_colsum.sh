# round 3: batched column sums with 128 row lanes per block -- kernel tests, timing, C3 / C2 benches
# against build/libimgcap_old.so (the same tree with 32 row lanes, built locally) on the same box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/colsum
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "colsum" -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 120 python tools/colsum_bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
cat $O/bench.log
IMGCAP_LIB=$PWD/build/libimgcap_old.so timeout -k 10 120 python tools/colsum_bench.py > $O/bench_old.log 2>&1 || { tail -20 $O/bench_old.log; exit 1; }
echo "previous kernel (32 row lanes):"; cat $O/bench_old.log
for i in 1 2; do
  for cfg in C3 C2; do
    for lib in new old; do
      if [ $lib = old ]; then L=$PWD/build/libimgcap_old.so; else L=""; fi
      IMGCAP_LIB=$L timeout -k 10 300 python bench.py --config $cfg --no-roofline --no-cpu-baseline > $O/${cfg}_${lib}_$i.log 2>&1 || { tail -20 $O/${cfg}_${lib}_$i.log; exit 1; }
      echo "$cfg $lib $i: $(tail -1 $O/${cfg}_${lib}_$i.log | cut -c1-110)"
    done
  done
done
