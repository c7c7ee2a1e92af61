# round 3: stem with pixel groups strided over a capped grid (weights staged once per block) --
# stem / encoder suites, then C4 / C5 same-box A/B (measured neutral; the kernel change was reverted)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/stem
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -k stem tests/test_encoder_gpu.py tests/test_encoder_train_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2; do
  for cfg in C4 C5; do
    for lib in new old; do
      if [ $lib = old ]; then L=$PWD/build/libimgcap_old.so; else L=""; fi
      IMGCAP_LIB=$L timeout -k 10 300 python bench.py --config $cfg --no-roofline --no-cpu-baseline > $O/${cfg}_${lib}_$i.log 2>&1 || { tail -20 $O/${cfg}_${lib}_$i.log; exit 1; }
      echo "$cfg $lib $i: $(tail -1 $O/${cfg}_${lib}_$i.log | cut -c1-110)"
    done
  done
done
