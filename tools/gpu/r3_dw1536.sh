# round 3: channel-pair depthwise without LN past C = 1024 (Large stage 4, fine-tuned at C5) --
# depthwise / encoder-train suites, then C5 same-box A/B against build/libimgcap_old.so (built locally)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/dw1536
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_dwconv_cp_gpu.py tests/test_encoder_train_gpu.py tests/test_encoder_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2; do
  for lib in new old; do
    if [ $lib = old ]; then L=$PWD/build/libimgcap_old.so; else L=""; fi
    IMGCAP_LIB=$L timeout -k 10 300 python bench.py --config C5 --no-roofline --no-cpu-baseline > $O/C5_${lib}_$i.log 2>&1 || { tail -20 $O/C5_${lib}_$i.log; exit 1; }
    echo "C5 $lib $i: $(tail -1 $O/C5_${lib}_$i.log | cut -c1-110)"
  done
done
