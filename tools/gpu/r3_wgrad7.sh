# round 3: depthwise weight gradient at W = 7 with the row window requested at once -- encoder
# train / depthwise suites, then C5 same-box A/B (IMGCAP_DW_WGRAD_W7=0: the sliding-window kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/wgrad7
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_encoder_train_gpu.py tests/test_dwconv_cp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2; do
  for v in 1 0; do
    IMGCAP_DW_WGRAD_W7=$v timeout -k 10 300 python bench.py --config C5 --no-roofline --no-cpu-baseline > $O/C5_${v}_$i.log 2>&1 || { tail -20 $O/C5_${v}_$i.log; exit 1; }
    echo "C5 w7=$v $i: $(tail -1 $O/C5_${v}_$i.log | cut -c1-110)"
  done
done
