# round 3: column-segment depthwise kernel for W = 56 / 28 -- depthwise / kernel / encoder suites,
# microbench vs the channel-tiled kernel, then C4 / C3 same-box A/B (IMGCAP_DW_SEG=0)
# (measured while the kernel was the default; it is opt-in now, IMGCAP_DW_SEG=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/dwseg
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dwconv_cp_gpu.py tests/test_kernels_gpu.py tests/test_encoder_gpu.py tests/test_encoder_train_gpu.py tests/test_mx_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 120 python tools/dw_wide_bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
cat $O/bench.log
for i in 1 2; do
  for cfg in C4 C3; do
    for sg in 1 0; do
      IMGCAP_DW_SEG=$sg timeout -k 10 300 python bench.py --config $cfg --no-roofline --no-cpu-baseline > $O/${cfg}_${sg}_$i.log 2>&1 || { tail -20 $O/${cfg}_${sg}_$i.log; exit 1; }
      echo "$cfg seg=$sg $i: $(tail -1 $O/${cfg}_${sg}_$i.log | cut -c1-110)"
    done
  done
done
