# round 3: channel-pair depthwise kernel at W = 14 / 7 -- kernel + encoder suites, then C3 / C4
# benches, same-box A/B against the channel-tiled kernel (IMGCAP_DW_CP=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/dwcp
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dwconv_cp_gpu.py tests/test_kernels_gpu.py tests/test_encoder_gpu.py tests/test_encoder_train_gpu.py tests/test_mx_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for cfg in C4 C3; do
  for cp in 1 0; do
    IMGCAP_DW_CP=$cp timeout -k 10 300 python bench.py --config $cfg --no-roofline --no-cpu-baseline > $O/${cfg}_$cp.log 2>&1 || { tail -20 $O/${cfg}_$cp.log; exit 1; }
    echo "$cfg dw_cp=$cp: $(tail -1 $O/${cfg}_$cp.log | cut -c1-110)"
  done
done
