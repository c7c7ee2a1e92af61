# round 3: channel-pair depthwise, rolled kernel rows / two output rows per block / channel-group
# blocks -- kernel + encoder suites, then C5 same-box A/B (IMGCAP_DW_CP_R=1: one row per block)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/dwr2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dwconv_cp_gpu.py tests/test_kernels_gpu.py tests/test_encoder_gpu.py tests/test_encoder_train_gpu.py tests/test_mx_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for r in "" 1 ""; do
  IMGCAP_DW_CP_R=$r timeout -k 10 300 python bench.py --config C5 --no-roofline --no-cpu-baseline > $O/C5_r$r.log 2>&1 || { tail -20 $O/C5_r$r.log; exit 1; }
  echo "C5 rows=${r:-auto}: $(tail -1 $O/C5_r$r.log | cut -c1-110)"
done
