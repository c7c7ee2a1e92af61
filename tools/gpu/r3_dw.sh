# round 3: depthwise kernel variants -- parity (tile counts, fp32 staging), microbench, C3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3dw
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_encoder_train_gpu.py -k "dwconv" > $O/t.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t.log | head -20; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for v in "1 0" "1 1" "2 1"; do
  set -- $v
  IMGCAP_DW_NTL=$1 IMGCAP_DW_F32L=$2 timeout -k 10 120 python -u tools/microbench.py dw > $O/mb_$1_$2.log 2>&1 || { tail -20 $O/mb_$1_$2.log; exit 1; }
  echo "== NTL=$1 F32L=$2"; grep dwconv7 $O/mb_$1_$2.log
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_train_step_gpu.py tests/test_lstm_gpu.py > $O/t3.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t3.log | head -20; tail -30 $O/t3.log; exit 1; }
tail -1 $O/t3.log
for a in "--lengths coco" "--lengths coco --no-len-buckets" "--lengths full"; do
  timeout -k 10 300 python -u bench.py --config C2 --steps 100 --no-cpu-baseline --no-roofline $a > $O/c2b.log 2>&1 || { tail -30 $O/c2b.log; exit 1; }
  echo "C2 $a: $(tail -1 $O/c2b.log | cut -c1-100)"
done
