# round 3: rolling depthwise kernel -- parity (every row-tile count), microbench by tile count, C3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3dw
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_encoder_train_gpu.py -k "dwconv" > $O/t.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t.log | head -20; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for n in 0 1 2 3 4; do
  IMGCAP_DW_NTL=$n timeout -k 10 120 python -u tools/microbench.py dw > $O/mb_$n.log 2>&1 || { tail -20 $O/mb_$n.log; exit 1; }
  echo "== NTL=$n"; grep dwconv7 $O/mb_$n.log
done
timeout -k 10 120 python -u tools/microbench.py dw > $O/mb_auto.log 2>&1 && { echo "== auto"; grep dwconv7 $O/mb_auto.log; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_encoder_gpu.py tests/test_encoder_train_gpu.py > $O/t2.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t2.log | head -20; tail -30 $O/t2.log; exit 1; }
tail -1 $O/t2.log
for c in C3 C2; do
timeout -k 10 300 python -u bench.py --config $c --steps 60 --no-cpu-baseline --no-roofline > $O/$c.log 2>&1 || { tail -30 $O/$c.log; exit 1; }
echo "$c: $(tail -1 $O/$c.log | cut -c1-110)"
done
