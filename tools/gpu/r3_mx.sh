# round 3: MX GEMM tile choice (128 tile by default, 256 opt-in) -- MX suite, then C5 same-box
# A/B (IMGCAP_MX_TILE=256: the 256 tile everywhere)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/mx3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mx_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for t in "" 256 ""; do
  IMGCAP_MX_TILE=$t timeout -k 10 300 python bench.py --config C5 --no-roofline --no-cpu-baseline > $O/C5_t$t.log 2>&1 || { tail -20 $O/C5_t$t.log; exit 1; }
  echo "C5 tile=${t:-auto}: $(tail -1 $O/C5_t$t.log | cut -c1-110)"
done
