# round 3: wide fused CNBlock MLP -- parity tests, then timing vs the LN + two-GEMM path
# (full kernel; IMGCAP_WIDE_DBG=1 DMA only, =2 compute only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/wide
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mlp_wide_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for m in ${WIDE_MODES:-0}; do
  IMGCAP_WIDE_DBG=$m timeout -k 10 200 python -u tools/mlp_wide_bench.py --rounds 3 > $O/dbg$m.log 2>&1 || { tail -20 $O/dbg$m.log; exit 1; }
  echo "== dbg $m"; grep -v amdgpu.ids $O/dbg$m.log | cut -c1-200
done
