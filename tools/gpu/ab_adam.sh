# round 3: same-box A/B of the decoder's clip + Adam inside the backward (IMGCAP_INLINE_ADAM=1)
# vs after it (=0), C2 default bench, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_adam
mkdir -p $O
for r in 1 2 3; do
  for a in 1 0; do
    IMGCAP_INLINE_ADAM=$a timeout -k 10 300 python bench.py --no-roofline --no-cpu-baseline > $O/b_${a}_$r.log 2>&1 || { tail -20 $O/b_${a}_$r.log; exit 1; }
    echo "inline=$a round $r: $(tail -1 $O/b_${a}_$r.log | cut -c1-120)"
  done
done
