# backward-recurrence K-slice sweep (IMGCAP_LSTM_XS / _YS) at the C2 shape
set -o pipefail
cd $GRAFT_REPO_ROOT
for xs in ${XS:-1 2 3 4 6}; do for ys in ${YS:-4 8 12 16}; do
  echo "xs=$xs ys=$ys $(IMGCAP_LSTM_XS=$xs IMGCAP_LSTM_YS=$ys timeout -k 10 60 python tools/microbench.py lstm 2>&1 | grep 'bwd recurrence')" || exit 1
done; done
