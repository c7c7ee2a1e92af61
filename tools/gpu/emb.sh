set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "embedding" tests/test_train_step_gpu.py tests/test_checkpoint_gpu.py > gpurun_out/emb.log 2>&1; rc=$?
tail -3 gpurun_out/emb.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python - <<'PY'
import torch, time
from imagecaptioningconvnext_amd import kernels as K
from imagecaptioningconvnext_amd.roofline import time_launch
for n, V in ((1632, 9490), (3328, 9490)):
    ids = torch.randint(0, V, (n,), device="cuda")
    d = torch.randn(n, 512, device="cuda").bfloat16()
    t = torch.zeros(V, 512, device="cuda")
    print(n, "embedding_bwd us", round(time_launch(lambda: K.embedding_bwd(ids, d, t)) * 1e6, 2))
PY
