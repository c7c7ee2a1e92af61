# depthwise lane-mapping A/B: parity with IMGCAP_DW_NARROW=1, microbench both ways, C2/C3 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
IMGCAP_DW_NARROW=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_encoder_gpu.py tests/test_encoder_train_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_dw.log 2>&1 || { tail -30 gpurun_out/t_dw.log; exit 1; }
tail -1 gpurun_out/t_dw.log
for n in 0 1; do
  echo "narrow=$n"
  IMGCAP_DW_NARROW=$n timeout -k 10 200 python tools/microbench.py dw 2>&1 | grep dwconv || exit 1
  for c in C2 C3; do
    IMGCAP_DW_NARROW=$n timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'][:3], d['value'], d['ms_per_step'], d['roofline']['others_us_per_step'])"
  done
done
