# build + run MLP kernel variants (GPU box): bash tools/kbench/run_mlp.sh
set -e
cd $GRAFT_REPO_ROOT/tools/kbench
for v in "0:erf" "1:identity" "2:fast"; do
  id=${v%%:*}; tag=${v##*:}
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -munsafe-fp-atomics -DMLP_GELU=$id -DMLP_TAG="\"$tag\"" mlp_bench.hip -o /tmp/mlp_$tag
  timeout -k 5 60 /tmp/mlp_$tag
done
