# fused MLP kernel-bench variants: bash tools/gpu/mlp_v.sh "FLAGS" ...
set -o pipefail
cd $GRAFT_REPO_ROOT/tools/kbench
for f in "$@"; do
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fno-slp-vectorize -munsafe-fp-atomics $f -DMLP_TAG="\"$f\"" mlp_bench.hip -o /tmp/mlp_v 2>/dev/null || exit 1
timeout -k 5 60 /tmp/mlp_v || exit 1
done
