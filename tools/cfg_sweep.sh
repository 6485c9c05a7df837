# GEMM tile-config sweep on the ViT-B shapes (one box): bash tools/cfg_sweep.sh <tag> "<cfgs>"
set -o pipefail
TAG=$1; CFGS=${2:-"8 9 2 3 6 7"}
cd "$GRAFT_REPO_ROOT/tools" && mkdir -p ../gpurun_out
for c in $CFGS; do FERVIT_GEMM_CFG=$c timeout -k 10 150 python -u gemm_bench.py 2>&1 | grep -v amdgpu.ids || exit 1; done | tee ../gpurun_out/sweep_$TAG.txt
