# GEMM config parity tests + tile-config sweep on the ViT-B shapes. usage: bash tools/gpu_gemm.sh <tag> "<cfgs>" [pytest -k]
set -o pipefail
TAG=${1:-g}; CFGS=${2:-"8 10"}; K=${3:-tile_config}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "$K" > gpurun_out/gemm_t_$TAG.txt 2>&1 || { tail -30 gpurun_out/gemm_t_$TAG.txt; exit 1; }
tail -1 gpurun_out/gemm_t_$TAG.txt
bash tools/cfg_sweep.sh $TAG "$CFGS"
