# Quick GPU iteration: kernel parity tests + GEMM microbench.  usage: bash tools/gpu_quick.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-q}; K=${2:-}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/qt_$TAG.txt 2>&1 || { tail -30 gpurun_out/qt_$TAG.txt; exit 1; }
tail -1 gpurun_out/qt_$TAG.txt
cd tools && timeout -k 10 150 python -u gemm_bench.py 2>&1 | grep -v amdgpu.ids | tee ../gpurun_out/gb_$TAG.txt
