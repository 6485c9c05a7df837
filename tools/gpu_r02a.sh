# Round-2 check: changed GPU tests + bench (new probe phase, percentiles, PMC traffic over gemm_8ph).
set -o pipefail
TAG=${1:-r02a}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_graph.py tests/test_gpu_checkpoint.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/tests_$TAG.txt 2>&1 || { tail -40 gpurun_out/tests_$TAG.txt; exit 1; }
tail -3 gpurun_out/tests_$TAG.txt
timeout -k 10 500 python -u bench.py > gpurun_out/bench_$TAG.txt 2>&1 || { tail -20 gpurun_out/bench_$TAG.txt; exit 1; }
tail -1 gpurun_out/bench_$TAG.txt
