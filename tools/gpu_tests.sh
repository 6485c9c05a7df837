# GPU tests: the named files first (-k expression optional), then the whole -m gpu suite.
# usage: bash tools/gpu_tests.sh <tag> "<test files>" [k-expr]
set -o pipefail
TAG=${1:-t}; FILES=${2:-tests}; K=${3:-}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest $FILES -m gpu -v -p no:cacheprovider --timeout 150 --timeout-method thread \
  ${K:+-k "$K"} > gpurun_out/tests_$TAG.txt 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/tests_$TAG.txt | tail -40
exit $rc
