# Round-end style GPU check: gpu tests, smoke, bench (with CPU baseline), rocprofv3 kernel stats.
# usage (from this container): gpurun --timeout 1100 -- 'bash tools/gpu_check.sh <tag> [steps]'
set -o pipefail
TAG=${1:-run}
STEPS=${2:-20}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/tests_$TAG.txt 2>&1 || { tail -30 gpurun_out/tests_$TAG.txt; exit 1; }
tail -2 gpurun_out/tests_$TAG.txt
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 \
  || { tail -20 gpurun_out/smoke_$TAG.txt; exit 1; }
tail -3 gpurun_out/smoke_$TAG.txt
timeout -k 10 300 python -u bench.py --steps $STEPS --warmup 5 > gpurun_out/bench_$TAG.txt 2>&1 \
  || { tail -20 gpurun_out/bench_$TAG.txt; exit 1; }
tail -1 gpurun_out/bench_$TAG.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic > gpurun_out/prof_$TAG.log 2>&1 \
  || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
tail -1 gpurun_out/prof_$TAG.log
f=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
python tools/prof_csv_summary.py "$f" 15 30 > gpurun_out/prof_${TAG}_summary.txt && cat gpurun_out/prof_${TAG}_summary.txt
