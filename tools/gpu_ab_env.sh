# GPU tests, then the ViT-B bench under two environments A / B (interleaved twice).
# usage: bash tools/gpu_ab_env.sh <tag> "<A: VAR=val ...>" "<B: VAR=val ...>" [steps] [pytest -k | -]
# (an empty spec runs with the box's environment; "-" as pytest -k skips the tests)
set -o pipefail
TAG=$1; A=$2; B=$3; STEPS=${4:-30}; K=${5:-}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
if [ "$K" != "-" ]; then
  if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    "${KA[@]}" > gpurun_out/abt_$TAG.txt 2>&1 || { tail -30 gpurun_out/abt_$TAG.txt; exit 1; }
  tail -1 gpurun_out/abt_$TAG.txt
fi
for r in 1 2; do for v in A B; do
  if [ $v = A ]; then spec=$A; else spec=$B; fi
  env $spec timeout -k 10 200 python -u bench.py --steps $STEPS --warmup 5 --no-cpu-baseline --no-traffic \
    > gpurun_out/ab_${TAG}_${v}_$r.txt 2>&1 || { tail -20 gpurun_out/ab_${TAG}_${v}_$r.txt; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['step_ms_p10'], d['step_ms_p90'])" gpurun_out/ab_${TAG}_${v}_$r.txt "$v[$spec]"
done; done
