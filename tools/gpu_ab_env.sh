# GPU tests, then the ViT-B bench with an env switch off/on (interleaved twice).
# usage: bash tools/gpu_ab_env.sh <tag> <VAR> [steps] [pytest -k]
set -o pipefail
TAG=$1; VAR=$2; STEPS=${3:-30}; K=${4:-}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  "${KA[@]}" > gpurun_out/abt_$TAG.txt 2>&1 || { tail -30 gpurun_out/abt_$TAG.txt; exit 1; }
tail -1 gpurun_out/abt_$TAG.txt
for r in 1 2; do for v in 0 1; do
  env $VAR=$v timeout -k 10 200 python -u bench.py --steps $STEPS --warmup 5 --no-cpu-baseline --no-traffic \
    > gpurun_out/ab_${TAG}_${v}_$r.txt 2>&1 || { tail -20 gpurun_out/ab_${TAG}_${v}_$r.txt; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['step_ms_p10'], d['step_ms_p90'])" gpurun_out/ab_${TAG}_${v}_$r.txt "$VAR=$v"
done; done
