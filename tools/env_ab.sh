# bench.py --config <cfg> with an environment switch off / on, interleaved (same box)
# usage: bash tools/env_ab.sh <tag> <cfg> <VAR>
TAG=$1; CFG=$2; VAR=$3
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2 3; do for v in 0 1; do
  env $VAR=$v timeout -k 10 300 python -u bench.py --config $CFG --steps 100 --warmup 10 --no-cpu-baseline --no-traffic \
    > gpurun_out/${TAG}_${v}_$rep.json 2> gpurun_out/${TAG}.err || { tail -5 gpurun_out/${TAG}.err; exit 1; }
  echo "[$VAR=$v] $CFG $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'])" gpurun_out/${TAG}_${v}_$rep.json)" | tee -a gpurun_out/${TAG}_env_ab.txt
done; done
