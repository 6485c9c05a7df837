# bench.py --config <cfg> under two library builds, interleaved (same box): ms/step per run
# usage: bash tools/cfg_ab.sh <tag> <cfg> [libs...]
TAG=$1; CFG=$2; shift 2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do for lib in ${*:-libfervit.so libfervit_base.so}; do
  FERVIT_LIB=$GRAFT_REPO_ROOT/fer-vit_amd/fervit/$lib timeout -k 10 300 python -u bench.py --config $CFG --steps 100 --warmup 10 \
    --no-cpu-baseline --no-traffic > gpurun_out/${TAG}_${CFG}_${lib%.so}_$rep.json 2> gpurun_out/${TAG}_${CFG}.err \
    || { tail -5 gpurun_out/${TAG}_${CFG}.err; exit 1; }
  echo "[$lib] $CFG $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'])" gpurun_out/${TAG}_${CFG}_${lib%.so}_$rep.json)" | tee -a gpurun_out/${TAG}_cfg_ab.txt
done; done
