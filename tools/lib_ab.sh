# bench.py --config <cfg> under several libfervit builds, interleaved (same box)
# usage: bash tools/lib_ab.sh <tag> <cfg> [lib ...]   (libs under fer-vit_amd/fervit/; default: libfervit.so libfervit_prev.so)
TAG=$1; CFG=$2; shift 2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2 3; do for lib in ${*:-libfervit.so libfervit_prev.so}; do
  FERVIT_LIB=$GRAFT_REPO_ROOT/fer-vit_amd/fervit/$lib timeout -k 10 300 python -u bench.py --config $CFG --steps 100 \
    --warmup 15 --no-cpu-baseline --no-traffic > gpurun_out/${TAG}_${lib%.so}_$rep.json 2> gpurun_out/${TAG}.err \
    || { tail -5 gpurun_out/${TAG}.err; exit 1; }
  echo "[$lib] $CFG $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('step_ms_p10'), d.get('step_ms_p90'))" gpurun_out/${TAG}_${lib%.so}_$rep.json)" | tee -a gpurun_out/${TAG}_lib_ab.txt
done; done
