# Kernel-trace statistics of `bench.py --config <cfg>` under several library builds (rocprofv3 each).
# usage: bash tools/prof_cfg.sh <tag> <cfg> [libs...]
TAG=$1; CFG=$2; shift 2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for lib in ${*:-libfervit.so libfervit_base.so}; do
  d=gpurun_out/${TAG}_prof_${CFG}_${lib%.so}
  FERVIT_LIB=$GRAFT_REPO_ROOT/fer-vit_amd/fervit/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $d -o run -- python3 bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $d.log 2>&1 \
    || { tail -5 $d.log; exit 1; }
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  echo "== $lib"
  python3 tools/prof_csv_summary.py "$f" 27 14 | head -16
done
