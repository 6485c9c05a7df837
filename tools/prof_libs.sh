# Kernel-trace statistics of one tool under several libfervit builds (one rocprofv3 run each).
# usage: bash tools/prof_libs.sh <tag> <tool.py> [lib ...]   (libs under fer-vit_amd/fervit/)
TAG=$1; TOOL=$2; shift 2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for lib in ${*:-libfervit.so libfervit_base.so}; do
  d=gpurun_out/${TAG}_prof_${lib%.so}
  (cd tools && FERVIT_LIB=$GRAFT_REPO_ROOT/fer-vit_amd/fervit/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats \
    --output-format csv -d ../$d -o run -- python3 $TOOL > ../$d.log 2>&1) || { tail -5 $d.log; exit 1; }
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  echo "== $lib"
  python3 tools/prof_csv_summary.py "$f" 1 12 | head -12
done
