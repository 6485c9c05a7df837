# Kernel trace + two-stream timeline of short ViT-B bench runs under several libfervit builds (same box).
# usage: bash tools/prof_step_libs.sh <tag> [lib ...]   (libs under fer-vit_amd/fervit/; default: libfervit.so)
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for lib in ${*:-libfervit.so}; do
  d=gpurun_out/${TAG}_prof_${lib%.so}
  FERVIT_LIB=$GRAFT_REPO_ROOT/fer-vit_amd/fervit/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $d -o run -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-traffic \
    > $d.json 2>&1 || { tail -20 $d.json; exit 1; }
  f=$(find $d -name "*kernel_trace.csv" | head -1)
  python3 tools/timeline.py "$f" 5 5 > gpurun_out/${TAG}_timeline_${lib%.so}.txt 2>&1 || true
  echo "== $lib"; head -4 gpurun_out/${TAG}_timeline_${lib%.so}.txt
done
