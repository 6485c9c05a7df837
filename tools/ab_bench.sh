# A/B the full training step of two libfervit builds on ONE box.
# usage: bash tools/ab_bench.sh <tag> [libA] [libB] [extra bench args]
set -o pipefail
TAG=$1; A=${2:-fer-vit_amd/fervit/libfervit_base.so}; B=${3:-fer-vit_amd/fervit/libfervit.so}; shift 3; X="$@"
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do
  for L in $A $B; do
    echo "== $L (round $r)"
    FERVIT_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic $X 2>&1 \
      | grep -v amdgpu.ids | python -c "import sys,json; [print(l.strip()[:120]) if not l.startswith('{') else print('ms/step', json.loads(l)['ms_per_step'], 'fc1', json.loads(l)['roofline']['mean_launch_ms']) for l in sys.stdin]" || exit 1
  done
done | tee gpurun_out/abb_$TAG.txt
