# A/B two builds of libfervit on ONE box (box-to-box clock variance is ~10%).
# usage: bash tools/ab.sh <tag> <script.py under tools/> [libA] [libB]
set -o pipefail
TAG=$1; S=$2; A=${3:-fer-vit_amd/fervit/libfervit_base.so}; B=${4:-fer-vit_amd/fervit/libfervit.so}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do
  for L in $A $B; do
    echo "== $L (round $r)"
    (cd tools && FERVIT_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 150 python -u $S 2>&1 | grep -v amdgpu.ids) || exit 1
  done
done | tee gpurun_out/ab_$TAG.txt
